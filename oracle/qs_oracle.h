/*
 * qs_oracle.h — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * A straight-line C restatement of spec/semantics.md (= SURVEY.md Appendix A), which restates
 * upstream kube-scheduler v1.32 plugin semantics.  The mounted reference
 * (/root/reference/README.md:1) is a one-line title with no code, tests or fixtures, so
 * PARITY IS UNPINNED by the reference: this oracle is pinned only by the hand-computed
 * known-answer tests of spec/kat.md and by cross-checks against the
 * independent pure-Python restatement in oracle/oracle.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may call this.
 * All quantities are canonical int64 (millicores, bytes, counts); float64 only where upstream
 * uses float64 (BalancedAllocation).  No device-oriented shortcuts: true int64 division,
 * true IEEE double division.
 */
#ifndef QS_ORACLE_H
#define QS_ORACLE_H
#include <stdint.h>

#define OR_MAX_EXT 2
#define OR_MAX_TERMS 4
/* scoring-resource ids of the configurable resource lists (NodeResourcesFitArgs.ScoringStrategy.
 * Resources, NodeResourcesBalancedAllocationArgs.Resources): cpu, memory, extended resource 0 / 1 */
#define OR_MAX_SCORE_RES 4
enum { OR_RES_NONE = 0, OR_RES_CPU = 1, OR_RES_MEMORY = 2, OR_RES_EXT0 = 3, OR_RES_EXT1 = 4 };

typedef struct {
    uint32_t n;
    int64_t *alloc_cpu, *alloc_mem, *alloc_ext /* [n*OR_MAX_EXT] */, *max_pods;
    int64_t *req_cpu, *req_mem, *req_ext /* [n*OR_MAX_EXT] */, *nz_cpu, *nz_mem, *pods;
    uint64_t *taint_hard, *taint_soft, *label_bits /* [n*2] */;
    int32_t *zone; /* topology zone id (< 64), batched-mode zone anti-affinity */
} or_nodes; /* mutable: or_schedule applies Reserve in place */

typedef struct {
    uint32_t p;
    int64_t *req_cpu, *req_mem, *req_ext /* [p*OR_MAX_EXT] */, *nz_cpu, *nz_mem;
    int32_t *qos, *priority;
    uint64_t *tol_hard, *tol_soft, *sel /* [p*2] */;
    int32_t *n_req_terms, *n_pref_terms;
    uint64_t *req_terms /* [p*OR_MAX_TERMS*2] */, *pref_terms /* [p*OR_MAX_TERMS*2] */;
    int32_t *pref_weight /* [p*OR_MAX_TERMS] */;
    int32_t *app, *anti_affinity; /* spec S11: group < 1024; 0 none, 1 hostname, 2 zone */
} or_pods;

typedef struct {
    int64_t wc, wm;            /* LeastAllocated resource weights (cpu, memory) */
    int32_t w_fit[3], w_bal[3]; /* per QoS class: [BestEffort, Burstable, Guaranteed] */
    int32_t w_tt, w_na;
    int32_t enable_taint, enable_affinity, balanced_skip_besteffort, qos_sort;
    /* LeastAllocated scoring resources in list order (n_fit_res = 0: [(cpu, wc), (memory, wm)]) */
    int32_t n_fit_res, fit_res[OR_MAX_SCORE_RES], fit_w[OR_MAX_SCORE_RES];
    /* BalancedAllocation resources in list order (n_bal_res = 0: [cpu, memory]) */
    int32_t n_bal_res, bal_res[OR_MAX_SCORE_RES];
} or_config;

/* Per-node plugin scores for one pod against the current node table (no state change).
 * keys[n] = packed key of spec S7 (0 = infeasible). scores (nullable) = [n][4] {LA, BA, TT, NA}
 * after normalization. */
void or_score_pod(const or_config *cfg, const or_nodes *nodes, const or_pods *pods, uint32_t j,
                  uint64_t *keys, int64_t *scores);

/* Sequential exact stream (spec S7/S8).  placement[j] indexed by arrival position j.
 * best_key (nullable) = k* per arrival position.  order_out (nullable) = processing order.
 * nthreads > 1 parallelises the node scan of each pod (upstream Parallelizer analogue). */
void or_schedule(const or_config *cfg, or_nodes *nodes, const or_pods *pods, int32_t *placement,
                 uint64_t *best_key, uint32_t *order_out, int nthreads);

/* The same exact stream with an incremental argmax (per pod type a max tree over the nodes'
 * keys; only the reserved node is re-scored per pod): identical results, for profiles without
 * TaintToleration / NodeAffinity.  Returns -1 (nothing usable) for normalizing profiles or when
 * the trees would need more than max_bytes; nodes are then partially updated: pass a copy. */
int or_schedule_incremental(const or_config *cfg, or_nodes *nodes, const or_pods *pods, int32_t *placement,
                            uint64_t *best_key, uint32_t *order_out, int nthreads, uint64_t max_bytes);

/* Batched mode (spec S11): batches of `batch` (<= 64) pods; each pod's 64 best keys against the
 * batch-start table (required anti-affinity to its app per hostname / zone included), claims in
 * batch order (best key whose node, and for zone anti-affinity whose (app, zone), no earlier pod of
 * the batch claimed), all claims applied after the batch, pods with every candidate claimed carried
 * to the front of the next batch.  placement[j] by arrival position; best_key[j] = the claimed key
 * (0 if unschedulable).  Returns the number of batches.  Profile: Fit + Balanced (+ ext). */
uint32_t or_schedule_batched(const or_config *cfg, or_nodes *nodes, const or_pods *pods,
                             uint32_t batch, int32_t *placement, uint64_t *best_key, int nthreads);

/* The same batched stream with incremental lists (per pod type and zone a max tree over the
 * nodes' keys; only the claimed nodes are re-scored per batch): identical results for Fit +
 * Balanced (+ ext) profiles.  Returns 0xFFFFFFFF (nothing usable) for normalizing profiles. */
uint32_t or_schedule_batched_incremental(const or_config *cfg, or_nodes *nodes, const or_pods *pods,
                                         uint32_t batch, int32_t *placement, uint64_t *best_key, int nthreads);

/* Reserve / Unreserve of pod j on node n (spec S7). */
void or_reserve(or_nodes *nodes, const or_pods *pods, uint32_t j, uint32_t n, int sign);

/* spec/synth.md generator, independent restatement (counter-based SplitMix64). */
void or_generate(int config, uint64_t seed, or_nodes *nodes, or_pods *pods);

/* individual scorers exposed for KAT tests */
int64_t or_least_allocated(int64_t alloc_c, int64_t reqd_c, int64_t alloc_m, int64_t reqd_m,
                           int64_t wc, int64_t wm);
int64_t or_balanced(int64_t alloc_c, int64_t req_c, int64_t alloc_m, int64_t req_m);
/* The same scorers over a resource list: (alloc[i], reqd[i]) as calculateResourceAllocatableRequest
 * returns them ((0, 0) for an extended resource the pod does not request), w[i] the weights. */
int64_t or_least_allocated_v(int cnt, const int64_t *alloc, const int64_t *reqd, const int64_t *w);
int64_t or_balanced_v(int cnt, const int64_t *alloc, const int64_t *reqd);

#endif
