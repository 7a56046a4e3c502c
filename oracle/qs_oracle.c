/*
 * qs_oracle.c — CPU ORACLE (test infrastructure; see qs_oracle.h header for the parity status:
 * PARITY UNPINNED by the reference, which has no code; pinned by spec/kat.md KATs and the
 * independent oracle/oracle.py restatement).
 *
 * Straight-line restatement of spec/semantics.md, one pod × one node at a time, int64 integer
 * arithmetic and IEEE binary64 where upstream uses float64.  Every function names the upstream
 * kube-scheduler v1.32 symbol it restates.
 *
 * Build: oracle/Makefile -> oracle/liboracle.so (gcc -O2 -fopenmp -ffp-contract=off).
 */
#include "qs_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAX_NODE_SCORE 100 /* UP framework/interface.go#MaxNodeScore */

/* UP noderesources/least_allocated.go#leastRequestedScore */
static int64_t least_requested_score(int64_t requested, int64_t capacity) {
    if (capacity == 0) return 0;
    if (requested > capacity) return 0;
    return ((capacity - requested) * MAX_NODE_SCORE) / capacity;
}

/* UP noderesources/least_allocated.go#leastResourceScorer: requested[i] / allocatable[i] as
 * resource_allocation.go#score fills them (an entry with allocatable 0 is skipped, its weight not
 * counted). */
int64_t or_least_allocated_v(int cnt, const int64_t *alloc, const int64_t *reqd, const int64_t *w) {
    int64_t node_score = 0, weight_sum = 0;
    for (int i = 0; i < cnt; i++) {
        if (alloc[i] == 0) continue;
        node_score += least_requested_score(reqd[i], alloc[i]) * w[i];
        weight_sum += w[i];
    }
    if (weight_sum == 0) return 0;
    return node_score / weight_sum;
}

/* The default resource list [cpu, memory]: requested = NonZeroRequested + pod non-zero request
 * (resource_allocation.go#score, calculateResourceAllocatableRequest with useRequested=false). */
int64_t or_least_allocated(int64_t alloc_c, int64_t reqd_c, int64_t alloc_m, int64_t reqd_m,
                           int64_t wc, int64_t wm) {
    const int64_t alloc[2] = {alloc_c, alloc_m}, reqd[2] = {reqd_c, reqd_m}, w[2] = {wc, wm};
    return or_least_allocated_v(2, alloc, reqd, w);
}

/* UP noderesources/balanced_allocation.go#balancedResourceScorer (float64 throughout; Go on amd64
 * fuses nothing, so every product and sum below is rounded on its own: -ffp-contract=off, and
 * volatile where the compiler could otherwise keep a value in extended precision). */
int64_t or_balanced_v(int cnt, const int64_t *alloc, const int64_t *reqd) {
    double fr[OR_MAX_SCORE_RES];
    double total = 0;
    int k = 0;
    for (int i = 0; i < cnt && k < OR_MAX_SCORE_RES; i++) {
        if (alloc[i] == 0) continue;
        volatile double f = (double)reqd[i] / (double)alloc[i];
        double ff = f;
        if (ff > 1) ff = 1;
        volatile double t = total + ff; /* totalFraction += fraction */
        total = t;
        fr[k++] = ff;
    }
    double std = 0.0;
    if (k == 2) {
        volatile double d = (fr[0] - fr[1]) / 2;
        std = fabs(d);
    } else if (k > 2) {
        volatile double mean = total / (double)k;
        double sum = 0;
        for (int i = 0; i < k; i++) {
            volatile double d = fr[i] - mean;
            volatile double sq = d * d;
            volatile double t = sum + sq; /* sum = sum + (fraction-mean)*(fraction-mean) */
            sum = t;
        }
        volatile double var = sum / (double)k;
        std = sqrt(var); /* Go math.Sqrt: correctly rounded (SQRTSD on amd64) */
    }
    volatile double one_minus = 1 - std;
    volatile double scaled = one_minus * (double)MAX_NODE_SCORE;
    return (int64_t)scaled;
}

/* The default resource list [cpu, memory]; requested = Requested + pod request (useRequested=true). */
int64_t or_balanced(int64_t alloc_c, int64_t req_c, int64_t alloc_m, int64_t req_m) {
    const int64_t alloc[2] = {alloc_c, alloc_m}, reqd[2] = {req_c, req_m};
    return or_balanced_v(2, alloc, reqd);
}

/* UP noderesources/resource_allocation.go#calculateResourceAllocatableRequest for node n and pod j:
 * cpu / memory from NonZeroRequested (use_requested = 0, LeastAllocated) or Requested (1,
 * BalancedAllocation) plus the pod's request of the same kind (calculatePodResourceRequest: the
 * non-zero defaults only when !useRequested); an extended (scalar) resource the pod does not
 * request is (0, 0), i.e. skipped; otherwise Allocatable.ScalarResources and
 * Requested.ScalarResources + the pod's request. */
static void alloc_request(const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j, int res,
                          int use_requested, int64_t *alloc, int64_t *reqd) {
    *alloc = 0;
    *reqd = 0;
    switch (res) {
        case OR_RES_CPU:
            *alloc = nd->alloc_cpu[n];
            *reqd = use_requested ? nd->req_cpu[n] + pd->req_cpu[j] : nd->nz_cpu[n] + pd->nz_cpu[j];
            break;
        case OR_RES_MEMORY:
            *alloc = nd->alloc_mem[n];
            *reqd = use_requested ? nd->req_mem[n] + pd->req_mem[j] : nd->nz_mem[n] + pd->nz_mem[j];
            break;
        case OR_RES_EXT0:
        case OR_RES_EXT1: {
            const int k = res - OR_RES_EXT0;
            const int64_t q = pd->req_ext[j * OR_MAX_EXT + k];
            if (q == 0) break; /* podRequest == 0 && IsScalarResourceName */
            *alloc = nd->alloc_ext[n * OR_MAX_EXT + k];
            *reqd = nd->req_ext[n * OR_MAX_EXT + k] + q;
            break;
        }
        default:
            break;
    }
}

/* NodeResourcesFit.Score, ScoringStrategy LeastAllocated, over the configured resources. */
static int64_t least_allocated_node(const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t n,
                                    uint32_t j) {
    int64_t alloc[OR_MAX_SCORE_RES], reqd[OR_MAX_SCORE_RES], w[OR_MAX_SCORE_RES];
    int cnt = 0;
    if (cfg->n_fit_res <= 0) { /* defaults: [{cpu, wc}, {memory, wm}] */
        alloc_request(nd, pd, n, j, OR_RES_CPU, 0, &alloc[0], &reqd[0]);
        alloc_request(nd, pd, n, j, OR_RES_MEMORY, 0, &alloc[1], &reqd[1]);
        w[0] = cfg->wc;
        w[1] = cfg->wm;
        cnt = 2;
    } else {
        for (; cnt < cfg->n_fit_res && cnt < OR_MAX_SCORE_RES; cnt++) {
            alloc_request(nd, pd, n, j, cfg->fit_res[cnt], 0, &alloc[cnt], &reqd[cnt]);
            w[cnt] = cfg->fit_w[cnt];
        }
    }
    return or_least_allocated_v(cnt, alloc, reqd, w);
}

/* NodeResourcesBalancedAllocation.Score over the configured resources. */
static int64_t balanced_node(const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j) {
    int64_t alloc[OR_MAX_SCORE_RES], reqd[OR_MAX_SCORE_RES];
    int cnt = 0;
    if (cfg->n_bal_res <= 0) { /* defaults: [cpu, memory] */
        alloc_request(nd, pd, n, j, OR_RES_CPU, 1, &alloc[0], &reqd[0]);
        alloc_request(nd, pd, n, j, OR_RES_MEMORY, 1, &alloc[1], &reqd[1]);
        cnt = 2;
    } else {
        for (; cnt < cfg->n_bal_res && cnt < OR_MAX_SCORE_RES; cnt++)
            alloc_request(nd, pd, n, j, cfg->bal_res[cnt], 1, &alloc[cnt], &reqd[cnt]);
    }
    return or_balanced_v(cnt, alloc, reqd);
}

/* UP noderesources/fit.go#fitsRequest (+ TooManyPods check) */
static int fits_request(const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j) {
    if (nd->pods[n] + 1 > nd->max_pods[n]) return 0;
    int any_ext = 0;
    for (int k = 0; k < OR_MAX_EXT; k++) any_ext |= pd->req_ext[j * OR_MAX_EXT + k] != 0;
    if (pd->req_cpu[j] == 0 && pd->req_mem[j] == 0 && !any_ext) return 1;
    if (pd->req_cpu[j] > 0 && pd->req_cpu[j] > nd->alloc_cpu[n] - nd->req_cpu[n]) return 0;
    if (pd->req_mem[j] > 0 && pd->req_mem[j] > nd->alloc_mem[n] - nd->req_mem[n]) return 0;
    for (int k = 0; k < OR_MAX_EXT; k++) {
        int64_t q = pd->req_ext[j * OR_MAX_EXT + k];
        if (q == 0) continue;
        if (q > nd->alloc_ext[n * OR_MAX_EXT + k] - nd->req_ext[n * OR_MAX_EXT + k]) return 0;
    }
    return 1;
}

/* UP tainttoleration/taint_toleration.go#Filter on interned bitmasks (spec S5) */
static int taint_filter(const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j) {
    return (nd->taint_hard[n] & ~pd->tol_hard[j]) == 0;
}
/* UP tainttoleration/taint_toleration.go#Score: count of intolerable PreferNoSchedule taints */
static int64_t taint_raw(const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j) {
    return (int64_t)__builtin_popcountll(nd->taint_soft[n] & ~pd->tol_soft[j]);
}
static int mask_subset(const uint64_t *m, const uint64_t *bits) {
    return (m[0] & bits[0]) == m[0] && (m[1] & bits[1]) == m[1];
}
/* UP nodeaffinity/node_affinity.go#Filter (nodeSelector + required terms, OR over terms) */
static int affinity_filter(const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j) {
    const uint64_t *lb = &nd->label_bits[n * 2];
    if (!mask_subset(&pd->sel[j * 2], lb)) return 0;
    int nt = pd->n_req_terms[j];
    if (nt == 0) return 1;
    for (int t = 0; t < nt; t++)
        if (mask_subset(&pd->req_terms[(j * OR_MAX_TERMS + t) * 2], lb)) return 1;
    return 0;
}
/* UP nodeaffinity/node_affinity.go#Score: sum of weights of matching preferred terms */
static int64_t affinity_raw(const or_nodes *nd, const or_pods *pd, uint32_t n, uint32_t j) {
    const uint64_t *lb = &nd->label_bits[n * 2];
    int64_t s = 0;
    for (int t = 0; t < pd->n_pref_terms[j]; t++)
        if (mask_subset(&pd->pref_terms[(j * OR_MAX_TERMS + t) * 2], lb))
            s += pd->pref_weight[j * OR_MAX_TERMS + t];
    return s;
}

static int feasible(const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t n,
                    uint32_t j) {
    if (!fits_request(nd, pd, n, j)) return 0;
    if (cfg->enable_taint && !taint_filter(nd, pd, n, j)) return 0;
    if (cfg->enable_affinity && !affinity_filter(nd, pd, n, j)) return 0;
    return 1;
}

/* UP helper/normalize_score.go#DefaultNormalizeScore(100, reverse, scores) for one score */
static int64_t normalize(int64_t raw, int64_t max_count, int reverse) {
    if (max_count == 0) return reverse ? MAX_NODE_SCORE : raw;
    int64_t s = MAX_NODE_SCORE * raw / max_count;
    return reverse ? MAX_NODE_SCORE - s : s;
}

/* One pod's key for node n given the per-pod normalization maxima (spec S5-S7). */
static uint64_t node_key(const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t n,
                         uint32_t j, int64_t mt, int64_t ma, int64_t *sc) {
    if (!feasible(cfg, nd, pd, n, j)) return 0;
    int q = pd->qos[j];
    int64_t la = least_allocated_node(cfg, nd, pd, n, j);
    int64_t ba = balanced_node(cfg, nd, pd, n, j);
    if (cfg->balanced_skip_besteffort && q == 0) ba = 0;
    int64_t tt = 0, na = 0;
    if (cfg->enable_taint) tt = normalize(taint_raw(nd, pd, n, j), mt, 1);
    if (cfg->enable_affinity) na = normalize(affinity_raw(nd, pd, n, j), ma, 0);
    int64_t total = cfg->w_fit[q] * la + cfg->w_bal[q] * ba + cfg->w_tt * tt * (cfg->enable_taint != 0) +
                    cfg->w_na * na * (cfg->enable_affinity != 0);
    if (sc) { sc[0] = la; sc[1] = ba; sc[2] = tt; sc[3] = na; }
    return ((uint64_t)(total + 1) << 32) | (uint64_t)(0xFFFFFFFFu - n);
}

/* NormalizeScore maxima over the nodes that passed Filter (UP framework/runtime/framework.go#
 * RunScorePlugins -> NormalizeScore runs over the feasible node list only). */
static void norm_maxima(const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t j,
                        int64_t *mt, int64_t *ma, int nthreads) {
    int64_t t = 0, a = 0;
    if (cfg->enable_taint || cfg->enable_affinity) {
        int64_t n_ = nd->n;
#pragma omp parallel for reduction(max : t, a) num_threads(nthreads) if (nthreads > 1)
        for (int64_t n = 0; n < n_; n++) {
            if (!feasible(cfg, nd, pd, (uint32_t)n, j)) continue;
            if (cfg->enable_taint) { int64_t r = taint_raw(nd, pd, (uint32_t)n, j); if (r > t) t = r; }
            if (cfg->enable_affinity) { int64_t r = affinity_raw(nd, pd, (uint32_t)n, j); if (r > a) a = r; }
        }
    }
    *mt = t;
    *ma = a;
}

void or_score_pod(const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t j,
                  uint64_t *keys, int64_t *scores) {
    int64_t mt, ma;
    norm_maxima(cfg, nd, pd, j, &mt, &ma, 1);
    for (uint32_t n = 0; n < nd->n; n++)
        keys[n] = node_key(cfg, nd, pd, n, j, mt, ma, scores ? &scores[(size_t)n * 4] : NULL);
}

/* UP schedule_one.go#assume -> framework/types.go#NodeInfo.AddPod/RemovePod (update ±1) */
void or_reserve(or_nodes *nd, const or_pods *pd, uint32_t j, uint32_t n, int sign) {
    nd->req_cpu[n] += sign * pd->req_cpu[j];
    nd->req_mem[n] += sign * pd->req_mem[j];
    for (int k = 0; k < OR_MAX_EXT; k++)
        nd->req_ext[n * OR_MAX_EXT + k] += sign * pd->req_ext[j * OR_MAX_EXT + k];
    nd->nz_cpu[n] += sign * pd->nz_cpu[j];
    nd->nz_mem[n] += sign * pd->nz_mem[j];
    nd->pods[n] += sign;
}

/* spec S8: stable order by (qos desc, priority desc, arrival asc) — bottom-up stable merge sort
 * (shape of UP queuesort/priority_sort.go#Less with QoS rank ahead of priority). */
static void order_pods(const or_config *cfg, const or_pods *pd, uint32_t *order) {
    uint32_t P = pd->p;
    for (uint32_t j = 0; j < P; j++) order[j] = j;
    if (!cfg->qos_sort) return;
    uint32_t *tmp = (uint32_t *)malloc(sizeof(uint32_t) * (P ? P : 1));
    for (uint32_t j = 0; j < P; j++) tmp[j] = j;
    uint32_t *a = tmp, *b = order;
    for (uint32_t width = 1; width < P; width *= 2) {
        for (uint32_t lo = 0; lo < P; lo += 2 * width) {
            uint32_t mid = lo + width < P ? lo + width : P;
            uint32_t hi = lo + 2 * width < P ? lo + 2 * width : P;
            uint32_t i = lo, k = mid, o = lo;
            while (i < mid && k < hi) {
                uint32_t x = a[i], y = a[k];
                /* compare (qos desc, priority desc); equal -> take left (stable) */
                int64_t rx = (int64_t)pd->qos[x] * 4294967296LL + pd->priority[x];
                int64_t ry = (int64_t)pd->qos[y] * 4294967296LL + pd->priority[y];
                if (ry > rx) b[o++] = a[k++]; else b[o++] = a[i++];
            }
            while (i < mid) b[o++] = a[i++];
            while (k < hi) b[o++] = a[k++];
        }
        uint32_t *t = a; a = b; b = t;
    }
    if (a != order) memcpy(order, a, sizeof(uint32_t) * P);
    free(tmp);
}

void or_schedule(const or_config *cfg, or_nodes *nd, const or_pods *pd, int32_t *placement,
                 uint64_t *best_key, uint32_t *order_out, int nthreads) {
    uint32_t P = pd->p;
    uint32_t *order = (uint32_t *)malloc(sizeof(uint32_t) * (P ? P : 1));
    order_pods(cfg, pd, order);
    if (nthreads < 1) nthreads = 1;
    for (uint32_t s = 0; s < P; s++) {
        uint32_t j = order[s];
        int64_t mt, ma;
        norm_maxima(cfg, nd, pd, j, &mt, &ma, nthreads);
        uint64_t best = 0;
        int64_t n_ = nd->n;
        /* UP schedule_one.go#findNodesThatPassFilters + prioritizeNodes (Parallelizer over
         * nodes) fused with the deterministic selectHost of spec S7 (max of unique keys). */
#pragma omp parallel for reduction(max : best) num_threads(nthreads) if (nthreads > 1)
        for (int64_t n = 0; n < n_; n++) {
            uint64_t k = node_key(cfg, nd, pd, (uint32_t)n, j, mt, ma, NULL);
            if (k > best) best = k;
        }
        if (best_key) best_key[j] = best;
        if (best == 0) {
            placement[j] = -1;
        } else {
            uint32_t n = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
            placement[j] = (int32_t)n;
            or_reserve(nd, pd, j, n, +1);
        }
    }
    if (order_out) memcpy(order_out, order, sizeof(uint32_t) * P);
    free(order);
}

/* ---------------- exact stream, incremental argmax (same semantics as or_schedule) ----------
 * For profiles without NormalizeScore plugins (TaintToleration / NodeAffinity off) a node's key
 * for pod j depends only on the node's row and on the pod's "type" — its requests, non-zero
 * requests, extended requests and QoS class (weights) — and a Reserve changes exactly one row.
 * So instead of re-scoring all N nodes per pod, keep per pod type a max segment tree over the
 * nodes' packed keys (node_key(), the very function or_schedule evaluates; keys are unique and
 * embed ~index, so the root is spec S7's selectHost), and after each Reserve re-score only the
 * reserved node, once per type seen so far.  Identical placements, keys and final table to
 * or_schedule (tests/test_oracle_incremental.py checks that, bit for bit); used where the
 * brute-force oracle would take minutes (config 3: 50,000 nodes x 1,000,000 pods).
 * Returns 0, or -1 when the profile normalizes or the per-type trees would exceed `max_bytes`. */
typedef struct {
    int64_t f[7]; /* req_cpu, req_mem, req_ext[0], req_ext[1], nz_cpu, nz_mem, qos */
    uint32_t rep; /* a pod of this type (its arrival index) */
    uint64_t *tree; /* [2M] max tree, leaves at M + n */
} or_type;

static void type_fields(const or_pods *pd, uint32_t j, int64_t f[7]) {
    f[0] = pd->req_cpu[j]; f[1] = pd->req_mem[j];
    f[2] = pd->req_ext[j * OR_MAX_EXT]; f[3] = pd->req_ext[j * OR_MAX_EXT + 1];
    f[4] = pd->nz_cpu[j]; f[5] = pd->nz_mem[j]; f[6] = pd->qos[j];
}

static uint64_t type_hash(const int64_t f[7]) {
    uint64_t h = 0x9E3779B97F4A7C15ULL;
    for (int i = 0; i < 7; i++) {
        h ^= (uint64_t)f[i] + 0x9E3779B97F4A7C15ULL + (h << 6) + (h >> 2);
        h *= 0xBF58476D1CE4E5B9ULL;
    }
    return h ^ (h >> 31);
}

int or_schedule_incremental(const or_config *cfg, or_nodes *nd, const or_pods *pd, int32_t *placement,
                            uint64_t *best_key, uint32_t *order_out, int nthreads, uint64_t max_bytes) {
    if (cfg->enable_taint || cfg->enable_affinity) return -1;
    const uint32_t P = pd->p, N = nd->n;
    if (nthreads < 1) nthreads = 1;
    uint32_t M = 1;
    while (M < (N ? N : 1)) M <<= 1;
    const size_t tree_bytes = sizeof(uint64_t) * 2 * (size_t)M;
    uint32_t *order = (uint32_t *)malloc(sizeof(uint32_t) * (P ? P : 1));
    order_pods(cfg, pd, order);
    uint32_t cap = 0, T = 0, hcap = 1024;
    or_type *types = NULL;
    int32_t *htab = (int32_t *)malloc(sizeof(int32_t) * hcap); /* open addressing -> type index */
    for (uint32_t i = 0; i < hcap; i++) htab[i] = -1;
    int rc = 0;
    for (uint32_t s = 0; s < P; s++) {
        const uint32_t j = order[s];
        int64_t f[7];
        type_fields(pd, j, f);
        uint32_t h = (uint32_t)type_hash(f) & (hcap - 1);
        int32_t t = -1;
        while (htab[h] >= 0) {
            if (memcmp(types[htab[h]].f, f, sizeof f) == 0) { t = htab[h]; break; }
            h = (h + 1) & (hcap - 1);
        }
        if (t < 0) { /* a new type: its tree over the current table */
            if ((uint64_t)(T + 1) * tree_bytes > max_bytes) { rc = -1; break; }
            if (T == cap) {
                cap = cap ? 2 * cap : 64;
                types = (or_type *)realloc(types, sizeof(or_type) * cap);
            }
            if (2 * (T + 1) > hcap) { /* grow the hash table (load <= 1/2) */
                uint32_t nh = 2 * hcap;
                int32_t *nt = (int32_t *)malloc(sizeof(int32_t) * nh);
                for (uint32_t i = 0; i < nh; i++) nt[i] = -1;
                for (uint32_t u = 0; u < T; u++) {
                    uint32_t g = (uint32_t)type_hash(types[u].f) & (nh - 1);
                    while (nt[g] >= 0) g = (g + 1) & (nh - 1);
                    nt[g] = (int32_t)u;
                }
                free(htab);
                htab = nt;
                hcap = nh;
                h = (uint32_t)type_hash(f) & (hcap - 1);
                while (htab[h] >= 0) h = (h + 1) & (hcap - 1);
            }
            or_type *ty = &types[T];
            memcpy(ty->f, f, sizeof f);
            ty->rep = j;
            ty->tree = (uint64_t *)calloc(2 * (size_t)M, sizeof(uint64_t));
            uint64_t *tr = ty->tree;
            int64_t n_ = N;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
            for (int64_t n = 0; n < n_; n++) tr[M + n] = node_key(cfg, nd, pd, (uint32_t)n, j, 0, 0, NULL);
            for (uint32_t v = M - 1; v >= 1; v--) tr[v] = tr[2 * v] > tr[2 * v + 1] ? tr[2 * v] : tr[2 * v + 1];
            htab[h] = (int32_t)T;
            t = (int32_t)T++;
        }
        const uint64_t best = types[t].tree[1];
        if (best_key) best_key[j] = best;
        if (best == 0) {
            placement[j] = -1;
            continue;
        }
        const uint32_t n = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
        placement[j] = (int32_t)n;
        or_reserve(nd, pd, j, n, +1);
        /* the reserved node's key changes for every type: re-score it and fix the tree paths */
        int64_t T_ = T;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1 && T_ >= 64)
        for (int64_t u = 0; u < T_; u++) {
            uint64_t *tr = types[u].tree;
            uint32_t v = M + n;
            tr[v] = node_key(cfg, nd, pd, n, types[u].rep, 0, 0, NULL);
            for (v >>= 1; v >= 1; v >>= 1) {
                const uint64_t m = tr[2 * v] > tr[2 * v + 1] ? tr[2 * v] : tr[2 * v + 1];
                if (tr[v] == m) break; /* unchanged from here up */
                tr[v] = m;
            }
        }
    }
    if (order_out) memcpy(order_out, order, sizeof(uint32_t) * P);
    for (uint32_t u = 0; u < T; u++) free(types[u].tree);
    free(types);
    free(htab);
    free(order);
    return rc;
}

/* ---------------- spec S11: batched mode ---------------- */
#define OR_LIST 64
#define OR_APPS 1024
#define OR_ZONES 64

static int cmp_key_desc(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? 1 : (x > y ? -1 : 0);
}

/* required anti-affinity of pod j against node n (UP plugins/interpodaffinity, the config-5
 * subset: a term selecting the pod's own app, topologyKey hostname or zone) */
static int aa_ok(const or_pods *pd, uint32_t j, uint32_t n, const uint8_t *present,
                 const int32_t *zcount, const or_nodes *nd) {
    int32_t app = pd->app[j], aa = pd->anti_affinity[j];
    if (aa == 1) return !present[(size_t)app * nd->n + n];
    if (aa == 2) return zcount[app * OR_ZONES + nd->zone[n]] == 0;
    return 1;
}

uint32_t or_schedule_batched(const or_config *cfg, or_nodes *nd, const or_pods *pd, uint32_t batch,
                             int32_t *placement, uint64_t *best_key, int nthreads) {
    uint32_t P = pd->p, N = nd->n;
    if (batch == 0 || batch > OR_LIST) batch = OR_LIST;
    if (nthreads < 1) nthreads = 1;
    uint32_t *order = (uint32_t *)malloc(sizeof(uint32_t) * (P ? P : 1));
    order_pods(cfg, pd, order);
    uint8_t *present = (uint8_t *)calloc((size_t)OR_APPS * (N ? N : 1), 1);
    int32_t *zcount = (int32_t *)calloc((size_t)OR_APPS * OR_ZONES, sizeof(int32_t));
    uint8_t *claimed = (uint8_t *)calloc(N ? N : 1, 1);
    uint8_t *claimed_az = (uint8_t *)calloc((size_t)OR_APPS * OR_ZONES, 1);
    uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * (N ? N : 1));
    uint64_t(*lists)[OR_LIST] = malloc(sizeof(uint64_t) * OR_LIST * batch);
    uint32_t cur[OR_LIST], pend[OR_LIST], nb = 0, npend = 0, cursor = 0, batches = 0;
    int32_t won[OR_LIST];
    nb = P < batch ? P : batch;
    for (uint32_t i = 0; i < nb; i++) cur[i] = i;
    cursor = nb;
    while (nb > 0) {
        ++batches;
        /* each pod's 64 best keys against the batch-start state */
        for (uint32_t i = 0; i < nb; i++) {
            uint32_t j = order[cur[i]];
            int64_t n_ = N;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
            for (int64_t n = 0; n < n_; n++) {
                uint64_t k = node_key(cfg, nd, pd, (uint32_t)n, j, 0, 0, NULL);
                keys[n] = (k && aa_ok(pd, j, (uint32_t)n, present, zcount, nd)) ? k : 0;
            }
            /* the 64 largest keys (keys are unique): a bounded selection, then sorted */
            uint64_t top[OR_LIST];
            uint32_t nt = 0;
            for (uint32_t n = 0; n < N; n++) {
                uint64_t k = keys[n];
                if (!k) continue;
                if (nt < OR_LIST) { top[nt++] = k; continue; }
                uint32_t mi = 0;
                for (uint32_t t = 1; t < OR_LIST; t++) if (top[t] < top[mi]) mi = t;
                if (k > top[mi]) top[mi] = k;
            }
            qsort(top, nt, sizeof(uint64_t), cmp_key_desc);
            for (uint32_t t = 0; t < OR_LIST; t++) lists[i][t] = t < nt ? top[t] : 0;
        }
        /* claims in batch order */
        memset(claimed, 0, N ? N : 1);
        memset(claimed_az, 0, (size_t)OR_APPS * OR_ZONES);
        npend = 0;
        for (uint32_t i = 0; i < nb; i++) {
            uint32_t j = order[cur[i]];
            uint64_t best = 0;
            int any = 0;
            for (uint32_t t = 0; t < OR_LIST; t++) {
                uint64_t k = lists[i][t];
                if (!k) continue;
                any = 1;
                uint32_t n = 0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFu);
                if (claimed[n]) continue;
                if (pd->anti_affinity[j] == 2 && claimed_az[pd->app[j] * OR_ZONES + nd->zone[n]]) continue;
                if (k > best) best = k;
            }
            won[i] = -2;
            if (best) {
                uint32_t n = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
                claimed[n] = 1;
                if (pd->anti_affinity[j] == 2) claimed_az[pd->app[j] * OR_ZONES + nd->zone[n]] = 1;
                won[i] = (int32_t)n;
                if (best_key) best_key[j] = best;
            } else if (any) {
                pend[npend++] = cur[i];
            } else {
                won[i] = -1;
                if (best_key) best_key[j] = 0;
            }
        }
        /* apply the batch */
        for (uint32_t i = 0; i < nb; i++) {
            uint32_t j = order[cur[i]];
            if (won[i] == -2) continue;
            placement[j] = won[i];
            if (won[i] >= 0) {
                uint32_t n = (uint32_t)won[i];
                or_reserve(nd, pd, j, n, +1);
                present[(size_t)pd->app[j] * N + n] = 1;
                zcount[pd->app[j] * OR_ZONES + nd->zone[n]]++;
            }
        }
        /* next batch: carried pods first, then fresh ones */
        uint32_t take = batch - npend;
        if (take > P - cursor) take = P - cursor;
        for (uint32_t i = 0; i < npend; i++) cur[i] = pend[i];
        for (uint32_t i = 0; i < take; i++) cur[npend + i] = cursor + i;
        nb = npend + take;
        cursor += take;
    }
    free(order); free(present); free(zcount); free(claimed); free(claimed_az); free(keys); free(lists);
    return batches;
}

/* ---------------- spec S11 batched mode, incremental lists (same results as or_schedule_batched)
 * For Fit + Balanced (+ ext) profiles a node's key for pod j depends only on the node's row and the
 * pod's type (type_fields), and a batch changes at most `batch` rows (the claimed nodes).  Per pod
 * type and topology zone a max tree over the zone's nodes' keys (node_key(), as or_schedule_batched
 * evaluates them); a pod's list = the 64 largest keys of the zones its anti-affinity allows, by a
 * best-first walk over those trees that skips hostname-anti-affinity nodes, i.e. the 64 largest
 * keys k != 0 with aa_ok, in descending order — exactly or_schedule_batched's list.  Claims and
 * the apply step are or_schedule_batched's.  After a batch only the claimed nodes are re-scored,
 * once per type.  tests/test_oracle_incremental.py diffs it against or_schedule_batched bit for bit;
 * used for config 5's full 10,000 x 200,000 check, where the brute-force oracle takes minutes.
 * Returns the number of batches, or 0xFFFFFFFF for normalizing profiles / zones >= 64. */
typedef struct {
    int64_t f[7];
    uint32_t rep;
    uint64_t *tree; /* per zone z: [2 * zM[z]] at zoff[z] */
} or_btype;
typedef struct { uint64_t key; uint32_t z, v; } or_hent;

static void heap_push(or_hent **h, uint32_t *n, uint32_t *cap, or_hent e) {
    if (*n == *cap) { *cap = *cap ? 2 * *cap : 256; *h = (or_hent *)realloc(*h, sizeof(or_hent) * *cap); }
    or_hent *a = *h;
    uint32_t i = (*n)++;
    while (i > 0) {
        uint32_t p = (i - 1) / 2;
        if (a[p].key >= e.key) break;
        a[i] = a[p];
        i = p;
    }
    a[i] = e;
}
static or_hent heap_pop(or_hent *a, uint32_t *n) {
    or_hent top = a[0], last = a[--(*n)];
    uint32_t i = 0;
    for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= *n) break;
        if (c + 1 < *n && a[c + 1].key > a[c].key) c++;
        if (a[c].key <= last.key) break;
        a[i] = a[c];
        i = c;
    }
    if (*n) a[i] = last;
    return top;
}

typedef struct {
    or_btype *types;
    uint32_t T, cap, hcap;
    int32_t *htab;
    const uint32_t *zM, *zoff, *leaf;
} or_bset;
/* The type of pod j; its per-zone trees are built over the current table on first sight. */
static int32_t bt_type_of(or_bset *bs, const or_config *cfg, const or_nodes *nd, const or_pods *pd, uint32_t j,
                          int nthreads) {
    int64_t f[7];
    type_fields(pd, j, f);
    uint32_t h = (uint32_t)type_hash(f) & (bs->hcap - 1);
    while (bs->htab[h] >= 0) {
        if (memcmp(bs->types[bs->htab[h]].f, f, sizeof f) == 0) return bs->htab[h];
        h = (h + 1) & (bs->hcap - 1);
    }
    if (bs->T == bs->cap) {
        bs->cap = bs->cap ? 2 * bs->cap : 64;
        bs->types = (or_btype *)realloc(bs->types, sizeof(or_btype) * bs->cap);
    }
    if (2 * (bs->T + 1) > bs->hcap) { /* grow the hash table (load <= 1/2) */
        uint32_t nh = 2 * bs->hcap;
        int32_t *nt = (int32_t *)malloc(sizeof(int32_t) * nh);
        for (uint32_t i = 0; i < nh; i++) nt[i] = -1;
        for (uint32_t u = 0; u < bs->T; u++) {
            uint32_t g = (uint32_t)type_hash(bs->types[u].f) & (nh - 1);
            while (nt[g] >= 0) g = (g + 1) & (nh - 1);
            nt[g] = (int32_t)u;
        }
        free(bs->htab);
        bs->htab = nt;
        bs->hcap = nh;
        h = (uint32_t)type_hash(f) & (nh - 1);
        while (bs->htab[h] >= 0) h = (h + 1) & (nh - 1);
    }
    or_btype *ty = &bs->types[bs->T];
    memcpy(ty->f, f, sizeof f);
    ty->rep = j;
    const uint32_t *zM = bs->zM, *zoff = bs->zoff, *leaf = bs->leaf;
    ty->tree = (uint64_t *)calloc(zoff[OR_ZONES] ? zoff[OR_ZONES] : 1, sizeof(uint64_t));
    uint64_t *tr = ty->tree;
    const int64_t N = nd->n;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1)
    for (int64_t n = 0; n < N; n++) {
        const int z = nd->zone[n];
        tr[zoff[z] + zM[z] + leaf[n]] = node_key(cfg, nd, pd, (uint32_t)n, j, 0, 0, NULL);
    }
    for (int z = 0; z < OR_ZONES; z++) {
        uint64_t *b = tr + zoff[z];
        for (uint32_t v = zM[z] ? zM[z] - 1 : 0; v >= 1; v--) b[v] = b[2 * v] > b[2 * v + 1] ? b[2 * v] : b[2 * v + 1];
    }
    bs->htab[h] = (int32_t)bs->T;
    return (int32_t)bs->T++;
}

uint32_t or_schedule_batched_incremental(const or_config *cfg, or_nodes *nd, const or_pods *pd, uint32_t batch,
                                         int32_t *placement, uint64_t *best_key, int nthreads) {
    if (cfg->enable_taint || cfg->enable_affinity) return 0xFFFFFFFFu;
    uint32_t P = pd->p, N = nd->n;
    if (batch == 0 || batch > OR_LIST) batch = OR_LIST;
    if (nthreads < 1) nthreads = 1;
    /* zones: node lists in index order, leaf positions, tree offsets */
    uint32_t zcnt[OR_ZONES] = {0}, zM[OR_ZONES], zoff[OR_ZONES + 1];
    for (uint32_t n = 0; n < N; n++) {
        if (nd->zone[n] < 0 || nd->zone[n] >= OR_ZONES) return 0xFFFFFFFFu;
        zcnt[nd->zone[n]]++;
    }
    zoff[0] = 0;
    for (int z = 0; z < OR_ZONES; z++) {
        uint32_t m = 1;
        while (m < zcnt[z]) m <<= 1;
        zM[z] = zcnt[z] ? m : 0;
        zoff[z + 1] = zoff[z] + 2 * zM[z];
    }
    uint32_t *znodes = (uint32_t *)malloc(sizeof(uint32_t) * (N ? N : 1)); /* zone-major node lists */
    uint32_t *zbase = (uint32_t *)calloc(OR_ZONES + 1, sizeof(uint32_t));
    uint32_t *leaf = (uint32_t *)malloc(sizeof(uint32_t) * (N ? N : 1)); /* node -> position in its zone */
    for (int z = 0; z < OR_ZONES; z++) zbase[z + 1] = zbase[z] + zcnt[z];
    {
        uint32_t fill[OR_ZONES] = {0};
        for (uint32_t n = 0; n < N; n++) {
            const int z = nd->zone[n];
            leaf[n] = fill[z]++;
            znodes[zbase[z] + leaf[n]] = n;
        }
    }
    uint32_t *order = (uint32_t *)malloc(sizeof(uint32_t) * (P ? P : 1));
    order_pods(cfg, pd, order);
    uint8_t *present = (uint8_t *)calloc((size_t)OR_APPS * (N ? N : 1), 1);
    int32_t *zcount = (int32_t *)calloc((size_t)OR_APPS * OR_ZONES, sizeof(int32_t));
    uint8_t *claimed = (uint8_t *)calloc(N ? N : 1, 1);
    uint8_t *claimed_az = (uint8_t *)calloc((size_t)OR_APPS * OR_ZONES, 1);
    uint64_t(*lists)[OR_LIST] = malloc(sizeof(uint64_t) * OR_LIST * batch);
    int32_t tix[OR_LIST];
    uint32_t cur[OR_LIST], pend[OR_LIST], nb = 0, npend = 0, cursor = 0, batches = 0;
    int32_t won[OR_LIST];
    or_bset bs = {0};
    bs.hcap = 1024;
    bs.htab = (int32_t *)malloc(sizeof(int32_t) * bs.hcap);
    for (uint32_t i = 0; i < bs.hcap; i++) bs.htab[i] = -1;
    bs.zM = zM;
    bs.zoff = zoff;
    bs.leaf = leaf;
    nb = P < batch ? P : batch;
    for (uint32_t i = 0; i < nb; i++) cur[i] = i;
    cursor = nb;
    while (nb > 0) {
        ++batches;
        for (uint32_t i = 0; i < nb; i++)
            tix[i] = bt_type_of(&bs, cfg, nd, pd, order[cur[i]], nthreads);
        /* each pod's 64 best keys against the batch-start state (best-first over allowed zones) */
        int64_t nb_ = nb;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1) schedule(dynamic, 1)
        for (int64_t i = 0; i < nb_; i++) {
            const uint32_t j = order[cur[i]];
            const int32_t app = pd->app[j], aa = pd->anti_affinity[j];
            const uint64_t *tr = bs.types[tix[i]].tree;
            or_hent *hp = NULL;
            uint32_t hn = 0, hc = 0, nt = 0;
            for (int z = 0; z < OR_ZONES; z++) {
                if (!zM[z]) continue;
                if (aa == 2 && zcount[app * OR_ZONES + z] != 0) continue;
                const uint64_t k = tr[zoff[z] + 1]; /* the root (a single node's leaf when zM = 1) */
                if (k) heap_push(&hp, &hn, &hc, (or_hent){k, (uint32_t)z, 1u});
            }
            while (hn > 0 && nt < OR_LIST) {
                const or_hent e = heap_pop(hp, &hn);
                const uint32_t z = e.z, M = zM[z];
                if (e.v >= M) { /* a leaf: node znodes[zbase[z] + v - M] */
                    const uint32_t n = znodes[zbase[z] + (e.v - M)];
                    if (aa == 1 && present[(size_t)app * N + n]) continue;
                    lists[i][nt++] = e.key;
                    continue;
                }
                const uint64_t *b = tr + zoff[z];
                const uint32_t l = 2 * e.v, r = 2 * e.v + 1;
                if (b[l]) heap_push(&hp, &hn, &hc, (or_hent){b[l], z, l});
                if (b[r]) heap_push(&hp, &hn, &hc, (or_hent){b[r], z, r});
            }
            for (uint32_t t = nt; t < OR_LIST; t++) lists[i][t] = 0;
            free(hp);
        }
        /* claims in batch order (or_schedule_batched) */
        memset(claimed, 0, N ? N : 1);
        memset(claimed_az, 0, (size_t)OR_APPS * OR_ZONES);
        npend = 0;
        for (uint32_t i = 0; i < nb; i++) {
            uint32_t j = order[cur[i]];
            uint64_t best = 0;
            int any = 0;
            for (uint32_t t = 0; t < OR_LIST; t++) {
                uint64_t k = lists[i][t];
                if (!k) continue;
                any = 1;
                uint32_t n = 0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFu);
                if (claimed[n]) continue;
                if (pd->anti_affinity[j] == 2 && claimed_az[pd->app[j] * OR_ZONES + nd->zone[n]]) continue;
                if (k > best) best = k;
            }
            won[i] = -2;
            if (best) {
                uint32_t n = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
                claimed[n] = 1;
                if (pd->anti_affinity[j] == 2) claimed_az[pd->app[j] * OR_ZONES + nd->zone[n]] = 1;
                won[i] = (int32_t)n;
                if (best_key) best_key[j] = best;
            } else if (any) {
                pend[npend++] = cur[i];
            } else {
                won[i] = -1;
                if (best_key) best_key[j] = 0;
            }
        }
        /* apply the batch, then re-score the claimed nodes for every type */
        uint32_t chg[OR_LIST], nchg = 0;
        for (uint32_t i = 0; i < nb; i++) {
            uint32_t j = order[cur[i]];
            if (won[i] == -2) continue;
            placement[j] = won[i];
            if (won[i] >= 0) {
                uint32_t n = (uint32_t)won[i];
                or_reserve(nd, pd, j, n, +1);
                present[(size_t)pd->app[j] * N + n] = 1;
                zcount[pd->app[j] * OR_ZONES + nd->zone[n]]++;
                chg[nchg++] = n;
            }
        }
        int64_t T_ = bs.T;
#pragma omp parallel for num_threads(nthreads) if (nthreads > 1 && T_ >= 16)
        for (int64_t u = 0; u < T_; u++) {
            for (uint32_t c = 0; c < nchg; c++) {
                const uint32_t n = chg[c];
                const int z = nd->zone[n];
                uint64_t *b = bs.types[u].tree + zoff[z];
                uint32_t v = zM[z] + leaf[n];
                b[v] = node_key(cfg, nd, pd, n, bs.types[u].rep, 0, 0, NULL);
                for (v >>= 1; v >= 1; v >>= 1) {
                    const uint64_t m = b[2 * v] > b[2 * v + 1] ? b[2 * v] : b[2 * v + 1];
                    if (b[v] == m) break;
                    b[v] = m;
                }
            }
        }
        uint32_t take = batch - npend;
        if (take > P - cursor) take = P - cursor;
        for (uint32_t i = 0; i < npend; i++) cur[i] = pend[i];
        for (uint32_t i = 0; i < take; i++) cur[npend + i] = cursor + i;
        nb = npend + take;
        cursor += take;
    }
    for (uint32_t u = 0; u < bs.T; u++) free(bs.types[u].tree);
    free(bs.types); free(bs.htab); free(znodes); free(zbase); free(leaf);
    free(order); free(present); free(zcount); free(claimed); free(claimed_az); free(lists);
    return batches;
}

/* ---------------- spec/synth.md generator (independent restatement) ---------------- */
static uint64_t sm_at(uint64_t seed, uint64_t c) {
    uint64_t z = seed + (c + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint32_t pick(uint64_t seed, uint64_t c, uint32_t k) { return (uint32_t)((sm_at(seed, c) >> 33) % k); }

static const int64_t NODE_CPU[6] = {4000, 8000, 16000, 32000, 64000, 96000};
static const int64_t NODE_MPC[3] = {2, 4, 8};
static const int64_t POD_CPU[6] = {500, 1000, 1500, 2000, 4000, 8000};
static const int64_t POD_MEM[7] = {128, 256, 512, 1024, 2048, 4096, 8192};
static const int64_t GPU_CNT[4] = {1, 2, 4, 8};
#define GIB (1LL << 30)
#define MIB (1LL << 20)
#define DEF_CPU 100
#define DEF_MEM (200 * MIB)

static int pair_bit(int za, int zb) { /* za < zb, lexicographic index of the pair, + 3 */
    int idx = 0;
    for (int a = 0; a < za; a++) idx += 9 - a;
    return 3 + idx + (zb - za - 1);
}

void or_generate(int config, uint64_t seed, or_nodes *nd, or_pods *pd) {
    uint32_t N = nd->n, P = pd->p;
    int c4 = (config == 4), c5 = (config == 5);
    for (uint32_t i = 0; i < N; i++) {
        uint64_t c = 8ULL * i;
        int64_t cpu = NODE_CPU[pick(seed, c + 0, 6)];
        int64_t mpc = NODE_MPC[pick(seed, c + 1, 3)];
        nd->alloc_cpu[i] = cpu;
        nd->alloc_mem[i] = (cpu / 1000) * mpc * GIB;
        nd->max_pods[i] = 110;
        nd->req_cpu[i] = nd->req_mem[i] = nd->nz_cpu[i] = nd->nz_mem[i] = nd->pods[i] = 0;
        for (int k = 0; k < OR_MAX_EXT; k++) nd->alloc_ext[i * OR_MAX_EXT + k] = nd->req_ext[i * OR_MAX_EXT + k] = 0;
        nd->taint_hard[i] = nd->taint_soft[i] = 0;
        nd->label_bits[2 * i] = nd->label_bits[2 * i + 1] = 0;
        if (nd->zone) nd->zone[i] = (c4 || c5) ? (int32_t)pick(seed, c + 4, 10) : 0;
        if (c4) {
            int gpu = pick(seed, c + 2, 10) == 0;
            int maint = pick(seed, c + 3, 20) == 0;
            int zone = (int)pick(seed, c + 4, 10);
            int pool = gpu ? 2 : (int)pick(seed, c + 5, 2); /* 0 general, 1 highmem, 2 gpu */
            int ssd = pick(seed, c + 6, 2) == 0;
            uint64_t lo = 0, hi = 0;
            if (gpu) { nd->alloc_ext[i * OR_MAX_EXT] = 8; nd->taint_hard[i] |= 1ULL << 0; }
            if (maint) nd->taint_soft[i] |= 1ULL << 1;
            if (pool == 2) lo |= 1ULL << 0;
            if (ssd) lo |= 1ULL << 1;
            if (pool == 1) lo |= 1ULL << 2;
            for (int a = 0; a < 10; a++)
                for (int b = a + 1; b < 10; b++)
                    if (a == zone || b == zone) {
                        int bit = pair_bit(a, b);
                        if (bit < 64) lo |= 1ULL << bit; else hi |= 1ULL << (bit - 64);
                    }
            nd->label_bits[2 * i] = lo;
            nd->label_bits[2 * i + 1] = hi;
        }
    }
    for (uint32_t j = 0; j < P; j++) {
        uint64_t c = 8ULL * N + 16ULL * j;
        uint32_t qd = pick(seed, c + 0, 10);
        int64_t cpu = POD_CPU[pick(seed, c + 1, 6)];
        int64_t mem = POD_MEM[pick(seed, c + 2, 7)] * MIB;
        uint32_t memmode = pick(seed, c + 3, 4);
        (void)pick(seed, c + 4, 2); /* limmode: affects the emitted limits only, not S2/S3 */
        int q = qd < 2 ? 2 : (qd < 7 ? 1 : 0);
        int64_t rc = 0, rm = 0, zc = DEF_CPU, zm = DEF_MEM;
        if (q == 2) { rc = zc = cpu; rm = zm = mem; }
        else if (q == 1) { rc = zc = cpu; if (memmode != 0) { rm = zm = mem; } }
        pd->req_cpu[j] = rc; pd->req_mem[j] = rm; pd->nz_cpu[j] = zc; pd->nz_mem[j] = zm;
        pd->qos[j] = q; pd->priority[j] = 0;
        if (pd->app) {
            pd->app[j] = 0;
            pd->anti_affinity[j] = 0;
            if (c5) { /* spec/synth.md G5 */
                pd->app[j] = (int32_t)pick(seed, c + 13, 1000);
                uint32_t kind = pick(seed, 8ULL * N + 16ULL * P + (uint64_t)pd->app[j], 10);
                pd->anti_affinity[j] = kind < 5 ? 1 : (kind == 5 ? 2 : 0);
            }
        }
        for (int k = 0; k < OR_MAX_EXT; k++) pd->req_ext[j * OR_MAX_EXT + k] = 0;
        pd->tol_hard[j] = pd->tol_soft[j] = 0;
        pd->sel[2 * j] = pd->sel[2 * j + 1] = 0;
        pd->n_req_terms[j] = pd->n_pref_terms[j] = 0;
        for (int t = 0; t < OR_MAX_TERMS; t++) {
            size_t o = ((size_t)j * OR_MAX_TERMS + t) * 2;
            pd->req_terms[o] = pd->req_terms[o + 1] = pd->pref_terms[o] = pd->pref_terms[o + 1] = 0;
            pd->pref_weight[j * OR_MAX_TERMS + t] = 0;
        }
        if (c4) {
            if (pick(seed, c + 5, 20) == 0) {
                pd->req_ext[j * OR_MAX_EXT] = GPU_CNT[pick(seed, c + 6, 4)];
                pd->tol_hard[j] |= 1ULL << 0;
                pd->sel[2 * j] |= 1ULL << 0;
            }
            if (pick(seed, c + 7, 5) == 0) {
                int za = (int)pick(seed, c + 8, 10);
                int zb = (za + 1 + (int)pick(seed, c + 9, 9)) % 10;
                int a = za < zb ? za : zb, b = za < zb ? zb : za;
                int bit = pair_bit(a, b);
                size_t o = ((size_t)j * OR_MAX_TERMS) * 2;
                if (bit < 64) pd->req_terms[o] |= 1ULL << bit; else pd->req_terms[o + 1] |= 1ULL << (bit - 64);
                pd->n_req_terms[j] = 1;
            }
            if (pick(seed, c + 10, 5) == 0) {
                uint32_t which = pick(seed, c + 11, 3);
                int t = 0;
                if (which == 0 || which == 2) {
                    pd->pref_terms[((size_t)j * OR_MAX_TERMS + t) * 2] = 1ULL << 1;
                    pd->pref_weight[j * OR_MAX_TERMS + t] = 50; t++;
                }
                if (which == 1 || which == 2) {
                    pd->pref_terms[((size_t)j * OR_MAX_TERMS + t) * 2] = 1ULL << 2;
                    pd->pref_weight[j * OR_MAX_TERMS + t] = 20; t++;
                }
                pd->n_pref_terms[j] = t;
            }
            if (pick(seed, c + 12, 10) == 0) pd->tol_soft[j] |= 1ULL << 1;
        }
    }
}
