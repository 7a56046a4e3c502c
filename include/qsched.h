/*
 * qsched.h — C ABI of libqsched.so, the MI355X (gfx950) scheduling core.
 *
 * This is the drop-in boundary: the surface a kube-scheduler framework plugin
 * binds through cgo (or any FFI).  Plain C types only — no HIP, no torch, no C++.
 *
 * What each entry point replaces (upstream kube-scheduler v1.32, `UP <path>#<symbol>`; the mounted
 * reference /root/reference/README.md:1 is a title line, so there is no reference-side FFI to cite
 * beyond the north_star's "thin cgo C-ABI" in BASELINE.json:5):
 *   qs_open / qs_close        framework.Handle-scoped plugin state (UP cmd/kube-scheduler/app#WithPlugin
 *                             factory `func(ctx, runtime.Object, framework.Handle) (framework.Plugin, error)`)
 *   qs_nodes_load             Cache.UpdateSnapshot → Snapshot NodeInfo list (UP backend/cache#Snapshot)
 *   qs_node_upsert            per-NodeInfo Generation diff (UP framework/types.go#NodeInfo.Generation)
 *   qs_score_pod              PreFilter+Filter+PreScore+Score+NormalizeScore for ALL nodes of one pod
 *                             (UP framework/interface.go#{PreFilterPlugin,FilterPlugin,ScorePlugin,
 *                             ScoreExtensions}; UP schedule_one.go#{findNodesThatPassFilters,prioritizeNodes})
 *   qs_reserve / qs_unreserve ReservePlugin.Reserve / Unreserve → NodeInfo.AddPod / RemovePod
 *                             (UP framework/interface.go#ReservePlugin, framework/types.go#NodeInfo.update)
 *   qs_schedule_stream        ScheduleOne loop with deterministic selectHost (UP schedule_one.go#
 *                             {ScheduleOne,schedulingCycle,selectHost,assume}; spec/semantics.md S7/S8)
 *
 * Semantics: spec/semantics.md.  Ownership: every pointer argument is borrowed for the duration of
 * the call only (cgo rule: C never retains Go pointers); outputs go to caller-allocated arrays of
 * the stated length.  Quantities are canonical int64 (millicores, bytes, counts).  Errors are
 * return codes, never exceptions or aborts; `qs_last_error` holds the message.  Unschedulable is
 * not an error: placement −1.  Threading: one mutex per context serialises every call.
 */
#ifndef QSCHED_H
#define QSCHED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define QS_API __attribute__((visibility("default")))
#else
#define QS_API
#endif

#define QS_ABI_VERSION 3
#define QS_MAX_EXT 2   /* extended resources per node/pod (e.g. amd.com/gpu) */
#define QS_MAX_TERMS 4 /* node-affinity terms per pod (required OR-terms, preferred terms) */
#define QS_MAX_APPS 1024 /* anti-affinity groups (batched mode, spec S11) */
#define QS_MAX_ZONES 64  /* topology zones (batched mode zone anti-affinity) */
#define QS_MAX_SCORE_RES 4 /* entries of a scoring-resource list (cpu, memory, ext 0, ext 1) */

typedef enum qs_status {
    QS_OK = 0,
    QS_EINVAL = 1,   /* bad argument / input outside the device layout's range */
    QS_EDEVICE = 2,  /* HIP or RCCL failure (message in qs_last_error) */
    QS_ETIMEOUT = 3, /* an in-kernel wait (lookahead lists, resident hand-off, mailbox peer) hit its
                        0.5 s bound; the run is void and the device table rebuilt from the mirror */
    QS_ENOMEM = 4,
    QS_ESTATE = 5 /* call out of order (e.g. no nodes loaded) */
} qs_status;

typedef enum qs_qos { QS_QOS_BESTEFFORT = 0, QS_QOS_BURSTABLE = 1, QS_QOS_GUARANTEED = 2 } qs_qos;

typedef enum qs_mode { QS_MODE_EXACT = 0, QS_MODE_BATCHED = 1 } qs_mode;

/* Required pod anti-affinity to the pod's own app group (batched mode, spec S11; the subset of
 * UP plugins/interpodaffinity that config 5 uses): none, per node (topologyKey hostname), per zone. */
typedef enum qs_anti_affinity { QS_AA_NONE = 0, QS_AA_HOSTNAME = 1, QS_AA_ZONE = 2 } qs_anti_affinity;

/* Scoring resources (spec/semantics.md S5 "Scoring resources"): cpu, memory, or one of the table's
 * two extended-resource columns (the caller interns e.g. "amd.com/gpu" as QS_RES_EXT0). */
typedef enum qs_resource { QS_RES_NONE = 0, QS_RES_CPU = 1, QS_RES_MEMORY = 2, QS_RES_EXT0 = 3, QS_RES_EXT1 = 4 } qs_resource;
/* One entry of NodeResourcesFitArgs.ScoringStrategy.Resources (UP apis/config#ResourceSpec{Name, Weight}). */
typedef struct qs_resource_spec {
    int32_t resource; /* qs_resource */
    int32_t weight;   /* 1..100 (UP apis/config/validation#validateResources) */
} qs_resource_spec;

/* Which device engine runs the exact stream (all are bit-exact; AUTO picks the fastest). */
typedef enum qs_engine {
    QS_ENGINE_AUTO = 0,
    QS_ENGINE_PERSISTENT = 1, /* one resident workgroup, node rows in registers (N <= 8192) */
    QS_ENGINE_SCAN = 2,       /* per-pod grid scan + finalize/reserve launch chain (any N) */
    QS_ENGINE_LOOKAHEAD = 3,  /* exact top-K lookahead: chip-wide stale scan + sequential resolve */
    QS_ENGINE_BATCHED = 4,    /* reported by qs_stats.engine_used for QS_MODE_BATCHED streams */
    QS_ENGINE_ALLREDUCE = 5   /* sharded contexts with an RCCL communicator: per pod every rank scans its
                                 node shard and the ranks max-reduce one packed key with
                                 ncclAllReduce(count 1, ncclUint64, ncclMax) (+ the two normalize maxima for
                                 TaintToleration / NodeAffinity); the as-is RCCL baseline of SURVEY.md §8(e) C1 */
} qs_engine;

typedef struct qs_config {
    uint32_t abi_version;        /* = QS_ABI_VERSION */
    int32_t engine;              /* qs_engine */
    int64_t fit_weight_cpu;      /* NodeResourcesFitArgs.ScoringStrategy.Resources cpu weight (1) */
    int64_t fit_weight_mem;      /* ... memory weight (1) */
    int32_t w_fit[3];            /* NodeResourcesFit plugin weight per QoS class [BE, Bu, G] */
    int32_t w_bal[3];            /* NodeResourcesBalancedAllocation weight per QoS class */
    int32_t w_taint;             /* TaintToleration weight (3) */
    int32_t w_affinity;          /* NodeAffinity weight (2) */
    int32_t enable_taint;        /* TaintToleration filter+score on */
    int32_t enable_affinity;     /* NodeAffinity filter+score on */
    int32_t balanced_skip_besteffort; /* 0 = v1.32 behaviour */
    int32_t qos_sort;            /* 1 = QoSSort order (spec S8), 0 = arrival order */
    int32_t lookahead;           /* pods per lookahead window (0 = default) */
    int32_t record_timestamps;   /* 1 = per-pod device timestamps for p50/p99 cycle latency */
    int32_t profile_kernels;     /* 1 = time every kernel launch with HIP events (qs_stats.kernel_s) */
    int32_t virtual_shards;      /* >1: run the sharded LOOKAHEAD protocol with this many node shards
                                    inside one process (no collective; parity testing of the
                                    multi-GPU layout on one device).  Ignored by qs_open_shard. */
    int32_t lookahead_serial;    /* 1 = LOOKAHEAD windows back to back; 0 (default) = the select of
                                    window w+1 overlaps the resolve of window w (needs lookahead <= 32) */
    int32_t scan_soa_min_nodes;  /* tables with at least this many nodes also keep the column-major
                                    copy the SCAN engine / qs_score_pod stream (0 = 65,536; -1 never) */
    int32_t batch_pods;          /* QS_MODE_BATCHED: pods per batch (0 = 64; at most 64) */
    /* NodeResourcesFitArgs.ScoringStrategy.Resources of the LeastAllocated strategy, in list order
     * (replaces UP apis/config/types_pluginargs.go#ScoringStrategy.Resources); 0 entries = the
     * default [cpu: fit_weight_cpu, memory: fit_weight_mem].  Distinct resources, weights 1..100. */
    int32_t n_fit_resources;
    qs_resource_spec fit_resources[QS_MAX_SCORE_RES];
    /* NodeResourcesBalancedAllocationArgs.Resources in list order (UP types_pluginargs.go#
     * NodeResourcesBalancedAllocationArgs); 0 entries = the default [cpu, memory].  With three or
     * more resources requested the score takes the mean / sqrt standard deviation (spec S5). */
    int32_t n_balanced_resources;
    int32_t balanced_resources[QS_MAX_SCORE_RES]; /* qs_resource */
    int32_t reserved[3];
} qs_config;

/* Canonical node table, structure of arrays, n entries each.  alloc_ext/req_ext are [n][QS_MAX_EXT],
 * label_bits is [n][2], zone is the node's topology zone id (< QS_MAX_ZONES; batched-mode zone
 * anti-affinity).  Optional columns may be NULL (read as 0). */
typedef struct qs_node_soa {
    const int64_t *alloc_cpu, *alloc_mem, *alloc_ext, *max_pods;
    const int64_t *req_cpu, *req_mem, *req_ext, *nz_cpu, *nz_mem, *pods;
    const uint64_t *taint_hard, *taint_soft, *label_bits;
    const int32_t *zone;
} qs_node_soa;

/* Same layout, writable (qs_nodes_read, qs_synth_generate). */
typedef struct qs_node_soa_out {
    int64_t *alloc_cpu, *alloc_mem, *alloc_ext, *max_pods;
    int64_t *req_cpu, *req_mem, *req_ext, *nz_cpu, *nz_mem, *pods;
    uint64_t *taint_hard, *taint_soft, *label_bits;
    int32_t *zone;
} qs_node_soa_out;

typedef struct qs_node_row {
    int64_t alloc_cpu, alloc_mem, alloc_ext[QS_MAX_EXT], max_pods;
    int64_t req_cpu, req_mem, req_ext[QS_MAX_EXT], nz_cpu, nz_mem, pods;
    uint64_t taint_hard, taint_soft, label_bits[2];
    int32_t zone, reserved;
} qs_node_row;

/* One pod, precomputed on the host (spec S2/S3; qs_pod_from_containers helps). */
typedef struct qs_pod {
    int64_t req_cpu, req_mem, req_ext[QS_MAX_EXT]; /* effective requests, missing -> 0 */
    int64_t nz_cpu, nz_mem;                        /* non-zero requests (defaults 100m / 200Mi) */
    int32_t qos;                                   /* qs_qos */
    int32_t priority;
    uint64_t tol_hard; /* interned taint bits tolerated for NoSchedule/NoExecute */
    uint64_t tol_soft; /* interned taint bits tolerated for PreferNoSchedule */
    uint64_t sel[2];   /* nodeSelector requirement bits (all must hold) */
    int32_t n_req_terms, n_pref_terms;
    uint64_t req_terms[QS_MAX_TERMS][2];  /* required node-affinity terms (OR of ANDs) */
    uint64_t pref_terms[QS_MAX_TERMS][2]; /* preferred terms */
    int32_t pref_weight[QS_MAX_TERMS];
    int32_t app;           /* anti-affinity group (< QS_MAX_APPS) */
    int32_t anti_affinity; /* qs_anti_affinity: required anti-affinity to the pod's own app */
} qs_pod;

/* One container of a pod spec for qs_pod_from_containers (spec S2/S3). has_* = 0 means missing. */
typedef struct qs_container {
    int32_t kind; /* 0 regular, 1 init, 2 restartable init (sidecar) */
    int32_t has_req_cpu, has_req_mem, has_lim_cpu, has_lim_mem;
    int64_t req_cpu, req_mem, lim_cpu, lim_mem;
    int64_t req_ext[QS_MAX_EXT];
} qs_container;

typedef struct qs_stats {
    uint64_t pods, placed, unschedulable, evals;
    uint64_t batches, truncations;  /* lookahead windows run / pods resolved by an exact full
                                       rescan (normalizing profiles: a normalize maximum lost) */
    double wall_s;                  /* qs_stream_run wall, device-resident inputs */
    double h2d_s, d2h_s;            /* host<->device copies around it (qs_schedule_stream) */
    double p50_cycle_us, p99_cycle_us, max_cycle_us; /* per-pod decision interval (record_timestamps) */
    int32_t engine_used;
    int32_t table_layout;           /* device layout that ran: 0 compact (int32 columns, memory in
                                       2^u-byte units < 2^24), 1 wide (f64 memory columns in bytes) */
    uint64_t resumed_windows;       /* normalizing LOOKAHEAD: windows stopped for an exact rescan */
    uint64_t device_faults;         /* QS_EDEVICE results of this context so far (each one drops
                                       the device table; the next call rebuilds it from the mirror) */
    int32_t resident;               /* 1: LOOKAHEAD ran as one resident launch (resolver + selector
                                       workgroups, k_la_stream_res); 0: per-window launches */
    int32_t reserved;
    /* per-kernel device time (config.profile_kernels = 1; HIP events on the library's stream):
     * [0] persistent, [1] scan (all per-pod kernels), [2] lookahead select, [3] lookahead resolve
     * (a resident stream is one launch, counted under [3]) */
    double kernel_s[4];
    uint64_t kernel_launches[4];
} qs_stats;

typedef struct qs_ctx qs_ctx;
typedef struct qs_stream qs_stream;

/* ---- lifecycle ---- */
QS_API void qs_config_default(qs_config *cfg);
QS_API qs_status qs_open(const qs_config *cfg, int device, qs_ctx **out);
/* Sharded context for one rank of `world` (one process per GPU, world <= 16).  nccl_id = 128 bytes
 * from qs_dist_unique_id on rank 0, broadcast by the caller (any out-of-band channel); NULL selects
 * the peer-memory mailbox transport instead (qs_dist_mailbox_connect before the first stream).  Every rank
 * loads the SAME full node table (qs_nodes_load) and the SAME pod stream; rank r scores only its
 * contiguous node shard [r*n/world, (r+1)*n/world), the per-window top-L lists are exchanged with
 * one RCCL all-gather over xGMI, and every rank resolves the window identically, so placements and
 * the node table stay identical on all ranks.  Collective calls happen inside
 * qs_stream_run: all ranks must call it with the same stream. */
QS_API qs_status qs_open_shard(const qs_config *cfg, int device, int rank, int world,
                        const uint8_t nccl_id[128], qs_ctx **out);
QS_API qs_status qs_dist_unique_id(uint8_t out[128]);
/* Peer-memory mailbox transport, the alternative to RCCL: open
 * every rank with qs_open_shard(..., nccl_id = NULL, ...), call qs_dist_mailbox_export on each rank
 * (allocates this rank's ~5 MB mailbox and returns its 64-byte IPC handle), exchange the handles
 * out of band, and call qs_dist_mailbox_connect with all `world` handles in rank order.  Per
 * lookahead window every rank then writes its list block (and, for TaintToleration/NodeAffinity
 * profiles, its partial maxima) straight into every peer's mailbox over xGMI and raises a flag
 * there (one hop), instead of an RCCL all-gather; a peer that never posts makes the run return
 * QS_ETIMEOUT (bound: 5 s for a run's first window, 0.5 s for the others).  All ranks must run the
 * same streams in the same order.  After QS_ETIMEOUT the ranks are out of step: every later run
 * returns QS_ESTATE until every rank has called qs_dist_mailbox_connect again (the caller places a
 * barrier of its own before and after that call on every rank), which restarts all mailboxes empty.
 * Replaces (with qs_open_shard) the per-pod ncclAllReduce exchange of SURVEY.md §8(e). */
QS_API qs_status qs_dist_mailbox_export(qs_ctx *ctx, uint8_t handle[64]);
QS_API qs_status qs_dist_mailbox_connect(qs_ctx *ctx, const uint8_t *handles /* world x 64 bytes */);
QS_API qs_status qs_close(qs_ctx *ctx);
QS_API const char *qs_last_error(const qs_ctx *ctx);
QS_API const char *qs_version(void);

/* ---- node table (device-resident SoA, host mirror authoritative) ---- */
QS_API qs_status qs_nodes_load(qs_ctx *ctx, const qs_node_soa *nodes, uint32_t n);
QS_API qs_status qs_nodes_read(qs_ctx *ctx, const qs_node_soa_out *out, uint32_t n);
QS_API qs_status qs_node_upsert(qs_ctx *ctx, uint32_t idx, const qs_node_row *row, uint64_t generation);
/* Device-side snapshot of the whole node table (checkpoint/resume; bench resets between steps). */
QS_API qs_status qs_table_save(qs_ctx *ctx);
QS_API qs_status qs_table_restore(qs_ctx *ctx);
QS_API qs_status qs_reserve(qs_ctx *ctx, uint32_t node, const qs_pod *pod);
QS_API qs_status qs_unreserve(qs_ctx *ctx, uint32_t node, const qs_pod *pod);

/* ---- one pod, all nodes (framework-embedded path) ----
 * feasible_n (nullable): 1/0 per node; score_n (nullable): [n][4] {LeastAllocated, Balanced,
 * TaintToleration, NodeAffinity} normalized plugin scores (0 where infeasible); total_n (nullable):
 * QoS-weighted total per node (-1 where infeasible); best: node index of spec S7 or -1. */
QS_API qs_status qs_score_pod(qs_ctx *ctx, const qs_pod *pod, uint8_t *feasible_n, int32_t *score_n,
                       int32_t *total_n, int32_t *best);
/* The same call without the per-node copy-out: *packed_n (nullable) points at n context-owned words,
 * valid until the next call on ctx, one per node: 0xFFFFFFFF = infeasible, else the four normalized
 * plugin scores as bytes (LeastAllocated | Balanced << 8 | TaintToleration << 16 | NodeAffinity << 24).
 * The words are what the kernel wrote into pinned host memory, so a plugin's per-node Filter / Score
 * lookups read them in place (UP framework/interface.go#ScorePlugin.Score is called per node). */
QS_API qs_status qs_score_pod_packed(qs_ctx *ctx, const qs_pod *pod, const uint32_t **packed_n, int32_t *best);

/* ---- exact stream ---- */
QS_API qs_status qs_schedule_stream(qs_ctx *ctx, const qs_pod *pods, uint32_t p, qs_mode mode,
                             int32_t *placement_p, qs_stats *stats);
/* Split form: prepare (host precompute + H2D), run (device only, timed; may run again, e.g. after
 * qs_table_restore), results (D2H of the last run). */
QS_API qs_status qs_stream_prepare(qs_ctx *ctx, const qs_pod *pods, uint32_t p, qs_stream **out);
QS_API qs_status qs_stream_run(qs_ctx *ctx, qs_stream *s, qs_mode mode, qs_stats *stats);
QS_API qs_status qs_stream_results(qs_ctx *ctx, qs_stream *s, int32_t *placement_p, uint64_t *best_key_p);
QS_API qs_status qs_stream_free(qs_ctx *ctx, qs_stream *s);
/* Per-pod device timestamps (100 MHz s_memrealtime ticks, stream order; record_timestamps = 1). */
QS_API qs_status qs_stream_stamps(qs_ctx *ctx, qs_stream *s, uint64_t *stamps_p);
/* FitError diagnosis of an exact stream's unschedulable pods (replaces UP framework/types.go#FitError,
 * Diagnosis.NodeToStatusMap; the "0/N nodes are available: ..." message).  For each requested pod
 * (arrival index) the number of nodes that rejected it for each reason, against the table as it
 * stood when that pod was scheduled: the stream's device placements replayed over the host mirror.
 * A node counts under the first failing filter in upstream's default order (TaintToleration,
 * NodeAffinity, NodeResourcesFit) and, for NodeResourcesFit, under every insufficient resource
 * (UP noderesources/fit.go#fitsRequest).  counts = m x QS_FIT_REASONS; a placed pod gets zeros.
 * Call after qs_stream_run of an exact stream and before any other change to the table
 * (QS_ESTATE otherwise). */
typedef enum qs_fit_reason {
    QS_FIT_TOO_MANY_PODS = 0, /* "Too many pods" */
    QS_FIT_CPU = 1,           /* "Insufficient cpu" */
    QS_FIT_MEMORY = 2,        /* "Insufficient memory" */
    QS_FIT_EXT0 = 3,          /* "Insufficient <extended resource 0>" */
    QS_FIT_EXT1 = 4,          /* "Insufficient <extended resource 1>" */
    QS_FIT_TAINT = 5,         /* "node(s) had untolerated taint {key: value}" (split per taint:
                               * qs_stream_fit_taints) */
    QS_FIT_AFFINITY = 6,      /* "node(s) didn't match Pod's node affinity/selector" */
    QS_FIT_REASONS = 7
} qs_fit_reason;
QS_API qs_status qs_stream_fit_errors(qs_ctx *ctx, qs_stream *s, const uint32_t *pods, uint32_t m, uint32_t *counts);
/* The same counts, plus the QS_FIT_TAINT nodes split by taint (UP plugins/tainttoleration/
 * taint_toleration.go#Filter: "node(s) had untolerated taint {%s: %s}" names the FIRST untolerated
 * NoSchedule / NoExecute taint of the node, one reason string per distinct taint, which FitError.Error()
 * counts separately).  taint_counts = m x 64: per pod, per interned taint bit b, the nodes whose first
 * untolerated hard taint is bit b (the lowest set bit of taint_hard & ~tol_hard; the interning order
 * stands for the node's taint order, exact when every node lists its taints in interning order, as
 * the workload loader's and the synthetic generator's nodes do).  Row sums equal counts[QS_FIT_TAINT]. */
QS_API qs_status qs_stream_fit_taints(qs_ctx *ctx, qs_stream *s, const uint32_t *pods, uint32_t m, uint32_t *counts,
                                      uint32_t *taint_counts);

/* ---- host helpers (spec S2/S3, spec/synth.md) ---- */
QS_API qs_status qs_pod_from_containers(const qs_container *c, uint32_t nc, const int64_t *overhead_cpu_mem,
                                 qs_pod *out);
QS_API int32_t qs_compute_qos(const qs_container *c, uint32_t nc);
/* sizeof of the ABI structs for binding self-checks: 0 config, 1 node_soa, 2 node_row, 3 pod,
 * 4 container, 5 stats. */
QS_API size_t qs_struct_size(int which);
QS_API qs_status qs_synth_generate(int config, uint64_t seed, uint32_t n, uint32_t p,
                            const qs_node_soa_out *nodes, qs_pod *pods);

#ifdef __cplusplus
}
#endif
#endif /* QSCHED_H */
