// qs_launch.hpp — host-callable launchers of the gfx950 kernels (defined in qs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace qs {

struct DevTable;
struct DevCfg;
struct DPodX;  // pod records are DPod (compact layout) or DPodW (wide layout): passed as void*

// One node row for k_set_row (by value).  Compact layout: the int32 fields; wide layout
// (DevTable::wrows): wam / wrm / wzm carry memory in f64 bytes and am / rm / zm are unused.
struct HostRow {
    int32_t ac, am, rc, rm, zc, zm, np, mp;
    double yc, ym;
    int32_t ae0, re0, ae1, re1;
    uint64_t th, ts, lb0, lb1;
    int32_t zone, pad;
    double wam, wrm, wzm;
};

// Lookahead geometry: window K pods, list length L (= K), G node chunks of `chunk` nodes per pod,
// E nodes per lane in the select kernel (256-thread blocks); G > 1 adds the k_la_merge pass.
// epl = list entries per resolver lane (power of two); a pod's lists occupy 64*epl entries.
// waves = resolver geometry: 1 (single-wave) or 4 (pipelined four-wave resolver).
// k32 = keys fit 32 bits ((max total + 1) < 2^10, n <= 2^22): one 32-bit wave reduction per pod.
// Sharding: the node table splits into W contiguous shards (shard v = nodes [v*n/W, (v+1)*n/W));
// every shard has the same G/E/chunk and eplr = 2^lr entries per lane per pod; this process
// selects shards [v0, v0 + nv) (nv = W for virtual shards in one process, 1 per rank with RCCL).
// epl (total entries per resolver lane, power of two) >= W * eplr.
struct LaGeom {
    uint32_t K, L, G, E, chunk, epl, waves, k32;
    uint32_t W, v0, nv, eplr, lr;
    uint32_t e2 = 1;  // resident stream: chunk keys per merging thread (G * L <= 512 * e2)
};
// Kernel-side shard view of the lists: [W][K][GLp] uint64 keys, RS = K * GLp.
struct LaShard {
    uint32_t W, v0, kw, pad;
    uint64_t RS;
};

hipError_t launch_persistent(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P,
                             const DevCfg &c, int32_t *out_node, uint64_t *out_key,
                             uint64_t *stamps, hipStream_t stream);
uint32_t persistent_max_nodes(uint32_t feat);

hipError_t launch_scan_pod(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s,
                           const DevCfg &c, void *scratch, int32_t *out_node, uint64_t *out_key,
                           uint64_t *stamps, uint8_t *feas, int32_t *score, int32_t *total,
                           int part, hipStream_t stream);  // part: 1 keys (+norm), 2 commit
hipError_t launch_rows_to_soa(const DevTable &t, hipStream_t stream);
// qs_score_pod in ONE launch (two for NormalizeScore profiles): pod record (DPod / DPodW) and
// extension by value; outputs written into pinned host memory hout (score_pod1_pack_bytes(n) bytes:
// [best u64 | done u64 | packed u32 x n]: four byte scores per node, kScoreInfeasible = infeasible),
// done = seq stored last; pidx < n: the pending row prow is written to the table first (and scored
// as such).  gs: four zeroed device u64 (the multi-workgroup form's best key, arrival count and
// normalize maxima; left zeroed); gs == nullptr: the single-workgroup form, n <= score_pod1_max_nodes().
uint32_t score_pod1_max_nodes();
constexpr uint32_t kScoreInfeasible = 0xFFFFFFFFu;  // packed per-node word of an infeasible node
size_t score_pod1_pack_bytes(uint32_t n);
hipError_t launch_score_pod1(const DevTable &t, const void *pod, const DPodX *podx, const DevCfg &c, uint8_t *hout,
                             uint64_t *gs, uint64_t seq, uint32_t pidx, const HostRow &prow, hipStream_t stream);
size_t scan_scratch_bytes();
// The head of the SCAN engine's device scratch (ScanScratch, qs_kernels.hpp): the reduced key, the
// normalize maxima and the node range of the row scans (the per-pod all-reduce engine's shard).
struct ScanHead {
    unsigned long long best;
    uint32_t mt, ma, lo, hi;
};

// L = list length per pod and shard (>= K; 2K for overlapped windows).
LaGeom la_geometry(uint32_t n, uint32_t K, uint32_t W = 1, uint32_t L = 0);
// Device buffers of one lookahead window.  lists: final [W][K][64*eplr] keys the resolver reads;
// clists: chunk-list scratch of nv*K*G*L keys (select -> merge; unused when G == 1); npart / norm:
// normalizing profiles' [W][K][G] partial maxima and per-pod NormInfo; dprev/dcur (overlapped
// windows): {count, nodes[64]} dirtied by the previous window (read) and by this window
// (written), nullptr = windows back to back; nfall: count of exact-rescan pods (normalizing).
struct NormInfo;
struct LaBufs {
    uint64_t *lists, *clists;
    uint4 *npart;
    NormInfo *norm;
    const uint32_t *dprev;
    uint32_t *dcur;
    unsigned long long *nfall;
    // batched mode: the batch's stream positions and size on the device (nullptr: s0 + k, kw)
    const uint32_t *pidx = nullptr, *pcount = nullptr;
    // normalizing profiles, four-wave resolver: the stop record it hands to the resume kernel
    uint32_t *rec = nullptr;
    // batched mode: per pod chunk-arrival tickets (zeroed at the stream's start); with them the
    // select launch merges each pod's chunk lists itself (no k_la_merge launch)
    uint32_t *tickets = nullptr;
};
// In-kernel window hand-off (DevCfg::ready): publish a window's lists (value = run << 32 | w + 1).
hipError_t launch_ready_set(uint64_t *ready, uint64_t value, hipStream_t stream);

// Resident lookahead stream: the whole overlapped window sequence of an
// unsharded Fit + Balanced (+ extended) stream as ONE launch of 1 resolver + sel_blocks selector
// workgroups; ctl = la_stream_res_ctl_bytes() of device memory, zeroed before every launch, and
// c.werr the timeout word.  lists0 / clists0 / dio: the double-buffered window buffers of the
// per-window path (lwords / cwords per parity).
// G = 0: unsupported.  Sharded contexts (geo.W > 1, Fit + Balanced (+ ext) only) plan their own
// node range of ceil(n / W) nodes.
LaGeom la_stream_res_plan(const LaGeom &geo, uint32_t feat, uint32_t n, uint32_t cus, uint32_t per_cu = 1);
size_t la_stream_res_ctl_bytes();
// Workgroups of that launch guaranteed co-resident on `cus` CUs (occupancy query, one per CU of margin).
uint32_t la_stream_res_max_blocks(const LaGeom &geo, uint32_t feat, uint32_t n, uint32_t cus);
// Resident sharded stream: rank `rank` of W selects its node range and exchanges
// every pod's shard list (and, normalizing profiles, its partial maxima) through the peer-memory mailboxes (peers[r] = rank r's mailbox base as
// mapped here; hello / flags / lists = byte offsets of the resident regions in every mailbox);
// seq tags this run's flags.  W = 1: unsharded (peers unused).
// Normalizing profiles also exchange each pod's partial maxima {mt, ct, ma, ca} over the rank's node
// range in the launch: nflags / norm = offsets of [4 slots][32 pods][16 ranks] u64 flags and uint4
// partials.
struct ResShard {
    uint32_t W, rank;
    uint64_t seq;
    char *const *peers;
    uint64_t hello, flags, lists;
    uint64_t nflags, norm;
};
// Normalizing profiles (TaintToleration / NodeAffinity) also pass the pod extension records (podx),
// npart (2 x K x G uint4 partial maxima), norm (2 x 64 NormInfo), stat (2 x K x 128 u32 entry
// statics, res_stream_stat_words) and nfall ({rescans, windows with a rescan}); they need K <= 32
// and sel_blocks >= K * G.
hipError_t launch_la_stream_res(const DevTable &t, const void *pods, const DPodX *podx, const DevCfg &c, uint32_t P,
                                const LaGeom &geo, uint64_t *lists0, uint64_t *clists0, uint32_t lwords,
                                uint32_t cwords, uint4 *npart, NormInfo *norm, uint32_t *stat, unsigned long long *nfall, int32_t *on,
                                uint64_t *ok, uint64_t *st, void *ctl, uint32_t sel_blocks, uint64_t *rdiag,
                                const ResShard &rsh, hipStream_t stream);

hipError_t launch_la_window(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s0,
                            uint32_t P, const DevCfg &c, const LaGeom &geo, const LaBufs &bufs,
                            int32_t *out_node, uint64_t *out_key, uint64_t *stamps, uint64_t *diag,
                            hipStream_t stream, int part);  // part: 4 norm, 1 select(+merge), 2 resolve

// Batched mode (spec S11): ctrl = {pods in the current batch, stream cursor}, bidx = the batch's
// stream positions.  init sets up the first batch; claim resolves one batch, applies its claims
// and builds the next.
hipError_t launch_batch_init(uint32_t *ctrl, uint32_t *bidx, uint32_t P, uint32_t B, hipStream_t stream);
size_t batch_claim_lds(uint32_t n);
hipError_t batch_claim_prepare();  // dynamic LDS of the claim kernel (<= 160 KB)
hipError_t launch_batch_claim(const DevTable &t, const void *pods, const uint64_t *lists, uint32_t *ctrl,
                              uint32_t *bidx, uint32_t P, uint32_t B, int32_t *out_node,
                              uint64_t *out_key, hipStream_t stream);

__global__ void k_set_row(DevTable t, uint32_t i, HostRow v, uint32_t feat);

}  // namespace qs
