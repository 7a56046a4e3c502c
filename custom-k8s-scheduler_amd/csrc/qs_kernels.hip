// qs_kernels.hip — the compact-layout translation unit of the gfx950 kernels (qs_kernels.hpp,
// DESIGN.md §4): the non-template kernels, the instantiations for the compact row layout
// (F in {0, kFeatExt, kFeatExt|kFeatTaint|kFeatAffinity}) and the host-callable dispatchers of
// qs_launch.hpp, which route wide-layout tables (DevTable::wrows) to qs_kernels_wide.hip.
#include "qs_kernels.hpp"

namespace qs {

// Rebuild the SoA copy from the row table (after engines that update rows only).
__global__ __launch_bounds__(256) void k_rows_to_soa(DevTable t) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= t.n) return;
    const DRow r = t.rows[i];
    t.soa.c[kSAc][i] = r.ac; t.soa.c[kSAm][i] = r.am; t.soa.c[kSRc][i] = r.rc; t.soa.c[kSRm][i] = r.rm;
    t.soa.c[kSZc][i] = r.zc; t.soa.c[kSZm][i] = r.zm; t.soa.c[kSNp][i] = r.np; t.soa.c[kSMp][i] = r.mp;
    t.soa.c[kSAe0][i] = r.ae0; t.soa.c[kSRe0][i] = r.re0; t.soa.c[kSAe1][i] = r.ae1; t.soa.c[kSRe1][i] = r.re1;
}

__global__ void k_batch_init(uint32_t *ctrl, uint32_t *bidx, uint32_t P, uint32_t B) {
    const uint32_t nb = min(P, B);
    if (threadIdx.x < nb) bidx[threadIdx.x] = threadIdx.x;
    if (threadIdx.x == 0) { ctrl[0] = nb; ctrl[1] = nb; }
}

hipError_t launch_batch_init(uint32_t *ctrl, uint32_t *bidx, uint32_t P, uint32_t B, hipStream_t stream) {
    hipLaunchKernelGGL(k_batch_init, dim3(1), dim3(64), 0, stream, ctrl, bidx, P, B);
    return hipGetLastError();
}

hipError_t batch_claim_prepare() {
    QS_RET(batch_claim_prepare_f<kFeatExt>());
    return wide_batch_claim_prepare();
}

size_t batch_claim_lds(uint32_t n) {
    return batch_claim_lds_bytes(n);
}

hipError_t launch_batch_claim(const DevTable &t, const void *pods, const uint64_t *lists, uint32_t *ctrl,
                              uint32_t *bidx, uint32_t P, uint32_t B, int32_t *on, uint64_t *ok,
                              hipStream_t stream) {
    const size_t lds = batch_claim_lds(t.n);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (t.wrows) return wide_batch_claim(t, pods, lists, ctrl, bidx, P, B, on, ok, lds, stream);
    return batch_claim_f<kFeatExt>(t, pods, lists, ctrl, bidx, P, B, on, ok, lds, stream);
}

// =============================================================================================
// small row kernels (qs_node_upsert / qs_reserve / qs_unreserve)
// =============================================================================================
__global__ void k_set_row(DevTable t, uint32_t i, HostRow v, uint32_t feat) {
    (void)feat;
    set_row(t, i, v);
}

// =============================================================================================
// dispatchers (qs_launch.hpp)
// =============================================================================================
static uint32_t feat_class(uint32_t feat) {
    return feat == 0 ? 0u : (feat == kFeatExt ? kFeatExt : (kFeatExt | kFeatTaint | kFeatAffinity));
}

hipError_t launch_persistent(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P,
                             const DevCfg &c, int32_t *on, uint64_t *ok, uint64_t *st,
                             hipStream_t stream) {
    if (c.feat & kFeatRes)
        return t.wrows ? res_wide_persistent(t, pods, podx, P, c, on, ok, st, stream)
                       : res_compact_persistent(t, pods, podx, P, c, on, ok, st, stream);
    if (t.wrows) return wide_persistent(t, pods, podx, P, c, on, ok, st, stream);
    switch (feat_class(c.feat)) {
        case 0: return persistent_f<0>(t, pods, podx, P, c, on, ok, st, stream);
        case kFeatExt: return persistent_f<kFeatExt>(t, pods, podx, P, c, on, ok, st, stream);
        default:
            return persistent_f<kFeatExt | kFeatTaint | kFeatAffinity>(t, pods, podx, P, c, on, ok,
                                                                         st, stream);
    }
}

uint32_t persistent_max_nodes(uint32_t feat) {
    if (feat & kFeatRes)
        return (feat & kFeatWide) ? res_wide_persistent_max_nodes(feat) : res_compact_persistent_max_nodes(feat);
    if (feat & kFeatWide) return wide_persistent_max_nodes(feat);
    switch (feat_class(feat)) {
        case 0: return persistent_cap<0>();
        case kFeatExt: return persistent_cap<kFeatExt>();
        default: return persistent_cap<kFeatExt | kFeatTaint | kFeatAffinity>();
    }
}

hipError_t launch_rows_to_soa(const DevTable &t, hipStream_t stream) {
    if (!t.soa.c[0] || t.n == 0 || !t.rows) return hipSuccess;
    hipLaunchKernelGGL(k_rows_to_soa, dim3((t.n + 255) / 256), dim3(256), 0, stream, t);
    return hipGetLastError();
}

hipError_t launch_scan_pod(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s,
                           const DevCfg &c, void *scratch, int32_t *on, uint64_t *ok, uint64_t *st,
                           uint8_t *feas, int32_t *score, int32_t *total, int part,
                           hipStream_t stream) {
    if (c.feat & kFeatRes)
        return t.wrows ? res_wide_scan_pod(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream)
                       : res_compact_scan_pod(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
    if (t.wrows) return wide_scan_pod(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
    switch (feat_class(c.feat)) {
        case 0: return scan_pod_f<0>(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
        case kFeatExt: return scan_pod_f<kFeatExt>(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
        default:
            return scan_pod_f<kFeatExt | kFeatTaint | kFeatAffinity>(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
    }
}

size_t scan_scratch_bytes() { return sizeof(ScanScratch); }

uint32_t score_pod1_max_nodes() { return kScorePod1Max; }
size_t score_pod1_pack_bytes(uint32_t n) { return score_pack_bytes(n); }
hipError_t launch_score_pod1(const DevTable &t, const void *pod, const DPodX *podx, const DevCfg &c, uint8_t *hout,
                             uint64_t *gs, uint64_t seq, uint32_t pidx, const HostRow &prow, hipStream_t stream) {
    if (c.feat & kFeatRes)
        return t.wrows ? res_wide_score_pod1(t, pod, podx, c, hout, gs, seq, pidx, prow, stream)
                       : res_compact_score_pod1(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
    if (t.wrows) return wide_score_pod1(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
    switch (feat_class(c.feat)) {
        case 0: return score_pod1_f<0>(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
        case kFeatExt: return score_pod1_f<kFeatExt>(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
        default:
            return score_pod1_f<kFeatExt | kFeatTaint | kFeatAffinity>(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
    }
}

// Window hand-off: publishes window w's lists (ready = run << 32 | w + 1) once the
// select chain's kernels before it on the stream have finished; the release store orders them.
// (A stream memory write, hipStreamWriteValue64, measured slower: 92.5 vs 87.7 ms per stream.)
__global__ void k_ready_set(uint64_t *ready, uint64_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(ready, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
hipError_t launch_ready_set(uint64_t *ready, uint64_t value, hipStream_t stream) {
    hipLaunchKernelGGL(k_ready_set, dim3(1), dim3(64), 0, stream, ready, value);
    return hipGetLastError();
}

hipError_t launch_la_window(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s0,
                            uint32_t P, const DevCfg &c, const LaGeom &geo, const LaBufs &bf,
                            int32_t *on, uint64_t *ok, uint64_t *st, uint64_t *diag,
                            hipStream_t stream, int part) {
    if (bf.dprev && geo.waves == 1 && !(c.feat & kFeatNorm)) return hipErrorInvalidValue;
    if ((c.feat & kFeatNorm) && diag && geo.waves != 4) return hipErrorInvalidValue;
    if (c.feat & kFeatRes)
        return t.wrows ? res_wide_la_window(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part)
                       : res_compact_la_window(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
    if (t.wrows) return wide_la_window(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
    if (c.feat & kFeatNorm)
        return la_window_f<kFeatExt | kFeatTaint | kFeatAffinity>(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
    if (c.feat & kFeatExt) return la_window_f<kFeatExt>(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
    return la_window_f<0>(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
}

// Resident-stream geometry: every (pod, chunk) task of a window gets its own selector workgroup
// (K * G <= per_cu * cus - 1), chunks of E * 512 nodes with E from the instantiated set, G <= 8
// (a merge reads <= 512 keys, one per thread) or, with two workgroups per CU, G <= 16 (Fit +
// Balanced (+ext): e2 = 2 keys per merging thread); G = 0 when the table is too large or the
// profile / layout is not covered.  per_cu = 2 is tried first and kept when the occupancy check
// admits it (more, shorter selector tasks: the config-3 stream was selector-bound).
LaGeom la_stream_res_plan(const LaGeom &geo, uint32_t feat, uint32_t n, uint32_t cus, uint32_t per_cu) {
    LaGeom r = geo;
    r.G = 0;
    // Fit + Balanced (+ extended) profiles, and the normalizing ones (K <= kResNormK), both layouts;
    // sharded (geo.W > 1 ranks, one shard each): W * L <= 512
    const uint32_t fl = feat & ~(kFeatWide | kFeatRes);  // both row layouts, either scoring form
    const bool fit = fl == 0 || fl == kFeatExt;
    const bool norm = (feat & kFeatNorm) != 0 && geo.K <= kResNormK;
    const bool shard_ok = geo.W == 1 ? geo.nv == 1 && geo.epl == 1
                                     : geo.nv == 1 && geo.K <= 32 && geo.W * geo.L <= (uint32_t)kResBS;
    if (!((fit || norm) && shard_ok && geo.waves == 4 && geo.L <= 64 && n > 0 && cus > geo.K)) return r;
    n = (n + geo.W - 1) / geo.W;  // this rank's node range
    const bool two = per_cu >= 2 && fit;
    const uint32_t gmax = std::min(two ? 16u : 8u, ((two ? 2u : 1u) * cus - 1) / geo.K);
    if (gmax == 0) return r;
    constexpr uint32_t bs = kResBS;  // threads of a selector workgroup
    // chunks of up to 5 * 512 nodes, or, where one selector per CU still covers every task, of
    // 3 * 512: shorter tasks put a window's last list out earlier (config 2: 13.3 -> 12.2 us after
    // the previous window's start, so the resolver's prefetch check at its pod K-3 stops missing
    // it, and the boundary p99 drops 1.52 -> 1.20 us); QS_RES_G: at least that many (experiments)
    static const uint32_t gwant = getenv("QS_RES_G") ? (uint32_t)std::max(0, atoi(getenv("QS_RES_G"))) : 0u;
    const uint32_t gsmall = std::min((cus - 1) / geo.K, (n + 3 * bs - 1) / (3 * bs));
    const uint32_t G0 = std::min(gmax, std::max({gwant, gsmall, (n + 5 * bs - 1) / (5 * bs)}));
    const uint32_t e_need = ((n + G0 - 1) / G0 + bs - 1) / bs;
    uint32_t E = 0;
    for (uint32_t e : {3u, 5u, 7u, 8u, 16u})  // (7: config 3's 50,000 nodes in 14 chunks, 448 tasks: -5 % against 13 of 4,096)
        if (e >= e_need) { E = e; break; }
    if (E == 0) return r;  // more than 8 chunks of 8,192 nodes: per-window launches
    const uint32_t G = (n + E * bs - 1) / (E * bs);
    const uint32_t e2 = G * geo.L <= bs ? 1u : 2u;
    if (G * geo.L > e2 * bs || (e2 == 2 && (!two || E == 3))) return r;
    r.e2 = e2;
    r.E = E;
    r.chunk = E * bs;
    r.G = G;
    return r;
}
size_t la_stream_res_ctl_bytes() { return kResCtlBytes; }

// Co-residency bound of the resident stream: its selectors spin on the resolver and the resolver on
// them, so every workgroup of the launch must be resident at once.  The occupancy API's answer per
// CU can exceed what the hardware admits by one workgroup (MI355X_MICROARCH.md, residency), so one
// is taken off whenever the API allows two or more.
uint32_t la_stream_res_max_blocks(const LaGeom &geo, uint32_t feat, uint32_t n, uint32_t cus) {
    const int per = (feat & kFeatRes)   ? ((feat & kFeatWide) ? res_wide_la_stream_res_per_cu(geo, feat, n)
                                                              : res_compact_la_stream_res_per_cu(geo, feat, n))
                    : (feat & kFeatWide)  ? wide_la_stream_res_per_cu(geo, feat, n)
                    : (feat & kFeatNorm)  ? la_stream_res_per_cu<kFeatExt | kFeatTaint | kFeatAffinity>(geo, n)
                    : (feat & kFeatExt) ? la_stream_res_per_cu<kFeatExt>(geo, n)
                                        : la_stream_res_per_cu<0>(geo, n);
    // The API's answer can exceed what the hardware admits by one workgroup when the SGPR budget
    // (800 per SIMD, (ceil(sgpr / 16) * 16 + 16) per wave) binds first (MI355X_MICROARCH.md,
    // residency): cap it by that rule, with kResSgprMax >= every instantiation's sgpr_count
    // (tools/kres.sh: 104-106), two waves per SIMD for a 512-thread workgroup.
    const int sgpr_waves = 800 / (((int)kResSgprMax + 15) / 16 * 16 + 16);
    const int safe = std::min(per, sgpr_waves / (kResBS / 64 / 4));
    return (uint32_t)std::max(0, safe) * cus;
}

hipError_t launch_la_stream_res(const DevTable &t, const void *pods, const DPodX *podx, const DevCfg &c, uint32_t P,
                                const LaGeom &geo, uint64_t *lists0, uint64_t *clists0, uint32_t lwords,
                                uint32_t cwords, uint4 *npart, NormInfo *norm, uint32_t *stat, unsigned long long *nfall,
                                int32_t *on, uint64_t *ok, uint64_t *st, void *ctl, uint32_t sel_blocks, uint64_t *rdiag,
                                const ResShard &rsh, hipStream_t stream) {
    if (geo.G == 0 || (uint64_t)t.n * (t.wrows ? sizeof(DRowW) : sizeof(DRow)) >= (1ull << 31))
        return hipErrorInvalidValue;
    if (c.feat & kFeatRes)
        return (t.wrows ? res_wide_la_stream_res : res_compact_la_stream_res)(
            t, pods, podx, c, P, geo, lists0, clists0, lwords, cwords, npart, norm, stat, nfall, on, ok, st, ctl,
            sel_blocks, rdiag, rsh, stream);
    if (t.wrows)
        return wide_la_stream_res(t, pods, podx, c, P, geo, lists0, clists0, lwords, cwords, npart, norm, stat, nfall, on,
                                  ok, st, ctl, sel_blocks, rdiag, rsh, stream);
    if (c.feat & kFeatNorm)
        return la_stream_res_f<kFeatExt | kFeatTaint | kFeatAffinity>(t, pods, podx, c, P, geo, lists0, clists0, lwords,
                                                                      cwords, npart, norm, stat, nfall, on, ok, st, ctl,
                                                                      sel_blocks, rdiag, rsh, stream);
    if (c.feat & kFeatExt)
        return la_stream_res_f<kFeatExt>(t, pods, podx, c, P, geo, lists0, clists0, lwords, cwords, npart, norm, stat,
                                         nfall, on, ok, st, ctl, sel_blocks, rdiag, rsh, stream);
    return la_stream_res_f<0>(t, pods, podx, c, P, geo, lists0, clists0, lwords, cwords, npart, norm, stat, nfall, on,
                              ok, st, ctl, sel_blocks, rdiag, rsh, stream);
}

LaGeom la_geometry(uint32_t n, uint32_t K, uint32_t W, uint32_t L) {
    // Per shard (W shards of <= ceil(n/W) nodes; W = 1 unsharded): G node chunks of `chunk` nodes
    // per pod (E nodes per lane of a 256-thread select block; about 1,280 nodes by default, env
    // QS_LA_E overrides E), each keeping its top-L; k_la_merge reduces the G*L <= 2,048 keys to one
    // top-L per pod and shard, so a shard contributes L <= 64 keys (one 64-entry block, eplr = 1)
    // and the resolver reads epl = pow2 >= W entries per lane.
    static const uint32_t Es[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16};
    static const char *env_e = getenv("QS_LA_E");
    const uint32_t e_target = env_e ? (uint32_t)std::max(1, atoi(env_e)) : 5u;
    LaGeom g{};
    g.K = K;
    g.L = std::max(K, L);
    g.W = std::max(1u, W);
    g.v0 = 0;
    g.nv = g.W;
    if (g.W > 16 || g.L > 64) return g;  // G = 0: no geometry
    const uint32_t ns = (n + g.W - 1) / g.W;
    const uint32_t gmax = 2048u / g.L;
    const uint32_t target = e_target * 256u;
    uint32_t G = std::max(1u, std::min(gmax, (ns + target - 1) / target));
    const uint32_t per = (ns + G - 1) / G;
    const uint32_t e_need = std::max(1u, (per + 255) / 256);
    uint32_t E = 0;
    for (uint32_t e : Es)
        if (e >= e_need) { E = e; break; }
    if (E == 0) return g;  // shard too large for one level of chunk lists
    g.E = E;
    g.chunk = E * 256;
    G = std::max(1u, (ns + g.chunk - 1) / g.chunk);
    g.eplr = 1;
    g.lr = 0;
    g.epl = 1;
    while (g.epl < g.W) g.epl *= 2;
    g.G = G;
    return g;
}

}  // namespace qs
