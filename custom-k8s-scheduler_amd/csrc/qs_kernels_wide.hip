// qs_kernels_wide.hip — the wide-layout translation unit: instantiations of the
// kernels of qs_kernels.hpp for tables whose memory quantities need f64 byte columns (odd-Ki
// allocatable, decimal requests — anything the compact 2^u-byte int32 layout cannot hold below
// 2^24).  Two feature classes: Fit + Balanced (+ extended resources), and the normalizing profile
// (TaintToleration / NodeAffinity); extended-resource columns are always on (a zero request skips
// them, spec S4).  Every engine, the resident stream included.
#include "qs_kernels.hpp"

namespace qs {

namespace {
constexpr uint32_t kWideFit = kFeatWide | kFeatExt;
constexpr uint32_t kWideNorm = kFeatWide | kFeatExt | kFeatTaint | kFeatAffinity;
}  // namespace

hipError_t wide_persistent(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P,
                           const DevCfg &c, int32_t *on, uint64_t *ok, uint64_t *st, hipStream_t stream) {
    if (c.feat & kFeatNorm) return persistent_f<kWideNorm>(t, pods, podx, P, c, on, ok, st, stream);
    return persistent_f<kWideFit>(t, pods, podx, P, c, on, ok, st, stream);
}

uint32_t wide_persistent_max_nodes(uint32_t feat) {
    return (feat & kFeatNorm) ? persistent_cap<kWideNorm>() : persistent_cap<kWideFit>();
}

hipError_t wide_scan_pod(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s,
                         const DevCfg &c, void *scratch, int32_t *on, uint64_t *ok, uint64_t *st,
                         uint8_t *feas, int32_t *score, int32_t *total, int part, hipStream_t stream) {
    if (c.feat & kFeatNorm)
        return scan_pod_f<kWideNorm>(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
    return scan_pod_f<kWideFit>(t, pods, podx, s, c, scratch, on, ok, st, feas, score, total, part, stream);
}

hipError_t wide_la_window(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s0,
                          uint32_t P, const DevCfg &c, const LaGeom &geo, const LaBufs &bf,
                          int32_t *on, uint64_t *ok, uint64_t *st, uint64_t *diag,
                          hipStream_t stream, int part) {
    if (c.feat & kFeatNorm)
        return la_window_f<kWideNorm>(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
    return la_window_f<kWideFit>(t, pods, podx, s0, P, c, geo, bf, on, ok, st, diag, stream, part);
}

hipError_t wide_batch_claim_prepare() { return batch_claim_prepare_f<kWideFit>(); }

hipError_t wide_score_pod1(const DevTable &t, const void *pod, const DPodX *podx, const DevCfg &c, uint8_t *hout,
                           uint64_t *gs, uint64_t seq, uint32_t pidx, const HostRow &prow, hipStream_t stream) {
    if (c.feat & kFeatNorm) return score_pod1_f<kWideNorm>(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
    return score_pod1_f<kWideFit>(t, pod, podx, c, hout, gs, seq, pidx, prow, stream);
}

hipError_t wide_batch_claim(const DevTable &t, const void *pods, const uint64_t *lists, uint32_t *ctrl,
                            uint32_t *bidx, uint32_t P, uint32_t B, int32_t *on, uint64_t *ok,
                            size_t lds, hipStream_t stream) {
    return batch_claim_f<kWideFit>(t, pods, lists, ctrl, bidx, P, B, on, ok, lds, stream);
}

hipError_t wide_la_stream_res(const DevTable &t, const void *pods, const DPodX *podx, const DevCfg &c, uint32_t P,
                              const LaGeom &geo, uint64_t *lists0, uint64_t *clists0, uint32_t lwords, uint32_t cwords,
                              uint4 *npart, NormInfo *norm, uint32_t *stat, unsigned long long *nfall, int32_t *on,
                              uint64_t *ok, uint64_t *st, void *ctl, uint32_t sel_blocks, uint64_t *rdiag,
                              const ResShard &rsh, hipStream_t stream) {
    if (c.feat & kFeatNorm)
        return la_stream_res_f<kWideNorm>(t, pods, podx, c, P, geo, lists0, clists0, lwords, cwords, npart, norm, stat,
                                          nfall, on, ok, st, ctl, sel_blocks, rdiag, rsh, stream);
    return la_stream_res_f<kWideFit>(t, pods, podx, c, P, geo, lists0, clists0, lwords, cwords, npart, norm, stat, nfall,
                                     on, ok, st, ctl, sel_blocks, rdiag, rsh, stream);
}

int wide_la_stream_res_per_cu(const LaGeom &geo, uint32_t feat, uint32_t n) {
    return (feat & kFeatNorm) ? la_stream_res_per_cu<kWideNorm>(geo, n) : la_stream_res_per_cu<kWideFit>(geo, n);
}

}  // namespace qs
