// qs_kernels.hpp — gfx950 kernels of the exact per-pod scheduling cycle (spec/semantics.md S4–S7)
// and their templated launchers.  Every kernel is a template over the feature set F; the compact
// layout's instantiations live in qs_kernels.hip, the wide layout's (F & kFeatWide: f64 memory
// columns) in qs_kernels_wide.hip, so no kernel symbol exists in two code objects.
//
// Engines (all bit-exact with the oracle):
//   PERSISTENT  k_persistent: ONE resident workgroup runs the whole pod stream; node rows live in
//               VGPRs (NPT rows per lane), Filter+Score in registers, DPP wave argmax, one LDS
//               exchange + one barrier per pod, Reserve applied by the owning lane.  N <= 8192.
//   SCAN        k_scan_norm / k_scan_key / k_scan_commit: per-pod grid scan over the HBM table with
//               u64 atomicMax of packed keys, then a 1-thread commit that applies Reserve.  Any N.
//   LOOKAHEAD   k_la_select + k_la_resolve: exact top-K lookahead.  For a window of K pods the
//               whole chip scores all K×N (pod, node) pairs against the window-start table and
//               keeps, per pod and node-chunk, the top-L keys (L = K).  One wave then resolves the
//               window sequentially: pod i's winner is the max of (fresh keys of the <= i nodes
//               modified earlier in the window) and (the best stale key of an unmodified node,
//               which is always inside the top-L lists).  Bit-exact; SURVEY.md §7 H4 option 3.
#pragma once
#include <algorithm>
#include <cstring>

#include "qs_device.hpp"
#include "qs_launch.hpp"

// Timing-ablation hooks (tools/exp_run.sh): empty in the product build.  Only
// `make exp` defines them, by force-including csrc/exp/qs_exp.hpp, whose variants give wrong
// placements by construction (timing experiments, never the product library).
#ifndef QS_EXP_HOOKS
#define QS_EXP_NORM_AB(norm) (norm)
#define QS_EXP_SLOT_KEY(act, r, q)
#define QS_EXP_CAND_KEY(f, tot, cr, p)
#define QS_EXP_PARK_RETURN()
#endif

namespace qs {

constexpr uint32_t kFeatNorm = kFeatTaint | kFeatAffinity;

// =============================================================================================
// PERSISTENT engine
// =============================================================================================
template <int NPT, int BS, uint32_t F>
__global__ __launch_bounds__(BS) void k_persistent(DevTable t, const PodT<F> *__restrict__ pods,
                                                   const DPodX *__restrict__ podx, uint32_t P,
                                                   DevCfg c, int32_t *__restrict__ out_node,
                                                   uint64_t *__restrict__ out_key,
                                                   uint64_t *__restrict__ stamps) {
    constexpr int NW = BS / kWave;
    __shared__ uint64_t red[2][NW];
    __shared__ uint32_t redn[2][2][NW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t n = t.n;
    RowT<F> r[NPT];
    RowX x[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const uint32_t idx = tid + k * BS;
        if (idx < n) { r[k] = load_row<F>(t, idx); x[k] = load_rowx<F>(t, idx); }
        else { r[k] = empty_row<F>(); x[k] = RowX{0, 0, 0, 0, 0, 0, 0, 0}; }
    }
    PodT<F> pn = pods[0];
    for (uint32_t s = 0; s < P; ++s) {
        const PodT<F> p = pn;
        pn = pods[s + 1 < P ? s + 1 : s];  // prefetch the next pod record (scalar loads)
        DPodX px;
        if (F & kFeatNorm) px = podx[s];
        uint32_t mt = 0, ma = 0;
        double ymt = 0.0, yma = 0.0;
        if (F & kFeatNorm) {  // NormalizeScore maxima over feasible nodes (spec S5)
            uint32_t lt = 0, la = 0;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const bool f = feasible<F>(r[k], x[k], p, px);
                const uint32_t a = f ? taint_raw(x[k], px) : 0u;
                const uint32_t b = f ? affinity_raw(x[k], p, px) : 0u;
                lt = a > lt ? a : lt;
                la = b > la ? b : la;
            }
            lt = wave_max_u32(lt);
            la = wave_max_u32(la);
            if (lane == 0) { redn[s & 1][0][w] = lt; redn[s & 1][1][w] = la; }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const uint32_t a = redn[s & 1][0][i], b = redn[s & 1][1][i];
                mt = a > mt ? a : mt;
                ma = b > ma ? b : ma;
            }
            ymt = rcp_exact(mt);
            yma = rcp_exact(ma);
        }
        uint64_t best = 0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const bool f = feasible<F>(r[k], x[k], p, px);
            const uint32_t tot = node_total<F>(r[k], x[k], p, px, c, mt, ymt, ma, yma, nullptr);
            const uint64_t key = f ? pack_key(tot + 1, tid + k * BS) : 0ull;
            best = key > best ? key : best;
        }
        best = wave_max_u64(best);
        if (lane == 0) red[s & 1][w] = best;
        __syncthreads();
        uint64_t ks = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const uint64_t v = red[s & 1][i];
            ks = v > ks ? v : ks;
        }
        const uint32_t win = key_node(ks);
        if (ks != 0) {
#pragma unroll
            for (int k = 0; k < NPT; ++k)
                if (tid + k * BS == win) reserve(r[k], x[k], p, +1);
        }
        if (tid == 0) {
            out_node[s] = ks ? (int32_t)win : -1;
            if (out_key) out_key[s] = ks;
            if (stamps) stamps[s] = __builtin_amdgcn_s_memrealtime();
        }
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const uint32_t idx = tid + k * BS;
        if (idx < n) { store_dyn<F>(t, idx, r[k]); store_dynx<F>(t, idx, x[k]); }
    }
}

// =============================================================================================
// SCAN engine (and qs_score_pod)
// =============================================================================================
// Per-pod scratch: normalize maxima (taint / affinity) and one partial argmax key per block of the
// key scan; the commit kernel reduces the partials (no single-address atomics on the hot path:
// thousands of blocks hitting one u64 serialise at the memory-side atomic unit).
constexpr uint32_t kScanBlocksMax = 2048;
struct ScanScratch {
    unsigned long long best;  // reduced key of the last commit (qs_score_pod reads it)
    uint32_t mt, ma;          // normalize maxima (k_scan_norm)
    uint32_t lo, hi;          // node range the row scans cover (hi == 0: the whole table); a rank's
                              // shard for the per-pod all-reduce engine (QS_ENGINE_ALLREDUCE)
    uint64_t partial[kScanBlocksMax];
};
static_assert(offsetof(ScanScratch, lo) == offsetof(ScanHead, lo) && offsetof(ScanScratch, mt) == offsetof(ScanHead, mt),
              "ScanHead mirrors ScanScratch");

// Block-wide max of a u64 key: wave DPP max, then one LDS exchange.
template <int BS>
__device__ __forceinline__ uint64_t block_max_u64(uint64_t v) {
    __shared__ uint64_t red[BS / kWave];
    v = wave_max_u64(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < BS / kWave; ++i) m = red[i] > m ? red[i] : m;
    return m;
}

template <uint32_t F>
__global__ __launch_bounds__(256) void k_scan_norm(DevTable t, const PodT<F> *__restrict__ pods,
                                                   const DPodX *__restrict__ podx, uint32_t s,
                                                   ScanScratch *sc) {
    const PodT<F> p = pods[s];
    const DPodX px = podx[s];
    uint32_t lt = 0, la = 0;
    const uint32_t lo = sc->lo, hi = sc->hi ? sc->hi : t.n;
    for (uint32_t i = lo + blockIdx.x * 256 + threadIdx.x; i < hi; i += gridDim.x * 256) {
        const RowT<F> r = load_row<F>(t, i);
        const RowX x = load_rowx<F>(t, i);
        if (feasible<F>(r, x, p, px)) {
            const uint32_t a = taint_raw(x, px), b = affinity_raw(x, p, px);
            lt = a > lt ? a : lt;
            la = b > la ? b : la;
        }
    }
    // (normalizing profiles run this scan on row tables of a few thousand nodes: few blocks)
    lt = wave_max_u32(lt);
    la = wave_max_u32(la);
    if ((threadIdx.x & 63) == 0) {
        if (lt) atomicMax(&sc->mt, lt);
        if (la) atomicMax(&sc->ma, la);
    }
}

// Keys for every node from the row table; optionally per-node outputs for qs_score_pod.
template <uint32_t F>
__global__ __launch_bounds__(256) void k_scan_key(DevTable t, const PodT<F> *__restrict__ pods,
                                                  const DPodX *__restrict__ podx, uint32_t s,
                                                  DevCfg c, ScanScratch *sc, uint8_t *feas_out,
                                                  int32_t *score_out, int32_t *total_out) {
    const PodT<F> p = pods[s];
    DPodX px;
    uint32_t mt = 0, ma = 0;
    if (F & kFeatNorm) { px = podx[s]; mt = sc->mt; ma = sc->ma; }
    const double ymt = rcp_exact(mt), yma = rcp_exact(ma);
    uint64_t best = 0;
    const uint32_t lo = sc->lo, hi = sc->hi ? sc->hi : t.n;
    for (uint32_t i = lo + blockIdx.x * 256 + threadIdx.x; i < hi; i += gridDim.x * 256) {
        const RowT<F> r = load_row<F>(t, i);
        const RowX x = load_rowx<F>(t, i);
        const bool f = feasible<F>(r, x, p, px);
        uint32_t sco[4];
        const uint32_t tot = node_total<F>(r, x, p, px, c, mt, ymt, ma, yma, score_out ? sco : nullptr);
        const uint64_t key = f ? pack_key(tot + 1, i) : 0ull;
        best = key > best ? key : best;
        if (feas_out) feas_out[i] = f;
        if (total_out) total_out[i] = f ? (int32_t)tot : -1;
        if (score_out) {
#pragma unroll
            for (int q = 0; q < 4; ++q) score_out[4 * (size_t)i + q] = f ? (int32_t)sco[q] : 0;
        }
    }
    best = block_max_u64<256>(best);
    if (threadIdx.x == 0) sc->partial[blockIdx.x] = best;
}

// One 16-byte quad of a SoA column, read non-temporally: every byte of the scan is read once per
// pod, and the streaming hint took k_scan_soa from 5.2 to 5.9-6.0 TB/s on the 2^24-node table
// (65 -> 74 % of the 8 TB/s peak, tools/scan_probe.py; four quads in flight per lane instead of two
// was slower, 4.7-5.5 TB/s with or without the hint).
__device__ __forceinline__ int4 soa_quad(const int32_t *col, uint32_t q) {
    return __builtin_bit_cast(int4, __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(col) + q));
}

// Keys over the SoA copy (HBM-resident tables; F = 0 or kFeatExt): lane q covers nodes
// 4q..4q+3 with one 16-byte load per column; RN(1/alloc) is recomputed in registers (rcp_int:
// the same value the host stores in the row copy, so keys are bit-identical to k_scan_key).
template <uint32_t F>
__global__ __launch_bounds__(256) void k_scan_soa(DevTable t, const PodT<F> *__restrict__ pods,
                                                  uint32_t s, DevCfg c, ScanScratch *sc,
                                                  uint8_t *feas_out, int32_t *score_out,
                                                  int32_t *total_out) {
    const PodT<F> p = pods[s];
    const DPodX px{};
    const uint32_t nq = (t.n + 3) / 4;  // columns are zero-padded to a multiple of 64 nodes
    uint64_t best = 0;
    // two quads per lane in flight: both iterations' loads are issued before either is scored
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t q0 = blockIdx.x * 256 + threadIdx.x; q0 < nq; q0 += 2 * stride) {
        int4 cols[2][kSCols];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t qh = min(q0 + h * stride, nq - 1);
#pragma unroll
            for (int k = 0; k < 8; ++k) cols[h][k] = soa_quad(t.soa.c[k], qh);
            if (F & kFeatExt) {
#pragma unroll
                for (int k = 8; k < kSCols; ++k) cols[h][k] = soa_quad(t.soa.c[k], qh);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
        const uint32_t q = q0 + h * stride;
        if (q >= nq) break;
        const int4 *col = cols[h];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            auto el = [&](int k) { return e == 0 ? col[k].x : e == 1 ? col[k].y : e == 2 ? col[k].z : col[k].w; };
            RowT<F> r;
            r.ac = el(kSAc); r.am = el(kSAm); r.rc = el(kSRc); r.rm = el(kSRm);
            r.zc = el(kSZc); r.zm = el(kSZm); r.np = el(kSNp); r.mp = el(kSMp);
            r.yc = r.ac ? rcp_int(r.ac) : 0.0;
            r.ym = r.am ? rcp_int(r.am) : 0.0;
            RowX x{};
            if (F & kFeatExt) { x.ae0 = el(kSAe0); x.re0 = el(kSRe0); x.ae1 = el(kSAe1); x.re1 = el(kSRe1); }
            const uint32_t idx = 4 * q + e;
            const bool f = feasible<F>(r, x, p, px);  // padding rows: max_pods 0 -> infeasible
            uint32_t sco[4];
            const uint32_t tot = node_total<F>(r, x, p, px, c, 0, 0.0, 0, 0.0, score_out ? sco : nullptr);
            const uint64_t key = f ? pack_key(tot + 1, idx) : 0ull;
            best = key > best ? key : best;
            if (idx < t.n) {
                if (feas_out) feas_out[idx] = f;
                if (total_out) total_out[idx] = f ? (int32_t)tot : -1;
                if (score_out) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) score_out[4 * (size_t)idx + k] = f ? (int32_t)sco[k] : 0;
                }
            }
        }
        }
    }
    best = block_max_u64<256>(best);
    if (threadIdx.x == 0) sc->partial[blockIdx.x] = best;
}

// One 256-thread block: reduce the key scan's partials to the pod's winner (nblk == 0: take sc->best,
// e.g. after the ranks' all-reduce of it), then (stream mode, out_node != nullptr) apply Reserve to
// the row (and SoA) copy and emit the outputs.  Resets the normalize maxima for the next pod.
template <uint32_t F>
__global__ __launch_bounds__(256) void k_scan_commit(DevTable t, const PodT<F> *__restrict__ pods,
                                                     uint32_t s, uint32_t nblk, ScanScratch *sc,
                                                     int32_t *out_node, uint64_t *out_key,
                                                     uint64_t *stamps) {
    uint64_t v = 0;
    for (uint32_t i = threadIdx.x; i < nblk; i += 256) v = sc->partial[i] > v ? sc->partial[i] : v;
    const uint64_t ks = nblk ? block_max_u64<256>(v) : sc->best;
    if (threadIdx.x != 0) return;
    if (nblk && !out_node) {
        // the all-reduce engine's shard reduction (part 32): max INTO best, so the shards of a
        // virtual world (one context scanning every node range in turn) combine as the all-reduce
        // does; the commit (part 64) consumes best and clears it for the next pod
        sc->best = ks > sc->best ? ks : sc->best;
        return;
    }
    sc->best = nblk ? ks : 0ull;
    sc->mt = 0;
    sc->ma = 0;
    if (!out_node) return;
    const PodT<F> p = pods[s];
    if (ks) {
        const uint32_t w = key_node(ks);
        RowT<F> r = load_row<F>(t, w);
        RowX x = load_rowx<F>(t, w);
        reserve(r, x, p, +1);
        store_dyn<F>(t, w, r);
        store_dynx<F>(t, w, x);
        if (t.soa.c[0]) {
            t.soa.c[kSRc][w] = r.rc; t.soa.c[kSRm][w] = r.rm;
            t.soa.c[kSZc][w] = r.zc; t.soa.c[kSZm][w] = r.zm;
            t.soa.c[kSNp][w] = r.np;
            if (F & kFeatExt) { t.soa.c[kSRe0][w] = x.re0; t.soa.c[kSRe1][w] = x.re1; }
        }
    }
    out_node[s] = ks ? (int32_t)key_node(ks) : -1;
    if (out_key) out_key[s] = ks;
    if (stamps) stamps[s] = __builtin_amdgcn_s_memrealtime();
}

// One node row written from the host mirror (qs_node_upsert / qs_reserve / qs_unreserve; k_set_row
// and the pending-row write of k_score_pod1): row (compact or wide), masks, zone, SoA copy.
__device__ __forceinline__ void set_row(const DevTable &t, uint32_t i, const HostRow &v) {
    t.masks[i] = DMask{v.th, v.ts, v.lb0, v.lb1};
    if (t.zone) t.zone[i] = v.zone;
    if (t.wrows) {  // wide layout: memory columns in f64 bytes
        DRowW w;
        w.ac = v.ac; w.rc = v.rc; w.zc = v.zc; w.np = v.np;
        w.am = v.wam; w.rm = v.wrm; w.zm = v.wzm; w.ym = v.ym;
        w.yc = v.yc; w.mp = v.mp; w.pad = 0;
        w.ae0 = v.ae0; w.re0 = v.re0; w.ae1 = v.ae1; w.re1 = v.re1;
        t.wrows[i] = w;
        return;
    }
    DRow r;
    r.ac = v.ac; r.am = v.am; r.rc = v.rc; r.rm = v.rm; r.zc = v.zc; r.zm = v.zm;
    r.np = v.np; r.mp = v.mp; r.yc = v.yc; r.ym = v.ym;
    r.ae0 = v.ae0; r.re0 = v.re0; r.ae1 = v.ae1; r.re1 = v.re1;
    t.rows[i] = r;
    if (t.soa.c[0]) {
        const int32_t f[kSCols] = {v.ac, v.am, v.rc, v.rm, v.zc, v.zm, v.np, v.mp, v.ae0, v.re0, v.ae1, v.re1};
#pragma unroll
        for (int k = 0; k < kSCols; ++k) t.soa.c[k][i] = f[k];
    }
}
// The same row as the kernels' register form.
template <uint32_t F>
__device__ __forceinline__ void host_row_regs(const HostRow &v, RowT<F> &r, RowX &x) {
    if constexpr ((F & kFeatWide) != 0) {
        r.ac = v.ac; r.rc = v.rc; r.zc = v.zc; r.np = v.np; r.mp = v.mp;
        r.am = v.wam; r.rm = v.wrm; r.zm = v.wzm; r.yc = v.yc; r.ym = v.ym;
    } else {
        r.ac = v.ac; r.am = v.am; r.rc = v.rc; r.rm = v.rm; r.zc = v.zc; r.zm = v.zm;
        r.np = v.np; r.mp = v.mp; r.yc = v.yc; r.ym = v.ym;
    }
    x.ae0 = x.re0 = x.ae1 = x.re1 = 0;
    x.th = x.ts = x.lb0 = x.lb1 = 0;
    if (F & kFeatExt) { x.ae0 = v.ae0; x.re0 = v.re0; x.ae1 = v.ae1; x.re1 = v.re1; }
    if (F & (kFeatTaint | kFeatAffinity)) { x.th = v.th; x.ts = v.ts; x.lb0 = v.lb0; x.lb1 = v.lb1; }
}

// qs_score_pod (the framework-embedded path, one call per pod): the pod record and
// its extension passed by value (no H2D), every output written straight into pinned host memory (no
// D2H command): [best key u64 | done u64 | packed u32 x n], packed = the four plugin scores (0..100)
// as bytes {LeastAllocated, Balanced, TaintToleration, NodeAffinity}, 0xFFFFFFFF = infeasible (the
// host derives the QoS-weighted total from them: 4 bytes per node cross the host link);
// `done` = seq, stored last with a system-scope release after every thread's system fence, is what
// the host polls.  A pending row (the previous qs_reserve / qs_unreserve, folded into this launch)
// is written to the table by thread 0 and used from the argument by the thread that scores it.
// k_score_pod1 (ONE 1024-thread workgroup, normalize maxima and keys in the same launch, two passes
// separated by a barrier) is the form without the device words, for tables up to kScorePod1Max.
constexpr uint32_t kScorePod1Max = 16384;
__host__ __device__ constexpr size_t score_pack_bytes(uint32_t n) { return 16 + 4 * (size_t)n; }
__device__ __forceinline__ uint32_t pack_scores(bool f, const uint32_t (&sco)[4]) {
    return f ? (sco[0] | (sco[1] << 8) | (sco[2] << 16) | (sco[3] << 24)) : kScoreInfeasible;
}
template <uint32_t F>
__global__ __launch_bounds__(1024) void k_score_pod1(DevTable t, PodT<F> p, DPodX px, DevCfg c, uint8_t *hout,
                                                     uint64_t seq, uint32_t pidx, HostRow prow) {
    constexpr int NW = 1024 / kWave;
    __shared__ uint32_t red[2][NW];
    __shared__ uint64_t redk[NW];
    const uint32_t n = t.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t *packed = reinterpret_cast<uint32_t *>(hout + 16);
    RowT<F> pr;
    RowX prx;
    host_row_regs<F>(prow, pr, prx);
    if (tid == 0 && pidx < n) set_row(t, pidx, prow);
    auto row_at = [&](uint32_t i, RowT<F> &r, RowX &x) {
        r = load_row<F>(t, i);
        x = load_rowx<F>(t, i);
        if (i == pidx) { r = pr; x = prx; }
    };
    uint32_t mt = 0, ma = 0;
    if constexpr ((F & kFeatNorm) != 0) {  // NormalizeScore maxima over the feasible nodes (spec S5)
        for (uint32_t i = tid; i < n; i += 1024) {
            RowT<F> r;
            RowX x;
            row_at(i, r, x);
            if (feasible<F>(r, x, p, px)) {
                const uint32_t a = taint_raw(x, px), b = affinity_raw(x, p, px);
                mt = a > mt ? a : mt;
                ma = b > ma ? b : ma;
            }
        }
        mt = wave_max_u32(mt);
        ma = wave_max_u32(ma);
        if (lane == 0) { red[0][wv] = mt; red[1][wv] = ma; }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            mt = red[0][q] > mt ? red[0][q] : mt;
            ma = red[1][q] > ma ? red[1][q] : ma;
        }
    }
    const double ymt = rcp_exact(mt), yma = rcp_exact(ma);
    uint64_t best = 0;
    for (uint32_t i = tid; i < n; i += 1024) {
        RowT<F> r;
        RowX x;
        row_at(i, r, x);
        const bool f = feasible<F>(r, x, p, px);
        uint32_t sco[4];
        const uint32_t tot = node_total<F>(r, x, p, px, c, mt, ymt, ma, yma, sco);
        const uint64_t key = f ? pack_key(tot + 1, i) : 0ull;
        best = key > best ? key : best;
        packed[i] = pack_scores(f, sco);  // plugin scores are 0..100: one byte each
    }
    best = wave_max_u64(best);
    if (lane == 0) redk[wv] = best;
    __threadfence_system();  // every thread's host-memory stores before the barrier ...
    __syncthreads();
    if (tid == 0) {
#pragma unroll
        for (int q = 0; q < NW; ++q) best = redk[q] > best ? redk[q] : best;
        *reinterpret_cast<volatile uint64_t *>(hout) = best;
        __threadfence_system();
        // ... and the done word last: the host polls it
        __hip_atomic_store(reinterpret_cast<uint64_t *>(hout + 8), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The same call as ONE node per thread, ceil(n / 256) workgroups spread over the XCDs, so a row
// costs one memory round trip instead of ceil(n / 1024) dependent ones on a single CU.  The workgroup
// maxima meet in a device word (gs[0], atomic max); the workgroup that arrives last on gs[1]
// publishes best + done and re-arms the words (the next launch on the stream starts after this one
// has finished).  Same host layout as k_score_pod1.  NormalizeScore profiles first run
// k_score_podg_max (same grid: the feasible nodes' taint / affinity raw maxima into gs[2] / gs[3]);
// the kernel boundary makes them visible to every workgroup here.
constexpr uint32_t kScorePodGT = 1024;  // (fewer workgroups: fewer arrivals on the one counter)
template <uint32_t F>
__global__ __launch_bounds__(kScorePodGT) void k_score_podg_max(DevTable t, PodT<F> p, DPodX px, uint64_t *gs,
                                                                uint32_t pidx, HostRow prow) {
    static_assert((F & kFeatNorm) != 0, "maxima of the normalizing plugins only");
    const uint32_t n = t.n, i = blockIdx.x * kScorePodGT + threadIdx.x;
    uint32_t mt = 0, ma = 0;
    if (i < n) {
        RowT<F> r;
        RowX x;
        if (i == pidx) {
            host_row_regs<F>(prow, r, x);
        } else {
            r = load_row<F>(t, i);
            x = load_rowx<F>(t, i);
        }
        if (feasible<F>(r, x, p, px)) {
            mt = taint_raw(x, px);
            ma = affinity_raw(x, p, px);
        }
    }
    mt = wave_max_u32(mt);
    ma = wave_max_u32(ma);
    if ((threadIdx.x & 63) == 0) {  // one atomic per wave (words stay zero between calls)
        if (mt) __hip_atomic_fetch_max(gs + 2, (uint64_t)mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ma) __hip_atomic_fetch_max(gs + 3, (uint64_t)ma, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
template <uint32_t F>
__global__ __launch_bounds__(kScorePodGT) void k_score_podg(DevTable t, PodT<F> p, DPodX px, DevCfg c,
                                                            uint8_t *hout, uint64_t *gs, uint64_t seq,
                                                            uint32_t pidx, HostRow prow) {
    constexpr int NW = kScorePodGT / kWave;
    __shared__ uint64_t redk[NW];
    const uint32_t n = t.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t i = blockIdx.x * kScorePodGT + tid;
    if (blockIdx.x == 0 && tid == 0 && pidx < n) set_row(t, pidx, prow);
    uint32_t mt = 0, ma = 0;
    if constexpr ((F & kFeatNorm) != 0) {  // k_score_podg_max's maxima (the previous launch)
        mt = (uint32_t)__hip_atomic_load(gs + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ma = (uint32_t)__hip_atomic_load(gs + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t best = 0;
    if (i < n) {
        RowT<F> r;
        RowX x;
        if (i == pidx) {
            host_row_regs<F>(prow, r, x);
        } else {
            r = load_row<F>(t, i);
            x = load_rowx<F>(t, i);
        }
        const bool f = feasible<F>(r, x, p, px);
        uint32_t sco[4];
        const uint32_t tot = node_total<F>(r, x, p, px, c, mt, rcp_exact(mt), ma, rcp_exact(ma), sco);
        best = f ? pack_key(tot + 1, i) : 0ull;
        reinterpret_cast<uint32_t *>(hout + 16)[i] = pack_scores(f, sco);
    }
    best = wave_max_u64(best);
    if (lane == 0) redk[wv] = best;
    // this workgroup's host-memory stores before its arrival: every storing wave drains its own
    // stores, the barrier, then thread 0's system-scope release on the arrival counter (one
    // write-back per workgroup instead of a system fence in every thread)
    drain_stores();
    __syncthreads();
    if (tid == 0) {
#pragma unroll
        for (int q = 0; q < NW; ++q) best = redk[q] > best ? redk[q] : best;
        __hip_atomic_fetch_max(gs, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t old = __hip_atomic_fetch_add(gs + 1, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        if (old + 1 == gridDim.x) {  // last arrival: every workgroup's maximum and outputs are in
            const uint64_t b = __hip_atomic_load(gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gs, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gs + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if constexpr ((F & kFeatNorm) != 0) {  // every workgroup read them before arriving
                __hip_atomic_store(gs + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gs + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            *reinterpret_cast<volatile uint64_t *>(hout) = b;
            __threadfence_system();
            __hip_atomic_store(reinterpret_cast<uint64_t *>(hout + 8), seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// =============================================================================================
// LOOKAHEAD engine
// =============================================================================================
// Block-wide sum of a wave-uniform per-wave value (one barrier; parity-buffered LDS).
template <int NW>
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t (*buf)[NW], int &par, int lane,
                                              int w) {
    if (lane == 0) buf[par][w] = v;
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) s += buf[par][i];
    par ^= 1;
    return s;
}

// Descending bitonic sort of one 64-bit key per lane across the wave (21 compare-exchange steps).
__device__ __forceinline__ uint64_t wave_sort_desc(uint64_t v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, j);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), j);
            const uint64_t o = ((uint64_t)hi << 32) | lo;
            const bool keep_max = ((lane & j) == 0) == ((lane & k) == 0);
            v = keep_max ? (v > o ? v : o) : (v < o ? v : o);
        }
    }
    return v;
}

// Sorts a pod's final list (out[0..L), L <= 64, zero-padded) best-first, so that the top clean
// entries come first (the batched claim walks them in order).  Every thread of the block calls it.
__device__ __forceinline__ void sort_list_desc(uint64_t *__restrict__ out, uint32_t L) {
    __syncthreads();  // the block's stores of out[] are visible to wave 0
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        uint64_t v = (uint32_t)lane < L ? out[lane] : 0ull;
        v = wave_sort_desc(v, lane);
        if ((uint32_t)lane < L) out[lane] = v;
    }
}

// Block-wide top-L of per-position values tv (0 = empty).  Position order is (wave, j, lane):
// wave w owns positions [w*E*64, (w+1)*E*64), so when positions follow node-index order, ranks
// come from ballots and one cross-wave prefix.  Writes the keys of the L largest values to
// out[0..L): every value > T (the L-th largest) in position order, then the ties at T lowest
// position first; zero-fills the rest.  keyf(j) = key of this lane's j-th position.
// Used twice: per node chunk in k_la_select (positions = node indices) and per pod in
// k_la_merge (positions = chunk-major list slots, so equal totals stay in node-index order).
template <int BS, int E, class KeyF>
__device__ __forceinline__ void block_topl(const uint32_t (&tv)[E], uint32_t L,
                                           uint64_t *__restrict__ out, KeyF keyf) {
    constexpr int NW = BS / kWave;
    __shared__ uint32_t cnt[2][NW];
    __shared__ uint32_t cnt2[NW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t lmax = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) lmax = tv[j] > lmax ? tv[j] : lmax;
    int par = 0;
    // block max of tv (a max of wave maxima through the sum buffer)
    const uint32_t wmax = wave_max_u32(lmax);
    if (lane == 0) cnt[par][w] = wmax;
    __syncthreads();
    uint32_t maxtv = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) maxtv = cnt[par][i] > maxtv ? cnt[par][i] : maxtv;
    par ^= 1;
    auto count_ge = [&](uint32_t thr) -> uint32_t {
        uint32_t cw = 0;
#pragma unroll
        for (int j = 0; j < E; ++j) cw += (uint32_t)__popcll(__ballot(tv[j] >= thr));
        return block_sum<NW>(cw, cnt, par, lane, w);
    };
    // T = largest threshold with count(tv >= T) >= L, or 1 if fewer than L non-empty positions.
    uint32_t T = 1;
    if (maxtv > 0) {
        const uint32_t call = count_ge(1);
        if (call > L) {
            if (count_ge(maxtv) >= L) {
                T = maxtv;
            } else {
                uint32_t lo = 1, hi = maxtv;  // count(>=lo) >= L > count(>=hi)
                while (hi - lo > 1) {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    if (count_ge(mid) >= L) lo = mid; else hi = mid;
                }
                T = lo;
            }
        }
    }
    // ballots of "> T" and "== T" per j; one barrier publishes both per-wave counts
    uint64_t gb[E], tb[E];
    uint32_t gt_w = 0, tie_w = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        gb[j] = __ballot(tv[j] > T);
        tb[j] = __ballot(tv[j] == T && maxtv > 0);
        gt_w += (uint32_t)__popcll(gb[j]);
        tie_w += (uint32_t)__popcll(tb[j]);
    }
    if (lane == 0) { cnt[par][w] = gt_w; cnt2[w] = tie_w; }
    __syncthreads();
    uint32_t rg = 0, rt = 0, c_gt = 0, ties_total = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const uint32_t a = cnt[par][i], b = cnt2[i];
        rg += i < w ? a : 0u;
        rt += i < w ? b : 0u;
        c_gt += a;
        ties_total += b;
    }
    const uint32_t need = L > c_gt ? L - c_gt : 0;  // c_gt < L unless fewer than L positions
    const uint64_t lane_mask_lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        if ((gb[j] >> lane) & 1ull) {
            out[rg + (uint32_t)__popcll(gb[j] & lane_mask_lt)] = keyf(j);
        } else if ((tb[j] >> lane) & 1ull) {
            const uint32_t rk = rt + (uint32_t)__popcll(tb[j] & lane_mask_lt);
            if (rk < need) out[c_gt + rk] = keyf(j);
        }
        rg += (uint32_t)__popcll(gb[j]);
        rt += (uint32_t)__popcll(tb[j]);
    }
    const uint32_t written = c_gt + (ties_total < need ? ties_total : need);
    for (uint32_t i = written + tid; i < L; i += BS) out[i] = 0;
}

// Block (v, k, g) of the select grid: shard v owns nodes [v*n/W, (v+1)*n/W).
struct SelBlock {
    uint32_t vs, v, k, g, start, end;
};
__device__ __forceinline__ SelBlock sel_block(const DevTable &t, const LaShard &sh, uint32_t G,
                                              uint32_t chunk, uint32_t bid) {
    SelBlock b;
    const uint32_t per = sh.kw * G;
    b.vs = bid / per;
    const uint32_t rem = bid % per;
    b.v = sh.v0 + b.vs;
    b.k = rem / G;
    b.g = rem % G;
    const uint32_t lo = (uint32_t)((uint64_t)b.v * t.n / sh.W);
    const uint32_t hi = (uint32_t)((uint64_t)(b.v + 1) * t.n / sh.W);
    b.start = lo + b.g * chunk;
    b.end = min(hi, b.start + chunk);
    return b;
}

// Normalizing profiles, pass 1 (same grid as k_la_select): per (shard, pod, chunk) the maxima of
// the raw TaintToleration / NodeAffinity scores over the chunk's feasible nodes and their counts,
// into npart[(v*K + k)*G + g] (the [W][K][G] layout the RCCL all-gather completes).
template <int BS, int E, uint32_t F>
__global__ __launch_bounds__(BS) void k_la_norm(DevTable t, const PodT<F> *__restrict__ pods,
                                                const DPodX *__restrict__ podx, uint32_t s0,
                                                uint32_t P, LaShard sh, uint32_t G, uint32_t K,
                                                uint32_t chunk, uint4 *__restrict__ npart) {
    constexpr int NW = BS / kWave;
    __shared__ uint32_t red[4][NW];
    const SelBlock b = sel_block(t, sh, G, chunk, blockIdx.x);
    const uint32_t s = s0 + b.k;
    if (s >= P) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const PodT<F> p = pods[s];
    const DPodX px = load_vgpr(podx + s);
    const uint32_t base = b.start + (uint32_t)w * E * kWave + lane;
    uint32_t rt[E], ra[E], mt = 0, ma = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const uint32_t idx = base + j * kWave;
        rt[j] = ra[j] = 0xFFFFFFFFu;  // not feasible / not in the chunk
        if (idx < b.end) {
            const RowT<F> r = load_row<F>(t, idx);
            const RowX x = load_rowx<F>(t, idx);
            if (feasible<F>(r, x, p, px)) {
                rt[j] = taint_raw(x, px);
                ra[j] = affinity_raw(x, p, px);
                mt = rt[j] > mt ? rt[j] : mt;
                ma = ra[j] > ma ? ra[j] : ma;
            }
        }
    }
    mt = wave_max_u32(mt);
    ma = wave_max_u32(ma);
    if (lane == 0) { red[0][w] = mt; red[1][w] = ma; }
    __syncthreads();
    mt = ma = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) { mt = red[0][i] > mt ? red[0][i] : mt; ma = red[1][i] > ma ? red[1][i] : ma; }
    uint32_t ct = 0, ca = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        ct += (uint32_t)__popcll(__ballot(rt[j] == mt));
        ca += (uint32_t)__popcll(__ballot(ra[j] == ma));
    }
    if (lane == 0) { red[2][w] = ct; red[3][w] = ca; }
    __syncthreads();
    if (tid == 0) {
        uint4 o = make_uint4(mt, 0, ma, 0);
#pragma unroll
        for (int i = 0; i < NW; ++i) { o.y += red[2][i]; o.w += red[3][i]; }
        npart[((size_t)b.v * K + b.k) * G + b.g] = o;
    }
}

// Combine a pod's [W][G] partials into its NormInfo (max, and the count of nodes attaining it).
__device__ __forceinline__ NormInfo norm_reduce(const uint4 *__restrict__ npart, uint32_t W,
                                                uint32_t K, uint32_t G, uint32_t k) {
    NormInfo r{0, 0, 0, 0};
    for (uint32_t v = 0; v < W; ++v)
        for (uint32_t g = 0; g < G; ++g) {
            const uint4 q = npart[((size_t)v * K + k) * G + g];
            if (q.x > r.mt) { r.mt = q.x; r.ct = 0; }
            if (q.x == r.mt) r.ct += q.y;
            if (q.z > r.ma) { r.ma = q.z; r.ca = 0; }
            if (q.z == r.ma) r.ca += q.w;
        }
    return r;
}

// Grid: shards × pods × G node-chunks.  Block (v, k, g) scores pod s0+k on chunk g of shard v
// (Filter + Score in registers, against the window-start table) and writes the chunk's top-L
// keys to out: straight into the final lists when G == 1, else into the chunk-list scratch
// [nv][kw][G][L] that k_la_merge reduces to one top-L per pod and shard.  Normalizing profiles
// first combine the k_la_norm partials (uniform per pod: scalar loads) and block (0, k, 0) of
// this process publishes the pod's NormInfo for the resolver.
constexpr int kSelB = 4;  // compact rows whose loads a selector lane issues together (la_select_block, res_selector)
template <int BS, int E, uint32_t F>
__device__ __forceinline__ void la_select_block(uint32_t bid, const DevTable &t, const PodT<F> *__restrict__ pods,
                                                const DPodX *__restrict__ podx, const DevCfg &c,
                                                uint32_t s0, uint32_t P, const LaShard &sh,
                                                uint32_t G, uint32_t L, uint32_t chunk,
                                                uint32_t GLp, uint64_t *__restrict__ lists,
                                                uint64_t *__restrict__ clists,
                                                const uint4 *__restrict__ npart, uint32_t K,
                                                NormInfo *__restrict__ norm_out,
                                                const uint32_t *__restrict__ pidx,
                                                const uint32_t *__restrict__ pcount, uint32_t *tickets) {
    const SelBlock b = sel_block(t, sh, G, chunk, bid);
    uint32_t s;
    if (pidx) {  // batched mode: the batch's stream positions and size live on the device
        if (b.k >= *pcount) return;
        s = pidx[b.k];
    } else {
        s = s0 + b.k;
        if (s >= P) return;
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const PodT<F> p = pods[s];
    const bool aa = t.apps && pod_aa(p.flags) != 0;  // batched-mode anti-affinity (spec S11)
    DPodX px{};
    NormInfo nf{0, 0, 0, 0};
    if (F & kFeatNorm) {
        px = load_vgpr(podx + s);
        nf = norm_reduce(npart, sh.W, K, G, b.k);
        if (tid == 0 && b.vs == 0 && b.g == 0) norm_out[b.k] = nf;
    }
    const double ymt = rcp_exact(nf.mt), yma = rcp_exact(nf.ma);
    const uint32_t base = b.start + (uint32_t)w * E * kWave + lane;
    uint32_t tv[E];
    if constexpr ((F & (kFeatWide | kFeatNorm)) == 0) {
        // compact Fit + Balanced (+ext) rows: the loads of kSelB nodes issued together, then the
        // nodes scored one after another (res_selector's form; one round trip per group)
        const __amdgpu_buffer_rsrc_t rs = row_rsrc<F>(t);
#pragma unroll
        for (int j0 = 0; j0 < E; j0 += kSelB) {
            constexpr int B = E < kSelB ? E : kSelB;
            RowQ q[B];
#pragma unroll
            for (int bb = 0; bb < B && j0 + bb < E; ++bb) q[bb] = load_row_q<F>(rs, base + (j0 + bb) * kWave);
#pragma unroll
            for (int bb = 0; bb < B && j0 + bb < E; ++bb) {
                const int j = j0 + bb;
                const uint32_t idx = base + j * kWave;
                tv[j] = 0;
                if (idx < b.end) {
                    RowX x;
                    const Row r = decode_row_q<F>(q[bb], x);
                    const bool f = feasible<F>(r, x, p, px) && (!aa || aa_ok(t, p.flags, idx));
                    const uint32_t tot = node_total<F>(r, x, p, px, c, nf.mt, ymt, nf.ma, yma, nullptr);
                    tv[j] = f ? tot + 1 : 0;
                }
            }
        }
    } else {
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const uint32_t idx = base + j * kWave;
        tv[j] = 0;
        if (idx < b.end) {
            const RowT<F> r = load_row<F>(t, idx);
            const RowX x = load_rowx<F>(t, idx);
            const bool f = feasible<F>(r, x, p, px) && (!aa || aa_ok(t, p.flags, idx));
            const uint32_t tot = node_total<F>(r, x, p, px, c, nf.mt, ymt, nf.ma, yma, nullptr);
            tv[j] = f ? tot + 1 : 0;
        }
    }
    }
    uint64_t *out = G == 1 ? lists + (size_t)b.v * sh.RS + (size_t)b.k * GLp
                           : clists + (((size_t)b.vs * sh.kw + b.k) * G + b.g) * L;
    if (G > 1 && tickets) {
        // batched mode: the chunk list goes out write-through, and the pod's last-arriving chunk
        // block merges the G lists (k_la_merge's routine inside this launch: one launch and its
        // gap less per batch); the merger resets the pod's ticket for the next batch's launch
        __shared__ uint64_t cl_[64];
        __shared__ uint32_t last_;
        block_topl<BS, E>(tv, L, cl_, [&](int j) { return pack_key(tv[j], base + j * kWave); });
        __syncthreads();
        if ((uint32_t)tid < L) store_coh_u64(out + tid, cl_[tid]);
        drain_stores();
        __syncthreads();
        uint32_t *tk = tickets + (size_t)b.vs * sh.kw + b.k;
        if (tid == 0)
            last_ = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == G ? 1u : 0u;
        __syncthreads();
        if (!last_) return;
        if (tid == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        constexpr int E2 = 2;  // G * L <= 2 * BS (the launcher checks)
        const uint32_t M = G * L;
        const uint64_t *in = clists + ((size_t)b.vs * sh.kw + b.k) * M;
        uint64_t e[E2];
        uint32_t t2[E2];
#pragma unroll
        for (int j = 0; j < E2; ++j) {
            const uint32_t pos = (uint32_t)w * E2 * kWave + (uint32_t)j * kWave + lane;
            e[j] = pos < M ? load_coh_u64(in + pos) : 0ull;
            t2[j] = (uint32_t)(e[j] >> 32);
        }
        uint64_t *fin = lists + (size_t)(sh.v0 + b.vs) * sh.RS + (size_t)b.k * GLp;
        block_topl<BS, E2>(t2, L, fin, [&](int j) { return e[j]; });
        sort_list_desc(fin, L);
        return;
    }
    block_topl<BS, E>(tv, L, out, [&](int j) { return pack_key(tv[j], base + j * kWave); });
    if (G == 1) sort_list_desc(out, L);  // a final list (else k_la_merge sorts)
}

template <int BS, int E, uint32_t F>
__global__ __launch_bounds__(BS) void k_la_select(DevTable t, const PodT<F> *__restrict__ pods,
                                                  const DPodX *__restrict__ podx, DevCfg c,
                                                  uint32_t s0, uint32_t P, LaShard sh,
                                                  uint32_t G, uint32_t L, uint32_t chunk,
                                                  uint32_t GLp, uint64_t *__restrict__ lists,
                                                  uint64_t *__restrict__ clists,
                                                  const uint4 *__restrict__ npart, uint32_t K,
                                                  NormInfo *__restrict__ norm_out,
                                                  const uint32_t *__restrict__ pidx,
                                                  const uint32_t *__restrict__ pcount, uint32_t *tickets) {
    la_select_block<BS, E, F>(blockIdx.x, t, pods, podx, c, s0, P, sh, G, L, chunk, GLp, lists, clists,
                              npart, K, norm_out, pidx, pcount, tickets);
}

// Grid: shards × pods.  Reduces a pod's G chunk lists (M = G*L keys, chunk-major: equal totals
// sit in node-index order) to its top-L in the final [W][K][GLp] lists the resolver reads, so the
// resolver scans L keys per pod instead of G*L.
template <int E2>
__device__ __forceinline__ void la_merge_block(uint32_t bid, const uint64_t *__restrict__ clists, uint32_t M,
                                               uint32_t L, const LaShard &sh, uint32_t GLp,
                                               uint64_t *__restrict__ lists) {
    const uint32_t vs = bid / sh.kw, k = bid % sh.kw;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t *in = clists + ((size_t)vs * sh.kw + k) * M;
    uint64_t e[E2];
    uint32_t tv[E2];
#pragma unroll
    for (int j = 0; j < E2; ++j) {
        const uint32_t pos = (uint32_t)w * E2 * kWave + (uint32_t)j * kWave + lane;
        e[j] = pos < M ? in[pos] : 0ull;
        tv[j] = (uint32_t)(e[j] >> 32);
    }
    uint64_t *out = lists + (size_t)(sh.v0 + vs) * sh.RS + (size_t)k * GLp;
    block_topl<256, E2>(tv, L, out, [&](int j) { return e[j]; });
    sort_list_desc(out, L);
}

template <int E2, bool WIDE>
__global__ __launch_bounds__(256) void k_la_merge(const uint64_t *__restrict__ clists, uint32_t M,
                                                  uint32_t L, LaShard sh, uint32_t GLp,
                                                  uint64_t *__restrict__ lists) {
    la_merge_block<E2>(blockIdx.x, clists, M, L, sh, GLp, lists);
}

// Entry m (0 <= m < EPL) of resolver lane `lane` for window pod `pod`.  Lists are laid out
// [shard][pod][GLp] (GLp = 64 * 2^lr entries per pod and shard: the all-gathered layout of the
// sharded engine); entries of shards >= W read as empty.
__device__ __forceinline__ uint64_t list_ent(const uint64_t *__restrict__ lists, uint32_t pod,
                                             uint32_t GLp, uint32_t lr, const LaShard &sh, int m,
                                             int lane) {
    const uint32_t q = (uint32_t)m >> lr;
    if (q >= sh.W) return 0ull;
    return lists[(size_t)q * sh.RS + (size_t)pod * GLp + (uint32_t)lane +
                 64u * ((uint32_t)m & ((1u << lr) - 1u))];
}

// One wave resolves the window sequentially (spec S7 order).  Dirty (modified-in-window) node
// rows live in the lanes' registers (slot = lane); a dynamic-LDS bitmap marks dirty nodes.
// Per pod, off the critical path: the window's pod records sit one per lane (read by readlane),
// the next pod's list entries are prefetched, and every lane prefetches the row of its best clean
// candidate so that a newly dirtied winner's row is already in a register when the argmax lands.
// Results are kept one per lane (lane i = pod i) and stored once per window.
// Diagnostic build only (DIAG = true, QS_DIAG=1 at run time): shader-clock stamps per segment.
__device__ __forceinline__ uint64_t diag_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define QS_STAMP(k)                                  \
    if (DIAG) {                                      \
        const uint64_t t_ = diag_stamp();            \
        dsum[k] += t_ - tprev;                       \
        tprev = t_;                                  \
    }

template <uint32_t F, int EPL, bool DIAG>
__global__ __launch_bounds__(64) void k_la_resolve(DevTable t, const PodT<F> *__restrict__ pods,
                                                   DevCfg c, uint32_t s0, uint32_t P, uint32_t K,
                                                   uint32_t GLp, uint32_t lr, LaShard sh,
                                                   const uint64_t *__restrict__ lists,
                                                   int32_t *__restrict__ out_node,
                                                   uint64_t *__restrict__ out_key,
                                                   uint64_t *__restrict__ stamps,
                                                   uint64_t *__restrict__ diag) {
    wait_lists_ready(c, s0, K);
    uint64_t dsum[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tprev = 0;
    extern __shared__ __attribute__((aligned(16))) uint32_t dirty[];
    const int lane = threadIdx.x;
    const uint32_t nwords = (t.n + 31) / 32;
    for (uint32_t i = lane; i < nwords; i += 64) dirty[i] = 0;
    const uint32_t kend = min(K, P - s0);
    // staging area for a newly dirtied row (after the bitmap; 16-byte aligned)
    RowT<F> *stage = (RowT<F> *)(dirty + ((nwords + 3) & ~3u));
    RowX *stagex = (RowX *)(stage + 1);
    PodT<F> pn = pods[s0];  // uniform: scalar loads, prefetched one pod ahead
    const DPodX px{};
    RowT<F> dr = empty_row<F>();
    RowX dx{};
    uint32_t didx = 0xFFFFFFFFu;
    uint32_t nd = 0;
    uint64_t res_key = 0, res_stamp = 0;
    // Software pipeline (three pods in flight):
    //   pod i:   clean candidate = top-1 of the lane's entries, or top-2 when top-1 is the previous
    //            pod's winner (both rows loaded one pod earlier: no memory or LDS on the path);
    //   pod i+1: top-2 clean entries against the current dirty set (LDS bitmap) + their row loads;
    //   pod i+2: list entries loaded.
    uint64_t ent1[EPL], ent2[EPL];
#pragma unroll
    for (int m = 0; m < EPL; ++m) ent1[m] = list_ent(lists, 0, GLp, lr, sh, m, lane);
#pragma unroll
    for (int m = 0; m < EPL; ++m) ent2[m] = kend > 1 ? list_ent(lists, 1, GLp, lr, sh, m, lane) : 0ull;
    __syncthreads();
    // top-2 clean entries of a pod's list against the dirty bitmap
    auto top2 = [&](const uint64_t (&e)[EPL], uint64_t &c1, uint64_t &c2) {
        uint32_t word[EPL];
#pragma unroll
        for (int m = 0; m < EPL; ++m) {
            const uint32_t nidx = e[m] ? key_node(e[m]) : 0u;
            word[m] = dirty[nidx >> 5] >> (nidx & 31);
        }
        c1 = 0;
        c2 = 0;
#pragma unroll
        for (int m = 0; m < EPL; ++m) {
            const uint64_t x = (word[m] & 1u) ? 0ull : e[m];
            const bool gt1 = x > c1;
            c2 = gt1 ? c1 : (x > c2 ? x : c2);
            c1 = gt1 ? x : c1;
        }
    };
    uint64_t c1, c2;
    top2(ent1, c1, c2);
    RowT<F> r1 = load_row<F>(t, c1 ? key_node(c1) : 0u), r2 = load_row<F>(t, c2 ? key_node(c2) : 0u);
    RowX x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u), x2 = load_rowx<F>(t, c2 ? key_node(c2) : 0u);
    uint32_t wprev = 0xFFFFFFFFu;
    if (DIAG) tprev = diag_stamp();
    for (uint32_t i = 0; i < kend; ++i) {
        const PodT<F> p = pn;
        if (i + 1 < kend) pn = pods[s0 + i + 1];
        // this pod's clean candidate: the previous winner is the only node dirtied since top2()
        const bool use2 = c1 && key_node(c1) == wprev;
        const uint64_t cand = use2 ? c2 : c1;
        const RowT<F> crow = sel_row(use2, r2, r1);
        const RowX cx = sel_rowx(use2, x2, x1);
        QS_STAMP(0)
        // next pod: top-2 clean entries and their rows; the pod after: its list entries
        if (i + 1 < kend) {
            top2(ent2, c1, c2);
            r1 = load_row<F>(t, c1 ? key_node(c1) : 0u);
            r2 = load_row<F>(t, c2 ? key_node(c2) : 0u);
            x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u);
            x2 = load_rowx<F>(t, c2 ? key_node(c2) : 0u);
        }
        if (i + 2 < kend) {
#pragma unroll
            for (int m = 0; m < EPL; ++m) ent2[m] = list_ent(lists, i + 2, GLp, lr, sh, m, lane);
        }
        QS_STAMP(1)
        // fresh keys of the dirty slots
        const bool f = feasible<F>(dr, dx, p, px);
        const uint32_t tot = node_total<F>(dr, dx, p, px, c, 0, 0.0, 0, 0.0, nullptr);
        const uint64_t fk = ((uint32_t)lane < nd && f) ? pack_key(tot + 1, didx) : 0ull;
        const uint64_t best = fk > cand ? fk : cand;
        QS_STAMP(2)
        const uint64_t ks = wave_max_u64(best);
        QS_STAMP(3)
        if (ks) {
            const uint32_t win = key_node(ks);
            const bool own = (uint32_t)lane < nd && didx == win;
            if (__ballot(own)) {
                if (own) reserve(dr, dx, p, +1);
            } else {
                // the winner is a clean node: its row was prefetched by the lane whose cand == ks;
                // hand it to slot lane nd through LDS (same wave: LDS operations stay in order)
                const int src = (int)__builtin_ctzll(__ballot(cand == ks));
                if (lane == src) { *stage = crow; if (F & kFeatExt) *stagex = cx; }
                const RowT<F> nr = *stage;
                RowX nx{};
                if (F & kFeatExt) nx = *stagex;
                if ((uint32_t)lane == nd) {
                    dr = nr;
                    dx = nx;
                    reserve(dr, dx, p, +1);
                    didx = win;
                    dirty[win >> 5] |= 1u << (win & 31);
                }
                ++nd;
            }
        }
        wprev = ks ? key_node(ks) : 0xFFFFFFFFu;
        QS_STAMP(4)
        if ((uint32_t)lane == i) {
            res_key = ks;
            if (stamps) res_stamp = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (DIAG && lane == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd((unsigned long long *)&diag[k], (unsigned long long)dsum[k]);
        atomicAdd((unsigned long long *)&diag[5], (unsigned long long)kend);
    }
    if ((uint32_t)lane < kend) {
        const uint32_t s = s0 + lane;
        out_node[s] = res_key ? (int32_t)key_node(res_key) : -1;
        if (out_key) out_key[s] = res_key;
        if (stamps) stamps[s] = res_stamp;
    }
    if ((uint32_t)lane < nd) { store_dyn<F>(t, didx, dr); store_dynx<F>(t, didx, dx); }
}

// Single-wave resolver for normalizing profiles (TaintToleration / NodeAffinity on).  Keys carry
// per-pod normalized scores, so a list is only valid while the pod's selection-time maxima (nf)
// still hold.  The feasible set only shrinks during a stream, and only dirty nodes changed, so a
// maximum still holds whenever fewer of its holders than nf.ct / nf.ca are dirty AND infeasible
// now; otherwise (rare: few holders left) the wave rescans every node at the current state for
// the exact maxima and keys (`nfall` counts those pods).  Supports overlapped windows (dprev/dcur)
// like k_la_resolve4.  Four waves run the walk redundantly (identical lane state, LDS writes of
// identical values, one barrier per pod) so that an exact rescan is spread over all four SIMDs;
// only wave 0 writes results.
constexpr uint32_t kResNormWaves = 4;
template <uint32_t F, int EPL>
__device__ __forceinline__ void la_resolve_norm_body(
    uint32_t *lds, const DevTable &t, const PodT<F> *__restrict__ pods, const DPodX *__restrict__ podx,
    const DevCfg &c, uint32_t s0, uint32_t P, uint32_t K, uint32_t GLp, uint32_t lr, const LaShard &sh,
    const uint64_t *__restrict__ lists, const NormInfo *__restrict__ norm,
    int32_t *__restrict__ out_node, uint64_t *__restrict__ out_key, uint64_t *__restrict__ stamps,
    const uint32_t *__restrict__ dprev, uint32_t *__restrict__ dcur, unsigned long long *nfall,
    const uint32_t *__restrict__ rec) {
    __shared__ uint32_t red_m[2 * kResNormWaves];  // per-wave rescan maxima (taint, affinity)
    __shared__ uint64_t red_k[kResNormWaves];      // per-wave rescan best keys
    const int lane = threadIdx.x & 63;
    const uint32_t wid = threadIdx.x >> 6;
    // Resume mode (rec != nullptr, after the four-wave resolver of the same window): nothing to do
    // unless it stopped at pod rec[0]; then continue from there with its slots (rec[1] nodes at
    // rec[4..], rows already stored, won mask rec[2..3]) as the initial dirty set.
    uint32_t pbase = 0;
    uint64_t won0 = 0;
    const uint32_t *init = dprev;
    if (rec) {
        // (vector loads: the record may have been written earlier in this launch, by wave D)
        const uint32_t stop = load_coh_u32(rec);
        if (stop == 0xFFFFFFFFu) return;
        if (threadIdx.x == 0 && nfall) atomicAdd(nfall + 1, 1ull);  // resumed windows (QS_NORM_DIAG)
        pbase = stop;
        s0 += stop;
        K -= stop;
        won0 = (uint64_t)load_coh_u32(rec + 2) | ((uint64_t)load_coh_u32(rec + 3) << 32);
        init = rec + 3;  // init[1 + j] = rec[4 + j]; the count is rec[1]
    }
    const uint32_t n = t.n, nwords = (n + 31) / 32;
    uint32_t *dirty = lds;
    RowT<F> *srow = (RowT<F> *)(lds + ((nwords + 3) & ~3u));  // [64] slot rows, staged for a rescan
    RowX *sx = (RowX *)(srow + 64);                    // [64]
    RowT<F> *stage = (RowT<F> *)(sx + 64);                     // newly dirtied row hand-off
    RowX *stagex = (RowX *)(stage + 1);
    uint32_t *sidx = (uint32_t *)(stagex + 1);         // [64] slot -> node, staged for a rescan
    for (uint32_t i = lane; i < nwords; i += 64) dirty[i] = 0;
    const uint32_t kend = min(K, P - s0);
    const uint32_t nd0 = rec ? load_coh_u32(rec + 1) : (dprev ? dprev[0] : 0u);
    __syncthreads();
    RowT<F> dr = empty_row<F>();
    RowX dx{};
    uint32_t didx = 0xFFFFFFFFu;
    if ((uint32_t)lane < nd0) {
        didx = rec ? load_coh_u32(init + 1 + lane) : init[1 + lane];
        dr = load_row<F>(t, didx);
        dx = load_rowx<F>(t, didx);
        atomicOr(&dirty[didx >> 5], 1u << (didx & 31));
    }
    uint32_t nd = nd0;
    bool won = (uint32_t)lane < nd0 && ((won0 >> lane) & 1ull);
    uint64_t res_key = 0, res_stamp = 0;
    __syncthreads();
    auto top2 = [&](const uint64_t(&e)[EPL], uint64_t &c1, uint64_t &c2) {
        uint32_t word[EPL];
#pragma unroll
        for (int m = 0; m < EPL; ++m) {
            const uint32_t nidx = e[m] ? key_node(e[m]) : 0u;
            word[m] = dirty[nidx >> 5] >> (nidx & 31);
        }
        c1 = c2 = 0;
#pragma unroll
        for (int m = 0; m < EPL; ++m) {
            const uint64_t x = (word[m] & 1u) ? 0ull : e[m];
            const bool gt1 = x > c1;
            c2 = gt1 ? c1 : (x > c2 ? x : c2);
            c1 = gt1 ? x : c1;
        }
    };
    uint64_t ent1[EPL], ent2[EPL];
#pragma unroll
    for (int m = 0; m < EPL; ++m) ent1[m] = list_ent(lists, pbase, GLp, lr, sh, m, lane);
#pragma unroll
    for (int m = 0; m < EPL; ++m) ent2[m] = kend > 1 ? list_ent(lists, pbase + 1, GLp, lr, sh, m, lane) : 0ull;
    uint64_t c1, c2;
    top2(ent1, c1, c2);
    RowT<F> r1 = load_row<F>(t, c1 ? key_node(c1) : 0u), r2 = load_row<F>(t, c2 ? key_node(c2) : 0u);
    RowX x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u), x2 = load_rowx<F>(t, c2 ? key_node(c2) : 0u);
    uint32_t wprev = 0xFFFFFFFFu;
    // pod records + normalization facts, one pod ahead, through the vector path (scalar copies
    // of the 44-dword extension record spilled the SGPRs)
    PodT<F> pn = load_vgpr(pods + s0);
    DPodX pxn = load_vgpr(podx + s0);
    NormInfo nfn = load_vgpr(norm + pbase);
    for (uint32_t i = 0; i < kend; ++i) {
        const PodT<F> p = pn;
        const DPodX px = pxn;
        const NormInfo nf = nfn;
        if (i + 1 < kend) {
            pn = load_vgpr(pods + s0 + i + 1);
            pxn = load_vgpr(podx + s0 + i + 1);
            nfn = load_vgpr(norm + pbase + i + 1);
        }
        const bool use2 = c1 && key_node(c1) == wprev;
        const uint64_t cand = use2 ? c2 : c1;
        const RowT<F> crow = sel_row(use2, r2, r1);
        const RowX cx = sel_rowx(use2, x2, x1);
        if (i + 1 < kend) {  // next pod's candidates and rows; the pod after: its list entries
            top2(ent2, c1, c2);
            r1 = load_row<F>(t, c1 ? key_node(c1) : 0u);
            r2 = load_row<F>(t, c2 ? key_node(c2) : 0u);
            x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u);
            x2 = load_rowx<F>(t, c2 ? key_node(c2) : 0u);
        }
        if (i + 2 < kend) {
#pragma unroll
            for (int m = 0; m < EPL; ++m) ent2[m] = list_ent(lists, pbase + i + 2, GLp, lr, sh, m, lane);
        }
        const double ymt = rcp_exact(nf.mt), yma = rcp_exact(nf.ma);
        const bool act = (uint32_t)lane < nd;
        const bool f = feasible<F>(dr, dx, p, px);
        const uint32_t tot = node_total<F>(dr, dx, p, px, c, nf.mt, ymt, nf.ma, yma, nullptr);
        const uint64_t fk = (act && f) ? pack_key(tot + 1, didx) : 0ull;
        // do the selection-time maxima still hold?  (holders lost = dirty, infeasible now)
        bool unsafe = false;
        if (F & kFeatTaint) {
            const uint32_t lost = (uint32_t)__popcll(__ballot(act && !f && taint_raw(dx, px) == nf.mt));
            unsafe |= nf.mt > 0 && lost >= nf.ct;
        }
        if (F & kFeatAffinity) {
            const uint32_t lost = (uint32_t)__popcll(__ballot(act && !f && affinity_raw(dx, p, px) == nf.ma));
            unsafe |= nf.ma > 0 && lost >= nf.ca;
        }
        uint64_t ks;
        if (!unsafe) {
            ks = wave_max_u64(fk > cand ? fk : cand);
        } else {
            // exact rescan at the current state: slot rows from LDS, every other row from HBM
            if (act) { srow[lane] = dr; sx[lane] = dx; sidx[lane] = didx; }
            // both passes keep U rows per lane in flight (one wave, dependent loads otherwise):
            // every row is loaded unconditionally first, and only then are the few dirty ones
            // (held by a slot, stale in HBM) replaced from LDS, so no branch or search loop sits
            // between the loads and forces them to complete one by one
            constexpr uint32_t U = 8;
            auto rows_at = [&](uint32_t b0, RowT<F> (&r)[U], RowX (&x)[U]) {
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t idx = b0 + 64 * u < n ? b0 + 64 * u : 0u;
                    r[u] = load_row<F>(t, idx);
                    x[u] = load_rowx<F>(t, idx);
                }
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t idx = b0 + 64 * u;
                    if (idx < n && ((dirty[idx >> 5] >> (idx & 31)) & 1u)) {
                        uint32_t j = 0;
                        while (j < nd && sidx[j] != idx) ++j;  // dirty => held by a slot
                        r[u] = srow[j];
                        x[u] = sx[j];
                    }
                }
            };
            uint32_t mt = 0, ma = 0;
            for (uint32_t b0 = wid * 64 * U + lane; b0 < n; b0 += kResNormWaves * 64 * U) {
                RowT<F> r[U];
                RowX x[U];
                rows_at(b0, r, x);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    if (b0 + 64 * u < n && feasible<F>(r[u], x[u], p, px)) {
                        const uint32_t a = taint_raw(x[u], px), b2 = affinity_raw(x[u], p, px);
                        mt = a > mt ? a : mt;
                        ma = b2 > ma ? b2 : ma;
                    }
                }
            }
            mt = (F & kFeatTaint) ? wave_max_u32(mt) : 0u;
            ma = (F & kFeatAffinity) ? wave_max_u32(ma) : 0u;
            if (lane == 0) { red_m[2 * wid] = mt; red_m[2 * wid + 1] = ma; }
            __syncthreads();
#pragma unroll
            for (uint32_t w = 0; w < kResNormWaves; ++w) {
                mt = red_m[2 * w] > mt ? red_m[2 * w] : mt;
                ma = red_m[2 * w + 1] > ma ? red_m[2 * w + 1] : ma;
            }
            const double ymt2 = rcp_exact(mt), yma2 = rcp_exact(ma);
            uint64_t best = 0;
            for (uint32_t b0 = wid * 64 * U + lane; b0 < n; b0 += kResNormWaves * 64 * U) {
                RowT<F> r[U];
                RowX x[U];
                rows_at(b0, r, x);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t idx = b0 + 64 * u;
                    const uint32_t tv = node_total<F>(r[u], x[u], p, px, c, mt, ymt2, ma, yma2, nullptr);
                    const uint64_t key = (idx < n && feasible<F>(r[u], x[u], p, px)) ? pack_key(tv + 1, idx) : 0ull;
                    best = key > best ? key : best;
                }
            }
            ks = wave_max_u64(best);
            if (lane == 0) red_k[wid] = ks;
            __syncthreads();
#pragma unroll
            for (uint32_t w = 0; w < kResNormWaves; ++w) ks = red_k[w] > ks ? red_k[w] : ks;
            if (threadIdx.x == 0 && nfall) atomicAdd(nfall, 1ull);
        }
        __syncthreads();  // every wave has read this pod's dirty bits before any marks the winner
        if (ks) {
            const uint32_t win = key_node(ks);
            const uint64_t own = __ballot(act && didx == win);
            if (own) {
                if (lane == __builtin_ctzll(own)) { reserve(dr, dx, p, +1); won = true; }
            } else {
                // clean winner: its row was prefetched by a lane whose candidate it is (after a
                // rescan it may be nobody's candidate: then lane 0 loads it)
                const uint64_t srcm = __ballot(cand == ks);
                if (srcm) {
                    if (lane == __builtin_ctzll(srcm)) { *stage = crow; *stagex = cx; }
                } else if (lane == 0) {
                    *stage = load_row<F>(t, win);
                    *stagex = load_rowx<F>(t, win);
                }
                const RowT<F> nr = *stage;
                const RowX nx = *stagex;
                if ((uint32_t)lane == nd) {
                    dr = nr;
                    dx = nx;
                    reserve(dr, dx, p, +1);
                    didx = win;
                    won = true;
                    dirty[win >> 5] |= 1u << (win & 31);
                }
                ++nd;
            }
        }
        wprev = ks ? key_node(ks) : 0xFFFFFFFFu;
        if ((uint32_t)lane == i) {
            res_key = ks;
            if (stamps) res_stamp = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();  // no wave overwrites stage / the rescan partials while another reads them
    }
    if (wid != 0) return;
    if ((uint32_t)lane < kend) {
        const uint32_t s = s0 + lane;
        out_node[s] = res_key ? (int32_t)key_node(res_key) : -1;
        if (out_key) out_key[s] = res_key;
        if (stamps) stamps[s] = res_stamp;
    }
    if ((uint32_t)lane < nd) { store_dyn<F>(t, didx, dr); store_dynx<F>(t, didx, dx); }
    if (dcur) {
        const uint64_t wm = __ballot(won && (uint32_t)lane < nd);
        if (won && (uint32_t)lane < nd) dcur[1 + __popcll(wm & ((1ull << lane) - 1ull))] = didx;
        if (lane == 0) dcur[0] = (uint32_t)__popcll(wm);
    }
}

template <uint32_t F, int EPL>
__global__ __launch_bounds__(64 * kResNormWaves) void k_la_resolve_norm(
    DevTable t, const PodT<F> *__restrict__ pods, const DPodX *__restrict__ podx, DevCfg c,
    uint32_t s0, uint32_t P, uint32_t K, uint32_t GLp, uint32_t lr, LaShard sh,
    const uint64_t *__restrict__ lists, const NormInfo *__restrict__ norm,
    int32_t *__restrict__ out_node, uint64_t *__restrict__ out_key, uint64_t *__restrict__ stamps,
    const uint32_t *__restrict__ dprev, uint32_t *__restrict__ dcur, unsigned long long *nfall,
    const uint32_t *__restrict__ rec) {
    if (!rec) wait_lists_ready(c, s0, K);  // resume mode follows the four-wave kernel on its stream
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    la_resolve_norm_body<F, EPL>(lds, t, pods, podx, c, s0, P, K, GLp, lr, sh, lists, norm, out_node, out_key,
                                 stamps, dprev, dcur, nfall, rec);
}

// ---------------------------------------------------------------------------------------------
// Four-wave pipelined resolver (one wave per SIMD).  Pod i's dirty-slot keys never wait for an
// evaluation: they were computed during pod i-1 for both outcomes —
//   wave A: A_l = key_{i+1}(slot_l)              (slot l not the winner of pod i)
//   wave B: B_l = key_{i+1}(slot_l + pod i)      (slot l wins pod i)
//   wave C: C_l = key_{i+1}(cand_l(i) + pod i)   (lane l's clean candidate wins pod i: new slot),
//           plus the top-2 clean list entries of pod i+1 and their rows (loaded one pod ahead);
//   wave D: picks pod i's keys from A/B/C with pod i-1's winner, argmax, publishes the winner.
// One LDS exchange + one s_barrier per pod.  Slot rows are replicated in waves A and B; a new
// slot's row comes from wave C's staging copy of its candidate row.
struct alignas(16) ResPub {
    uint64_t ks;     // packed key of the winner (0 = unschedulable)
    uint32_t w;      // winner node
    int32_t slot;    // existing dirty slot that won, or -1
    int32_t src;     // lane whose clean candidate won (new slot)
    uint32_t nd_old; // lane of the new slot
    uint32_t pad[2];
};
// One 32-byte LDS read of the published winner (two ds_read_b128 issued together; reading the
// fields lazily under branches serialised four LDS round trips).
__device__ __forceinline__ ResPub read_pub(const ResPub *p) {
    const uint4 a = reinterpret_cast<const uint4 *>(p)[0];
    const uint4 b = reinterpret_cast<const uint4 *>(p)[1];
    ResPub r;
    r.ks = ((uint64_t)a.y << 32) | a.x;
    r.w = a.z;
    r.slot = (int32_t)a.w;
    r.src = (int32_t)b.x;
    r.nd_old = b.y;
    r.pad[0] = r.pad[1] = 0;
    return r;
}

template <uint32_t F, int EPL, bool DIAG, bool K32>
__device__ __forceinline__ void la_resolve4_block(uint32_t *lds, const DevTable &t, const PodT<F> *__restrict__ pods,
                                                  const DevCfg &c, uint32_t s0, uint32_t P,
                                                  uint32_t K, uint32_t GLp, uint32_t lr,
                                                  const LaShard &sh,
                                                  const uint64_t *__restrict__ lists,
                                                  int32_t *__restrict__ out_node,
                                                  uint64_t *__restrict__ out_key,
                                                  uint64_t *__restrict__ stamps,
                                                  uint64_t *__restrict__ diag,
                                                  const uint32_t *__restrict__ dprev,
                                                  uint32_t *__restrict__ dcur,
                                                  const DPodX *__restrict__ podx = nullptr,
                                                  const NormInfo *__restrict__ norm = nullptr,
                                                  uint32_t *__restrict__ rec = nullptr) {
    constexpr bool NORM = (F & kFeatNorm) != 0;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t t_start = DIAG ? diag_stamp() : 0ull;
    uint64_t t_loop = 0;
    const uint32_t nwords = (t.n + 31) / 32;
    uint32_t *dirty = lds;
    char *base = (char *)(lds + ((nwords + 3) & ~3u));
    uint64_t(*keyA)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*keyB)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*keyC)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*C1)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*C2)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    RowT<F>(*stage)[64] = (RowT<F>(*)[64])base; base += 2 * 64 * sizeof(RowT<F>);
    int4(*stagex)[64] = (int4(*)[64])base; base += 2 * 64 * sizeof(int4);
    ResPub *pub = (ResPub *)base; base += 2 * sizeof(ResPub);
    uint32_t *slotnode = (uint32_t *)base; base += 64 * 4;
    PodT<F> *wpods = (PodT<F> *)base; base += 64 * sizeof(PodT<F>);  // the window's pod records (K <= 64)
    // normalizing profiles only (the host sizes the LDS accordingly): pod extensions, the
    // selection-time maxima and their reciprocals, C's lost-holder flags, full staged RowX
    DPodX *wpodx = (DPodX *)base; base += 64 * sizeof(DPodX);
    NormInfo *wnorm = (NormInfo *)base; base += 64 * sizeof(NormInfo);
    double2 *wrcp = (double2 *)base; base += 64 * sizeof(double2);
    uint32_t(*flagC)[64] = (uint32_t(*)[64])base; base += 2 * 64 * 4;
    RowX(*stagexN)[64] = (RowX(*)[64])base;

    for (uint32_t i = threadIdx.x; i < nwords; i += 256) dirty[i] = 0;
    if (threadIdx.x == 0) pub[1] = ResPub{0, 0xFFFFFFFFu, -1, -1, 0, {0, 0}};
    const uint32_t kend = min(K, P - s0);
    if (threadIdx.x < kend) wpods[threadIdx.x] = pods[s0 + threadIdx.x];
    if (NORM) {
        constexpr uint32_t q = sizeof(DPodX) / 16;
        for (uint32_t j = threadIdx.x; j < kend * q; j += 256)
            reinterpret_cast<uint4 *>(wpodx)[j] = reinterpret_cast<const uint4 *>(podx + s0)[j];
        if (threadIdx.x < kend) {
            const NormInfo nf = norm[threadIdx.x];
            wnorm[threadIdx.x] = nf;
            wrcp[threadIdx.x] = make_double2(rcp_exact(nf.mt), rcp_exact(nf.ma));
        }
    }
    const DPodX px{};
    DevCfg cv = c;  // (weights in VGPRs, as in la_resolve4_stream)
    asm volatile("" : "+v"(cv.yd_both), "+v"(cv.yd_c), "+v"(cv.yd_m), "+v"(cv.wc), "+v"(cv.wm));
    // Overlapped windows (dprev != nullptr): this window's lists were selected against the table
    // as it stood BEFORE the previous window, so the nodes that window dirtied (dprev[1..nd0])
    // start as dirty slots: their list entries are stale and their rows are re-read here.
    const uint32_t nd0 = dprev ? dprev[0] : 0u;
    __syncthreads();
    if (threadIdx.x < nd0) {
        const uint32_t nn = dprev[1 + threadIdx.x];
        atomicOr(&dirty[nn >> 5], 1u << (nn & 31));
    }
    __syncthreads();
    if (kend == 0) return;
    uint64_t dsum = 0, tprev = 0, dpart = 0, dwait = 0;
#define QS_DIAG_BEGIN() if (DIAG) tprev = diag_stamp();
#define QS_DIAG_END() if (DIAG) { const uint64_t t_ = diag_stamp(); dsum += t_ - tprev; }

    // Each role runs its own loop; every wave executes one s_barrier per pod (+1 prologue), so
    // the barriers pair up.  Roles never share registers, which keeps waitcnt placement local.
    if (wv == 0) {
        // ---- D: pod i's winner from the precomputed keys ---------------------------------------
        uint32_t nd = nd0, didx = (uint32_t)lane < nd0 ? dprev[1 + lane] : 0xFFFFFFFFu;
        bool won = false;  // slot won a pod of THIS window (it belongs to the next window's dprev)
        uint64_t res_key = 0, res_stamp = 0;
        uint32_t kdone = kend;  // normalizing profiles: the pod a stop hands to the resume kernel
        ResPub pv{0, 0xFFFFFFFFu, -1, -1, 0, {0, 0}};  // D produced it: kept in registers
        __syncthreads();  // prologue barrier (wave C publishes pod 0's candidates)
        if (DIAG && lane == 0) atomicAdd((unsigned long long *)&diag[8], (unsigned long long)(diag_stamp() - t_start));
        for (uint32_t i = 0; i < kend; ++i) {
            QS_DIAG_BEGIN()
            const int par = i & 1, pp = par ^ 1;
            // every LDS read of the step is independent of this step: one batch, one wait
            const uint64_t a = keyA[pp][lane], b = keyB[pp][lane], cl = keyC[pp][lane];
            const uint64_t e1 = C1[pp][lane], e2 = EPL > 1 ? C2[pp][lane] : 0ull;
            const bool pnew = pv.ks != 0 && pv.slot < 0;
            uint64_t sc = (lane == pv.slot) ? b : a;
            uint32_t fl = 0;  // NORM: lost-holder flags of this slot (bit 0 taint, bit 1 affinity)
            if (NORM) {
                fl = (uint32_t)sc & 3u;
                sc &= ~3ull;
            }
            uint64_t fk = ((uint32_t)lane < nd && sc) ? (sc | (uint64_t)(0xFFFFFFFFu - didx)) : 0ull;
            if (pnew) {
                const uint64_t cw = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(cl >> 32), pv.src) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cl, pv.src);
                if ((uint32_t)lane == pv.nd_old) fk = cw;
                if (NORM) {
                    const uint32_t fc = (uint32_t)__builtin_amdgcn_readlane((int)flagC[pp][lane], pv.src);
                    if ((uint32_t)lane == pv.nd_old) fl = fc;
                }
            }
            if (NORM) {
                // do the selection-time maxima still hold for pod i?  A maximum is lost only when
                // every node attaining it is dirty and infeasible now; then the resume kernel
                // (k_la_resolve_norm) takes over from pod i with an exact rescan
                const NormInfo nf = wnorm[i];
                bool unsafe = false;
                if (F & kFeatTaint)
                    unsafe |= nf.mt > 0 && (uint32_t)__popcll(__ballot((uint32_t)lane < nd && (fl & 1u))) >= nf.ct;
                if (F & kFeatAffinity)
                    unsafe |= nf.ma > 0 && (uint32_t)__popcll(__ballot((uint32_t)lane < nd && (fl & 2u))) >= nf.ca;
                if (unsafe) {
                    if (lane == 0) pub[par] = ResPub{0, 0xFFFFFFFFu, -2, -1, nd, {0, 0}};  // STOP
                    kdone = i;
                    __syncthreads();
                    break;
                }
            }
            const uint64_t cand = (pv.ks != 0 && e1 != 0 && key_node(e1) == pv.w) ? e2 : e1;
            const uint64_t best = fk > cand ? fk : cand;
            uint64_t ks;
            if (K32) {  // (score+1) < 2^10 and n <= 2^22: one 32-bit reduction
                const uint32_t tv = (uint32_t)(best >> 32);
                const uint32_t k32 = tv ? (tv << 22) | (0x3FFFFFu - key_node(best)) : 0u;
                const uint32_t m = wave_max_u32(k32);
                ks = m ? (((uint64_t)(m >> 22) << 32) | (uint64_t)(0xFFFFFFFFu - (0x3FFFFFu - (m & 0x3FFFFFu)))) : 0ull;
            } else {
                ks = wave_max_u64(best);
            }
            ResPub np{ks, ks ? key_node(ks) : 0xFFFFFFFFu, -1, -1, nd, {0, 0}};
            if (ks) {
                const uint64_t own = __ballot((uint32_t)lane < nd && didx == np.w);
                if (own) {
                    np.slot = (int32_t)__builtin_ctzll(own);
                    won |= lane == np.slot;
                } else {
                    np.src = (int32_t)__builtin_ctzll(__ballot(cand == ks));
                    if ((uint32_t)lane == nd) { didx = np.w; won = true; }
                    ++nd;
                }
            }
            pv = np;
            if (lane == 0) pub[par] = np;
            if ((uint32_t)lane == i) {
                res_key = ks;
                if (stamps) res_stamp = __builtin_amdgcn_s_memrealtime();
            }
            QS_DIAG_END()
            __syncthreads();
        }
        if (DIAG) t_loop = diag_stamp();
        if ((uint32_t)lane < kdone) {
            const uint32_t s = s0 + lane;
            out_node[s] = res_key ? (int32_t)key_node(res_key) : -1;
            if (out_key) out_key[s] = res_key;
            if (stamps) stamps[s] = res_stamp;
        }
        if ((uint32_t)lane < nd) slotnode[lane] = didx;
        if (kdone < kend) {
            // stopped: hand the window state to the resume kernel — rec = {first pod left, slots,
            // won mask lo/hi, slot nodes}; it writes dcur when it finishes the window
            const uint64_t wm = __ballot(won && (uint32_t)lane < nd);
            if (lane == 0) {
                rec[0] = kdone;
                rec[1] = nd;
                rec[2] = (uint32_t)wm;
                rec[3] = (uint32_t)(wm >> 32);
            }
            if ((uint32_t)lane < nd) rec[4 + lane] = didx;
        } else {
            if (rec && lane == 0) rec[0] = 0xFFFFFFFFu;
            if (dcur) {  // nodes dirtied in this window, for the next (overlapped) window
                const uint64_t wm = __ballot(won && (uint32_t)lane < nd);
                if (won && (uint32_t)lane < nd) dcur[1 + __popcll(wm & ((1ull << lane) - 1ull))] = didx;
                if (lane == 0) dcur[0] = (uint32_t)__popcll(wm);
            }
        }
    } else if (wv <= 2) {
        // ---- A / B: apply pod i-1 to the slot copy, then the next pod's keys --------------------
        RowT<F> S = empty_row<F>();
        RowX SX{};
        uint32_t nd = nd0;
        if ((uint32_t)lane < nd0) {
            const uint32_t nn = dprev[1 + lane];
            S = load_row<F>(t, nn);
            SX = load_rowx<F>(t, nn);
        }
        // score half of a slot key for window pod k (+ NORM lost-holder flags in bits 0-1)
        // NORM: pod k's extension record, maxima and reciprocals, read from LDS one step ahead
        struct PodN {
            DPodX x;
            NormInfo nf;
            double2 yr;
        };
        auto podn = [&](uint32_t k) -> PodN {
            PodN r{};
            if (NORM && k < kend) r = PodN{wpodx[k], wnorm[k], wrcp[k]};
            return r;
        };
        auto slot_key = [&](const RowT<F> &r, const RowX &x, const PodT<F> &q, const PodN &pn) -> uint64_t {
            const bool act = (uint32_t)lane < nd;
            if (NORM) {
                const DPodX &qx = pn.x;
                const NormInfo nf = pn.nf;
                const double2 yr = pn.yr;
                const bool f = feasible<F>(r, x, q, qx);
                const uint32_t tot = node_total<F>(r, x, q, qx, cv, nf.mt, yr.x, nf.ma, yr.y, nullptr);
                uint32_t fl = 0;
                if (act && !f) {
                    if (F & kFeatTaint) fl |= taint_raw(x, qx) == nf.mt ? 1u : 0u;
                    if (F & kFeatAffinity) fl |= affinity_raw(x, q, qx) == nf.ma ? 2u : 0u;
                }
                return ((act && f) ? ((uint64_t)(tot + 1) << 32) : 0ull) | fl;
            }
            const bool f = feasible<F>(r, x, q, px);
            const uint32_t tot = node_total<F>(r, x, q, px, cv, 0, 0.0, 0, 0.0, nullptr);
            return (act && f) ? ((uint64_t)(tot + 1) << 32) : 0ull;
        };
        if (wv == 1 && nd0 > 0) keyA[1][lane] = slot_key(S, SX, wpods[0], podn(0));  // pod 0, inherited slots
        PodN pnx = podn(1);  // pod i+1's record at step i
        auto apply = [&](const ResPub &pv, int pp, const PodT<F> &pprev) {
            if (pv.ks == 0) return;
            if (pv.slot >= 0) {
                if (lane == pv.slot) reserve(S, SX, pprev, +1);
            } else {
                if ((uint32_t)lane == pv.nd_old) {
                    S = stage[pp][pv.src];
                    if (NORM) {
                        SX = stagexN[pp][pv.src];
                    } else if (F & kFeatExt) {
                        const int4 e = stagex[pp][pv.src];
                        SX.ae0 = e.x; SX.re0 = e.y; SX.ae1 = e.z; SX.re1 = e.w;
                    }
                    reserve(S, SX, pprev, +1);
                }
                ++nd;
            }
        };
        __syncthreads();
        bool stopped = false;
        PodT<F> pprev = wpods[0], pcur = wpods[0];  // pods i-1 and i (pod i+1's record is read each step)
        for (uint32_t i = 0; i < kend; ++i) {
            QS_DIAG_BEGIN()
            const int par = i & 1, pp = par ^ 1;
            const ResPub pv = read_pub(&pub[pp]);
            const PodT<F> pn1 = wpods[min(i + 1, kend - 1)];  // (K may be 64: stay inside the array)
            __builtin_amdgcn_sched_barrier(0);  // both LDS reads go out before the pub's wait
            if (NORM && pv.slot == -2) { stopped = true; break; }  // D stopped at pod i-1
            if (i > 0) apply(pv, pp, pprev);
            if (DIAG) { const uint64_t t_ = diag_stamp(); dpart += t_ - tprev; }
            if (i + 1 < kend) {
                const PodN pnc = pnx;
                if (NORM) pnx = podn(i + 2);  // next step's record: its LDS reads overlap this score
                RowT<F> s2 = S;
                RowX x2s = SX;
                if (wv == 2) reserve(s2, x2s, pcur, +1);
                // score half only: wave D owns the slot -> node map and fills the index half
                (wv == 1 ? keyA : keyB)[par][lane] = slot_key(s2, x2s, pn1, pnc);
            }
            pprev = pcur;
            pcur = pn1;
            QS_DIAG_END()
            __syncthreads();
        }
        // (a stop at the last pod publishes STOP, which apply() ignores: ks == 0)
        if (wv == 1 && !stopped) apply(read_pub(&pub[(kend - 1) & 1]), (kend - 1) & 1, wpods[kend - 1]);
        __syncthreads();  // slotnode written by wave D
        if (wv == 1 && (uint32_t)lane < nd) {
            const uint32_t node = slotnode[lane];
            store_dyn<F>(t, node, S);
            store_dynx<F>(t, node, SX);
        }
    } else {
        // ---- C: candidate rows, C keys, next pod's top-2 ------------------------------------
        auto top2 = [&](const uint64_t(&e)[EPL], uint64_t &a, uint64_t &b) {
            uint32_t word[EPL];
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                const uint32_t nidx = e[m] ? key_node(e[m]) : 0u;
                word[m] = dirty[nidx >> 5] >> (nidx & 31);
            }
            a = 0;
            b = 0;
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                const uint64_t x = (word[m] & 1u) ? 0ull : e[m];
                const bool gt = x > a;
                b = gt ? a : (x > b ? x : b);
                a = gt ? x : a;
            }
        };
        auto load_ent = [&](uint64_t(&e)[EPL], uint32_t pod) {
#pragma unroll
            for (int m = 0; m < EPL; ++m) e[m] = pod < kend ? list_ent(lists, pod, GLp, lr, sh, m, lane) : 0ull;
        };
        uint64_t c1, c2;
        uint64_t eX[EPL], eY[EPL];  // ping-pong: entries consumed two pods after their load
        {
            uint64_t e0[EPL];
            load_ent(e0, 0);
            top2(e0, c1, c2);
        }
        load_ent(eX, 1);
        load_ent(eY, 2);
        // EPL == 1 (merged lists): a lane holds one entry, so its second candidate is always empty
        constexpr bool TWO = EPL > 1;
        C1[1][lane] = c1;
        if (TWO) C2[1][lane] = c2;
        RowT<F> r1 = load_row<F>(t, c1 ? key_node(c1) : 0u), r2 = TWO ? load_row<F>(t, c2 ? key_node(c2) : 0u) : empty_row<F>();
        RowX x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u), x2 = TWO ? load_rowx<F>(t, c2 ? key_node(c2) : 0u) : RowX{};
        __syncthreads();
        PodT<F> pcurC = wpods[0];  // (EPL == 1 path) pod i's record, carried
        auto step = [&](uint32_t i, uint64_t(&en)[EPL]) -> bool {
            QS_DIAG_BEGIN()
            const int par = i & 1, pp = par ^ 1;
            if constexpr (EPL == 1) {
                // one entry per lane (merged lists): the step's LDS reads go out together (the
                // pub, the dirty word of pod i+1's entry through pod i-2 — pod i-1's winner is
                // masked by compare — and pod i+1's records), and the candidate's score, which
                // needs no pub, is computed while they land
                const ResPub pv = read_pub(&pub[pp]);
                const uint32_t en_node = en[0] ? key_node(en[0]) : 0u;
                const uint32_t dword = dirty[en_node >> 5];
                const uint32_t kn = min(i + 1, kend - 1);
                const PodT<F> pn1 = wpods[kn];
                DPodX qx{};
                NormInfo nf{0, 0, 0, 0};
                double2 yr = make_double2(0.0, 0.0);
                if (NORM) { qx = wpodx[kn]; nf = wnorm[kn]; yr = wrcp[kn]; }
                __builtin_amdgcn_sched_barrier(0);
                RowT<F> cr = r1;
                RowX crx = x1;
                reserve(cr, crx, pcurC, +1);
                const bool f = feasible<F>(cr, crx, pn1, NORM ? qx : px);
                const uint32_t tot = node_total<F>(cr, crx, pn1, NORM ? qx : px, cv, nf.mt, yr.x, nf.ma, yr.y, nullptr);
                uint32_t fl = 0;
                if (NORM && !f) {
                    if (F & kFeatTaint) fl |= taint_raw(crx, qx) == nf.mt ? 1u : 0u;
                    if (F & kFeatAffinity) fl |= affinity_raw(crx, pn1, qx) == nf.ma ? 2u : 0u;
                }
                if (NORM && pv.slot == -2) return false;  // D stopped at pod i-1
                stage[par][lane] = r1;
                if (NORM) stagexN[par][lane] = x1;
                else if (F & kFeatExt) stagex[par][lane] = make_int4(x1.ae0, x1.re0, x1.ae1, x1.re1);
                const bool use2 = pv.ks != 0 && c1 != 0 && key_node(c1) == pv.w;
                const uint64_t cc = use2 ? 0ull : c1;
                if (i + 1 < kend) {
                    keyC[par][lane] = (cc != 0 && f) ? pack_key(tot + 1, key_node(cc)) : 0ull;
                    if (NORM) flagC[par][lane] = fl;
                    const bool dirt = ((dword >> (en_node & 31)) & 1u) != 0 || (pv.ks != 0 && en_node == pv.w);
                    c1 = (en[0] != 0 && !dirt) ? en[0] : 0ull;  // pod i+1 against the dirty set through pod i-1
                    C1[par][lane] = c1;
                    r1 = load_row<F>(t, c1 ? key_node(c1) : 0u);
                    x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u);
                    load_ent(en, i + 3);
                }
                pcurC = pn1;
                if (lane == 0 && pv.ks != 0 && pv.slot < 0)  // (read by the next step's dirty word)
                    __hip_atomic_fetch_or(&dirty[pv.w >> 5], 1u << (pv.w & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                QS_DIAG_END()
                __syncthreads();
                return true;
            }
            const ResPub pv = read_pub(&pub[pp]);
            if (NORM && pv.slot == -2) return false;  // D stopped at pod i-1
            if (lane == 0 && pv.ks != 0 && pv.slot < 0)
                __hip_atomic_fetch_or(&dirty[pv.w >> 5], 1u << (pv.w & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_or: no round trip
            const bool use2 = pv.ks != 0 && c1 != 0 && key_node(c1) == pv.w;
            const uint64_t cc = use2 ? c2 : c1;
            uint64_t tw0 = 0;
            if (DIAG) tw0 = diag_stamp();
            const RowT<F> crow = sel_row(use2, r2, r1);
            const RowX cx = sel_rowx(use2, x2, x1);
            stage[par][lane] = crow;
            if (NORM) stagexN[par][lane] = cx;
            else if (F & kFeatExt) stagex[par][lane] = make_int4(cx.ae0, cx.re0, cx.ae1, cx.re1);
            if (DIAG) { const uint64_t t_ = diag_stamp(); dwait += t_ - tw0; }
            if (i + 1 < kend) {
                const PodT<F> p = wpods[i], pn1 = wpods[i + 1];
                top2(en, c1, c2);  // pod i+1 against the dirty set through pod i-1
                C1[par][lane] = c1;
                if (TWO) C2[par][lane] = c2;
                r1 = load_row<F>(t, c1 ? key_node(c1) : 0u);
                x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u);
                if (TWO) {
                    r2 = load_row<F>(t, c2 ? key_node(c2) : 0u);
                    x2 = load_rowx<F>(t, c2 ? key_node(c2) : 0u);
                }
                load_ent(en, i + 3);
                if (DIAG) { const uint64_t t_ = diag_stamp(); dpart += t_ - tprev; }
                RowT<F> cr = crow;
                RowX crx = cx;
                reserve(cr, crx, p, +1);
                if (NORM) {
                    const DPodX &qx = wpodx[i + 1];
                    const NormInfo nf = wnorm[i + 1];
                    const double2 yr = wrcp[i + 1];
                    const bool f = feasible<F>(cr, crx, pn1, qx);
                    const uint32_t tot = node_total<F>(cr, crx, pn1, qx, cv, nf.mt, yr.x, nf.ma, yr.y, nullptr);
                    keyC[par][lane] = (cc != 0 && f) ? pack_key(tot + 1, key_node(cc)) : 0ull;
                    uint32_t fl = 0;
                    if (!f) {
                        if (F & kFeatTaint) fl |= taint_raw(crx, qx) == nf.mt ? 1u : 0u;
                        if (F & kFeatAffinity) fl |= affinity_raw(crx, pn1, qx) == nf.ma ? 2u : 0u;
                    }
                    flagC[par][lane] = fl;
                } else {
                    const bool f = feasible<F>(cr, crx, pn1, px);
                    const uint32_t tot = node_total<F>(cr, crx, pn1, px, cv, 0, 0.0, 0, 0.0, nullptr);
                    keyC[par][lane] = (cc != 0 && f) ? pack_key(tot + 1, key_node(cc)) : 0ull;
                }
            }
            QS_DIAG_END()
            __syncthreads();
            return true;
        };
        uint32_t i = 0;
        for (; i + 1 < kend; i += 2) {
            if (!step(i, eX) || !step(i + 1, eY)) { i = kend; break; }
        }
        if (i < kend) step(i, eX);
        __syncthreads();
    }
    if (DIAG && lane == 0) {
        atomicAdd((unsigned long long *)&diag[wv], (unsigned long long)dsum);
        if (wv == 0) atomicAdd((unsigned long long *)&diag[5], (unsigned long long)kend);
        if (wv == 1) atomicAdd((unsigned long long *)&diag[6], (unsigned long long)dpart);
        if (wv == 3) atomicAdd((unsigned long long *)&diag[7], (unsigned long long)dpart);
        if (wv == 3) atomicAdd((unsigned long long *)&diag[4], (unsigned long long)dwait);
        if (wv == 0) atomicAdd((unsigned long long *)&diag[9], (unsigned long long)(diag_stamp() - t_loop));
    }
    if (wv == 0) __syncthreads();  // pairs with the post-loop barrier of waves A/B and C
#undef QS_DIAG_BEGIN
#undef QS_DIAG_END
}

template <uint32_t F, int EPL, bool DIAG, bool K32>
__global__ __launch_bounds__(256) void k_la_resolve4(DevTable t, const PodT<F> *__restrict__ pods,
                                                     DevCfg c, uint32_t s0, uint32_t P,
                                                     uint32_t K, uint32_t GLp, uint32_t lr,
                                                     LaShard sh,
                                                     const uint64_t *__restrict__ lists,
                                                     int32_t *__restrict__ out_node,
                                                     uint64_t *__restrict__ out_key,
                                                     uint64_t *__restrict__ stamps,
                                                     uint64_t *__restrict__ diag,
                                                     const uint32_t *__restrict__ dprev,
                                                     uint32_t *__restrict__ dcur,
                                                     const DPodX *__restrict__ podx,
                                                     const NormInfo *__restrict__ norm,
                                                     uint32_t *__restrict__ rec,
                                                     unsigned long long *nfall) {
    wait_lists_ready(c, s0, K);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    la_resolve4_block<F, EPL, DIAG, K32>(lds, t, pods, c, s0, P, K, GLp, lr, sh, lists, out_node, out_key,
                                         stamps, diag, dprev, dcur, podx, norm, rec);
    if constexpr ((F & kFeatNorm) != 0) {
        // a window that stopped on a lost maximum resumes here (no second launch per window): the
        // stop record wave D just wrote decides, after the barrier, in every wave alike
        if (rec) {
            __syncthreads();
            la_resolve_norm_body<F, 1>(lds, t, pods, podx, c, s0, P, K, GLp, lr, sh, lists, norm, out_node, out_key,
                                       stamps, dprev, dcur, nfall, rec);
        }
    }
}

// =============================================================================================
// Resident lookahead stream: the whole window sequence of an unsharded,
// non-normalizing stream in ONE launch.  Block 0 runs the four-wave resolver (la_resolve4_block)
// over every window; blocks 1..S are selectors that loop over each window's (pod, chunk) tasks and
// merge a pod's chunk lists in whichever selector delivers its last chunk.  Nothing per window goes
// through the host, an event, a kernel boundary or a cache write-back / invalidate: the three
// in-launch hand-offs use the form MI355X_MICROARCH.md § inter-workgroup visibility lists as valid
// (row 1: every handed-off byte stored write-through `sc1`, every storing wave drained, a workgroup
// barrier, ONE lane signals with an agent-scope atomic; the consumer polls relaxed and reads every
// handed-off byte with `sc1` loads):
//   resolver -> selectors   dynamic row quads of window w's slots (16-B sc1)   done = w + 1
//   selector -> merger      the chunk's top-L list (8-B sc1)                    ticket[w&1][k] += 1
//   merger   -> resolver    the pod's sorted final list (8-B sc1)               rdy[w&1] += 1
// Selects of window w read the table as it stood after window w-2 (overlapped windows, §4.1 item
// 4), so a selector waits for done >= w-1; lists, chunk lists and tickets are double-buffered by
// window parity and window w+2 reuses them only after done >= w+1.  Every wait is bounded: on a
// timeout the waiter raises werr, every other wait gives up when it sees werr, and the host voids
// the run (QS_ETIMEOUT).  Placements are those of the launched windows (same kernels' arithmetic).
// =============================================================================================
// Workgroup size of the resident stream: selectors score with eight waves; the resolver workgroup
// runs its four pipeline waves and parks the other four at the same barriers.
constexpr int kResBS = 512;
struct ResCtl {                // zeroed before every launch; each counter on its own 128-B line
    uint32_t done, pad0[31];   // windows resolved
    uint32_t rdy[2][32];       // pods merged, per window parity
    uint32_t ticket[2][64];    // chunk lists delivered, per window parity and window pod
    uint32_t nticket[2][64];   // normalizing profiles: chunk partial maxima published, likewise
};
// Bounded relaxed poll by one lane: true once *p >= want; false on werr or after `ticks` (100 MHz;
// 0.5 s, or DevCfg::first_ticks in a run's first window).
constexpr uint64_t kResWaitTicks = 50000000ull;
__device__ __forceinline__ uint64_t res_bound(const DevCfg &c, uint32_t w) {
    return (w == 0 && c.first_ticks) ? c.first_ticks : kResWaitTicks;
}
__device__ __forceinline__ bool res_wait_ge(const uint32_t *p, uint32_t want, uint32_t *werr,
                                            uint64_t ticks = kResWaitTicks) {
    if (load_coh_u32(p) >= want) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // one sc1 load per round on the polled word (a round trip to the Infinity Cache): the error word
    // and the clock only every 16th round, so a waiter sees its signal one round trip after it lands
    for (uint32_t it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (load_coh_u32(p) >= want) return true;
        if ((it & 15u) == 0u) {
            if (load_coh_u32(werr) != 0u) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                __hip_atomic_store((gu32 *)werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
}
__device__ __forceinline__ uint32_t res_add(uint32_t *p) {
    return __hip_atomic_fetch_add((gu32 *)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wave 0 sorts a pod's list (LDS, L <= 64 entries) best-first into its final slot; then the block
// signals the resolver (every storing wave drained, barrier, one lane adds).
__device__ __forceinline__ uint32_t res_publish_list(const uint64_t *lbuf, uint32_t L, uint64_t *out, uint32_t *rdy) {
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        uint64_t v = (uint32_t)lane < L ? lbuf[lane] : 0ull;
        v = wave_sort_desc(v, lane);
        if ((uint32_t)lane < L) store_coh_u64(out + lane, v);
        drain_stores();
    }
    __syncthreads();
    return threadIdx.x == 0 ? res_add(rdy) : 0u;  // (thread 0: the count before this list)
}
// Normalizing profiles: the same, plus the static parts (static_raw) of the pod's sorted entries
// against the next two stream pods, sout[0][lane] vs pod s + 1 and sout[1][lane] vs pod s + 2 (the
// resolver's wave C scores a candidate entry for the next pod, waves A/B a new slot taken from it
// for the pod after that).  Waves 0 and 1, one pod each; published before the list's signal.
template <class PodRec>
__device__ __forceinline__ uint32_t res_publish_list_norm(uint64_t *lbuf, uint32_t L, uint64_t *out, uint32_t *rdy,
                                                      const DevTable &t, const PodRec *__restrict__ pods,
                                                      const DPodX *__restrict__ podx, uint32_t s, uint32_t P,
                                                      uint32_t *sout) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (wv == 0) {
        uint64_t v = (uint32_t)lane < L ? lbuf[lane] : 0ull;
        v = wave_sort_desc(v, lane);
        if ((uint32_t)lane < L) store_coh_u64(out + lane, v);
        lbuf[lane] = v;
    }
    __syncthreads();
    if (wv < 2) {
        const uint32_t q = min(s + 1 + (uint32_t)wv, P - 1);
        const uint64_t v = lbuf[lane];
        const DMask m = t.masks[v ? key_node(v) : 0u];
        const DPodX px = load_vgpr(podx + q);
        const uint32_t st = static_raw(m.th, m.ts, m.lb0, m.lb1, pods[q].flags, px);
        __hip_atomic_store((gu32 *)(sout + wv * 64 + lane), st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    drain_stores();
    __syncthreads();
    return threadIdx.x == 0 ? res_add(rdy) : 0u;
}

// Sharded resident stream: the block holding rank `rank`'s shard list of window
// pod k (lbuf, L keys, node-index order among equal totals) writes it into EVERY rank's mailbox
// (lists[w % 4][k][rank], system-scope stores over xGMI) and raises flags[w % 4][k][rank] = seq << 32
// | w + 1 there with a system-scope release after a system fence; then waits (bounded) until all W
// ranks' flags for pod k have arrived in its own mailbox and reduces the W * L keys, rank-major (so
// equal totals stay in node-index order), to the pod's top-L in lbuf.  Before its first remote
// write of a run a block waits for every rank's hello (posted by each rank's resolver block at
// launch start): a peer still finishing its previous run could otherwise see its slots reused.
// Slot w % 4 is safe to reuse: a rank writes window w only after resolving window w - 2, which took
// every rank's lists of window w - 2, produced after those ranks resolved window w - 4, whose
// cross merges read slot (w - 4) % 4.  Returns false on a timeout (werr raised).
__device__ __forceinline__ bool res_cross_merge(uint64_t *lbuf, uint32_t L, uint32_t k, uint32_t w,
                                                const ResShard &rsh, bool &hello_ok, uint32_t &okflag,
                                                uint32_t *werr, uint64_t first_ticks) {
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t W = rsh.W;
    const uint64_t tag = (rsh.seq << 32) | (uint64_t)(w + 1);
    const size_t cell = ((size_t)(w & 3) * 32 + k) * 16;  // [slot][pod][rank] index base
    // the hello and window 0's flags may wait for a peer still in host-side prepare: first_ticks
    const uint64_t bound = (w == 0 || !hello_ok) && first_ticks ? first_ticks : kResWaitTicks;
    auto sys_poll = [&](const uint64_t *p, uint64_t want) -> bool {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (load_coh_u32(werr) != 0u) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {
                __hip_atomic_store((gu32 *)werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        return true;
    };
    const char *own = rsh.peers[rsh.rank];
    if (!hello_ok) {
        if (tid == 0) {
            bool ok = true;
            for (uint32_t r = 0; r < W && ok; ++r)
                ok = sys_poll(reinterpret_cast<const uint64_t *>(own + rsh.hello) + r, rsh.seq);
            okflag = ok ? 1u : 0u;
        }
        __syncthreads();
        if (!okflag) return false;
        hello_ok = true;
    }
    if (tid < 64) {
        for (uint32_t r = 0; r < W; ++r) {
            uint64_t *dst = reinterpret_cast<uint64_t *>(rsh.peers[r] + rsh.lists) + (cell + rsh.rank) * 64;
            if ((uint32_t)lane < L)
                __hip_atomic_store(dst + lane, lbuf[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __threadfence_system();
        if (lane == 0)
            for (uint32_t r = 0; r < W; ++r)
                __hip_atomic_store(reinterpret_cast<uint64_t *>(rsh.peers[r] + rsh.flags) + cell + rsh.rank, tag,
                                   __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (tid == 0) {
        bool ok = true;
        for (uint32_t r = 0; r < W && ok; ++r) ok = sys_poll(reinterpret_cast<const uint64_t *>(own + rsh.flags) + cell + r, tag);
        // a flag beyond this window's tag means a peer already reused the slot (the reuse argument
        // above broken): fail the run loudly instead of merging a newer window's keys
        for (uint32_t r = 0; r < W && ok; ++r)
            ok = __hip_atomic_load(reinterpret_cast<const uint64_t *>(own + rsh.flags) + cell + r, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM) == tag;
        if (!ok) __hip_atomic_store((gu32 *)werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        okflag = ok ? 1u : 0u;
    }
    __syncthreads();  // every wave is past its lbuf reads; the flags have been seen
    if (!okflag) return false;
    const uint32_t M = W * L;  // <= 512 = one key per thread, rank-major positions
    const uint32_t pos = (uint32_t)tid;
    uint64_t e[1];
    uint32_t te[1];
    e[0] = pos < M ? __hip_atomic_load(reinterpret_cast<const uint64_t *>(own + rsh.lists) + (cell + pos / L) * 64 + pos % L,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                   : 0ull;
    te[0] = (uint32_t)(e[0] >> 32);
    block_topl<kResBS, 1>(te, L, lbuf, [&](int) { return e[0]; });
    __syncthreads();  // lbuf complete
    return true;
}

// Sharded normalizing profiles: this rank's partial maxima of window pod k (over its node range,
// combined from its G chunk partials) go to EVERY rank's mailbox (norm[w % 4][k][rank], system-scope
// stores, then a system fence and the tagged flag nflags[w % 4][k][rank] = seq << 32 | w + 1), sent by
// the pod's chunk-0 task; every chunk task of the pod then waits (bounded) for all W ranks' flags in
// its own mailbox and combines the W partials into the pod's global NormInfo (max, and the counts of
// the ranks attaining it: the order does not matter).  Slot reuse as for the lists (res_cross_merge):
// a rank writes window w after resolving w - 2, which needed every rank's lists of w - 2, produced
// after every chunk task of those ranks had left window w - 4.  Both 64-bit payload words carry the
// window (w + 1 in their high half, mt << 24 | ct and ma << 22 | ca in the low), and a reader accepts a
// partial only when its flag equals this window's tag and both words carry this window; anything
// newer means the slot was reused early, and the run fails (werr) instead of combining it (ADVICE
// r4).  Thread 0 only; false on a timeout or a mismatch.
__device__ __forceinline__ bool res_norm_exchange(const NormInfo &part, uint32_t k, uint32_t w, uint32_t g,
                                                  const ResShard &rsh, bool &hello_ok, NormInfo &out,
                                                  uint32_t *werr, uint64_t first_ticks) {
    const uint32_t W = rsh.W;
    const uint64_t tag = (rsh.seq << 32) | (uint64_t)(w + 1);
    const size_t cell = ((size_t)(w & 3) * 32 + k) * 16;  // [slot][pod][rank] index base
    const uint64_t bound = (w == 0 || !hello_ok) && first_ticks ? first_ticks : kResWaitTicks;
    auto sys_poll = [&](const uint64_t *p, uint64_t want) -> bool {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (load_coh_u32(werr) != 0u) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {
                __hip_atomic_store((gu32 *)werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        return true;
    };
    const char *own = rsh.peers[rsh.rank];
    if (!hello_ok) {
        for (uint32_t r = 0; r < W; ++r)
            if (!sys_poll(reinterpret_cast<const uint64_t *>(own + rsh.hello) + r, rsh.seq)) return false;
        hello_ok = true;
    }
    if (g == 0) {
        // mt <= 64 (a popcount), ma <= 400 (four preferred weights <= 100), counts < 2^22 nodes
        const uint64_t wt = (uint64_t)(w + 1) << 32;
        const uint64_t lo = wt | (uint64_t)part.mt << 24 | part.ct, hi = wt | (uint64_t)part.ma << 22 | part.ca;
        for (uint32_t r = 0; r < W; ++r) {
            uint64_t *dst = reinterpret_cast<uint64_t *>(rsh.peers[r] + rsh.norm) + 2 * (cell + rsh.rank);
            __hip_atomic_store(dst, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(dst + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __threadfence_system();
        for (uint32_t r = 0; r < W; ++r)
            __hip_atomic_store(reinterpret_cast<uint64_t *>(rsh.peers[r] + rsh.nflags) + cell + rsh.rank, tag,
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    NormInfo nf{0, 0, 0, 0};
    for (uint32_t r = 0; r < W; ++r) {
        if (!sys_poll(reinterpret_cast<const uint64_t *>(own + rsh.nflags) + cell + r, tag)) return false;
        const uint64_t *src = reinterpret_cast<const uint64_t *>(own + rsh.norm) + 2 * (cell + r);
        const uint64_t lo = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t hi = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t f = __hip_atomic_load(reinterpret_cast<const uint64_t *>(own + rsh.nflags) + cell + r,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (f != tag || (uint32_t)(lo >> 32) != w + 1 || (uint32_t)(hi >> 32) != w + 1) {
            __hip_atomic_store((gu32 *)werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        const uint32_t qx = (uint32_t)(lo >> 24) & 0xFFu, qy = (uint32_t)lo & 0xFFFFFFu;
        const uint32_t qz = (uint32_t)(hi >> 22) & 0x3FFu, qw = (uint32_t)hi & 0x3FFFFFu;
        if (qx > nf.mt) { nf.mt = qx; nf.ct = 0; }
        if (qx == nf.mt) nf.ct += qy;
        if (qz > nf.ma) { nf.ma = qz; nf.ca = 0; }
        if (qz == nf.ma) nf.ca += qw;
    }
    out = nf;
    return true;
}

// Normalizing profiles (TaintToleration / NodeAffinity): a task first scores everything but the
// normalized parts and the chunk's partial maxima {mt, ct, ma, ca} over its feasible nodes,
// publishes the partial (sc1, ticket nticket[w&1][k]), waits until all G chunks of its pod have
// published (every task has its own workgroup, so they all run at once), combines them into the
// pod's NormInfo and only then finishes the totals and its top-L.  The merger publishes the
// NormInfo with the pod's list, for the resolver's lost-maximum test.
template <int E, int E2, uint32_t F>
__device__ __forceinline__ void res_selector(const DevTable &t, const PodT<F> *__restrict__ pods, const DevCfg &c,
                                             uint32_t P, uint32_t K, uint32_t G, uint32_t L, uint32_t chunk,
                                             uint32_t nwin, uint64_t *lists0, uint64_t *clists0, uint32_t lwords,
                                             uint32_t cwords, ResCtl *ctl, uint32_t sid, uint32_t S,
                                             uint64_t *rdiag, const DPodX *__restrict__ podx, uint4 *npart0,
                                             NormInfo *norm0, uint32_t *stat0, const ResShard &rsh) {
    constexpr bool NORM = (F & kFeatNorm) != 0;
    // sharded (rsh.W > 1): this rank's node range; the chunks tile it
    const uint32_t lo = (uint32_t)((uint64_t)rsh.rank * t.n / rsh.W);
    const uint32_t hi = (uint32_t)((uint64_t)(rsh.rank + 1) * t.n / rsh.W);
    bool hello_ok = rsh.W == 1;
    // rdiag (QS_RES_DIAG=1): summed s_memrealtime ticks of the selectors' phases, [16] scoring,
    // [17] chunk top-L, [18] publish / merge, [19] tasks, [20] merges
    uint64_t ts0 = 0, ts1 = 0, ts2 = 0, dsc = 0, dtl = 0, dpm = 0, ntask = 0, nmerge = 0;
    // QS_RES_DIAG: selector 0 — `done` seen / its task finished, after the resolver's window start
    uint64_t tdone_ = 0, wstart_ = 0, seen_ = 0, fin_ = 0, nwt_ = 0, lastp_ = 0, nlast_ = 0, late13_ = 0, late15_ = 0;
    __shared__ uint64_t lbuf[64];
    __shared__ uint32_t okflag_[4];  // (16 B: keeps the dynamic-LDS base 16-byte aligned)
    __shared__ uint32_t nred[4][8];  // NORM: per-wave partial maxima and counts
    uint32_t &okflag = okflag_[0];
    const int tid = threadIdx.x, lane = tid & 63, w8 = tid >> 6;
    const __amdgpu_buffer_rsrc_t rs = row_rsrc<F>(t);
    DevCfg cv = c;  // (weights in VGPRs, as in la_resolve4_stream)
    asm volatile("" : "+v"(cv.yd_both), "+v"(cv.yd_c), "+v"(cv.yd_m), "+v"(cv.wc), "+v"(cv.wm));
    for (uint32_t w = 0; w < nwin; ++w) {
        const uint32_t s0 = w * K, kw = min(K, P - s0), b = w & 1;
        if (sid >= kw * G) continue;  // no task of this window (uniform per block)
        // large chunks (E = 7, 8; Fit + Balanced: config 3's 50,000 nodes, selector-bound): this workgroup's first
        // task's pod record is read before the wait for the table (pod records never change during
        // a stream), so its latency hides behind the wait (config 3 652-657 -> 647 ms; with the small
        // chunks of config 2, whose selectors wait on the resolver anyway, the same code cost 2 %)
        static_assert(sizeof(PodT<F>) % 16 == 0, "pod record in 16-byte words");
        constexpr int PW = (int)(sizeof(PodT<F>) / 16);
        constexpr bool kPodPre = (F & kFeatNorm) == 0 && E >= 7 && E <= 8;  // (registers: not at 16)
        u32x4 pq[PW];
        if constexpr (kPodPre) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(pods + s0 + min(sid / G, kw - 1));
#pragma unroll
            for (int q = 0; q < PW; ++q) pq[q] = src[q];
#pragma unroll
            for (int q = 0; q < PW; ++q) asm volatile("" : "+v"(pq[q]));
        }
        if (w >= 2) {  // the table after window w-2, and this parity's buffers free again
            if (tid == 0) okflag = res_wait_ge(&ctl->done, w - 1, c.werr) ? 1u : 0u;
            if (rdiag && tid == 0) {  // (the resolver posts each window's start time)
                tdone_ = __builtin_amdgcn_s_memrealtime();
                wstart_ = load_coh_u64(&rdiag[15]);
            }
            __syncthreads();
            if (!okflag) return;
        }
        uint64_t *lists = lists0 + (size_t)b * lwords;
        uint64_t *clists = clists0 + (size_t)b * cwords;
        for (uint32_t task = sid; task < kw * G; task += S) {
            if (c.inject == 1u && w == 3 && task == 0) continue;  // test hook: window 3 never completes
            if (c.inject == 2u && w >= 40 && w < 44) {  // test hook: this rank's selectors run 3 ms late
                if (tid == 0) {
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    while (__builtin_amdgcn_s_memrealtime() - t0 < 300000ull) __builtin_amdgcn_s_sleep(10);
                }
                __syncthreads();
            }
            const uint32_t k = task / G, g = task % G;
            if (rdiag && c.sel_diag) ts0 = __builtin_amdgcn_s_memrealtime();
            PodT<F> p;
            if (kPodPre && task == sid) __builtin_memcpy(&p, pq, sizeof p);
            else p = pods[s0 + k];
            const uint32_t start = lo + g * chunk, end = min(hi, start + chunk);
            const uint32_t base = start + (uint32_t)w8 * E * kWave + lane;
            uint32_t tv[E];
            NormInfo nf{0, 0, 0, 0};
            if constexpr (NORM) {
                const DPodX px = load_vgpr(podx + s0 + k);
                uint32_t raw[E];  // (taint raw | affinity raw << 16), 0xFFFFFFFF = infeasible / outside
                uint32_t mt = 0, ma = 0;
                if constexpr ((F & kFeatWide) == 0) {
                    // compact rows: a lane issues the loads of kSelB nodes (rows and masks) before it
                    // decodes any (one round trip per group instead of one per node), then scores them
                    // one after another
                    // (configurable scoring resources at 16 nodes per lane: two nodes per group, so the
                    // kernel stays within 256 VGPRs without spills — tests/test_kernel_resources.py)
                    constexpr int SB = ((F & kFeatRes) != 0 && E >= 16) ? 2 : kSelB;
#pragma unroll
                    for (int j0 = 0; j0 < E; j0 += SB) {
                        constexpr int B = E < SB ? E : SB;
                        RowQ q[B];
                        DMask mk[B];
#pragma unroll
                        for (int b = 0; b < B && j0 + b < E; ++b) {
                            const uint32_t idx = base + (j0 + b) * kWave;
                            q[b] = load_row_q<F>(rs, idx);
                            mk[b] = t.masks[idx < end ? idx : start];
                        }
#pragma unroll
                        for (int b = 0; b < B && j0 + b < E; ++b) {  // one node after another (bounded registers)
                            const int j = j0 + b;
                            tv[j] = 0;
                            raw[j] = 0xFFFFFFFFu;
                            if (base + j * kWave < end) {
                                RowX x;
                                const Row r = decode_row_q<F>(q[b], x);
                                x.th = mk[b].th; x.ts = mk[b].ts; x.lb0 = mk[b].lb0; x.lb1 = mk[b].lb1;
                                if (feasible<F>(r, x, p, px)) {
                                    const uint32_t rt = (F & kFeatTaint) ? taint_raw(x, px) : 0u;
                                    const uint32_t ra = (F & kFeatAffinity) ? affinity_raw(x, p, px) : 0u;
                                    raw[j] = rt | (ra << 16);
                                    mt = rt > mt ? rt : mt;
                                    ma = ra > ma ? ra : ma;
                                    tv[j] = __umul24((uint32_t)p.wfit, la_score<F>(r, x, p, cv)) +
                                            __umul24((uint32_t)p.wbal, ba_score<F>(r, x, p, cv));
                                }
                            }
                        }
                    }
                } else {
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    const uint32_t idx = base + j * kWave;
                    tv[j] = 0;
                    raw[j] = 0xFFFFFFFFu;
                    if (idx < end) {
                        RowX x;
                        const RowT<F> r = load_row_coh<F>(t, rs, idx, x);
                        const DMask m = t.masks[idx];  // static during a stream
                        x.th = m.th; x.ts = m.ts; x.lb0 = m.lb0; x.lb1 = m.lb1;
                        if (feasible<F>(r, x, p, px)) {
                            const uint32_t rt = (F & kFeatTaint) ? taint_raw(x, px) : 0u;
                            const uint32_t ra = (F & kFeatAffinity) ? affinity_raw(x, p, px) : 0u;
                            raw[j] = rt | (ra << 16);
                            mt = rt > mt ? rt : mt;
                            ma = ra > ma ? ra : ma;
                            tv[j] = __umul24((uint32_t)p.wfit, la_score<F>(r, x, p, cv)) +
                                    __umul24((uint32_t)p.wbal, ba_score<F>(r, x, p, cv));
                        }
                    }
                }
                }
                // the chunk's maxima and the counts of feasible nodes attaining them
                mt = wave_max_u32(mt);
                ma = wave_max_u32(ma);
                if (lane == 0) { nred[0][w8] = mt; nred[1][w8] = ma; }
                __syncthreads();
                mt = ma = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    mt = nred[0][i] > mt ? nred[0][i] : mt;
                    ma = nred[1][i] > ma ? nred[1][i] : ma;
                }
                uint32_t ct = 0, ca = 0;
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    ct += (uint32_t)__popcll(__ballot(raw[j] != 0xFFFFFFFFu && (raw[j] & 0xFFFFu) == mt));
                    ca += (uint32_t)__popcll(__ballot(raw[j] != 0xFFFFFFFFu && (raw[j] >> 16) == ma));
                }
                if (lane == 0) { nred[2][w8] = ct; nred[3][w8] = ca; }
                __syncthreads();
                __shared__ NormInfo nfx;  // sharded: the pod's global maxima (thread 0 -> the block)
                if (G == 1) {
                    nf = NormInfo{mt, 0, ma, 0};
#pragma unroll
                    for (int i = 0; i < 8; ++i) { nf.ct += nred[2][i]; nf.ca += nred[3][i]; }
                } else {
                    // publish this chunk's partial, then combine all G partials of the pod
                    uint4 *np = npart0 + ((size_t)b * K + k) * G;
                    if (tid == 0) {
                        uint4 o = make_uint4(mt, 0, ma, 0);
#pragma unroll
                        for (int i = 0; i < 8; ++i) { o.y += nred[2][i]; o.w += nred[3][i]; }
                        store_coh_u64(reinterpret_cast<uint64_t *>(np + g), (uint64_t)o.x | ((uint64_t)o.y << 32));
                        store_coh_u64(reinterpret_cast<uint64_t *>(np + g) + 1, (uint64_t)o.z | ((uint64_t)o.w << 32));
                        drain_stores();
                        res_add(&ctl->nticket[b][k]);
                        okflag = res_wait_ge(&ctl->nticket[b][k], ((w >> 1) + 1) * G, c.werr, res_bound(c, w)) ? 1u : 0u;
                    }
                    __syncthreads();
                    if (!okflag) return;
                    for (uint32_t gg = 0; gg < G; ++gg) {  // spec S5 maxima over the pod's feasible nodes
                        const uint64_t lo = load_coh_u64(reinterpret_cast<const uint64_t *>(np + gg));
                        const uint64_t hi = load_coh_u64(reinterpret_cast<const uint64_t *>(np + gg) + 1);
                        const uint32_t qx = (uint32_t)lo, qy = (uint32_t)(lo >> 32), qz = (uint32_t)hi,
                                       qw = (uint32_t)(hi >> 32);
                        if (qx > nf.mt) { nf.mt = qx; nf.ct = 0; }
                        if (qx == nf.mt) nf.ct += qy;
                        if (qz > nf.ma) { nf.ma = qz; nf.ca = 0; }
                        if (qz == nf.ma) nf.ca += qw;
                    }
                }
                if (rsh.W > 1) {  // nf covers this rank's node range: combine with every rank's
                    if (tid == 0) {
                        NormInfo gnf{0, 0, 0, 0};
                        okflag = res_norm_exchange(nf, k, w, g, rsh, hello_ok, gnf, c.werr, c.first_ticks) ? 1u : 0u;
                        nfx = gnf;
                    }
                    __syncthreads();
                    if (!okflag) return;
                    nf = nfx;
                    hello_ok = true;
                    __syncthreads();  // (nfx / okflag reused by the next task)
                }
                const double ymt = rcp_exact(nf.mt), yma = rcp_exact(nf.ma);
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    uint32_t tot = tv[j];
                    if (F & kFeatTaint) tot += __umul24((uint32_t)cv.wtt, tt_norm(raw[j] & 0xFFFFu, nf.mt, ymt));
                    if (F & kFeatAffinity) tot += __umul24((uint32_t)cv.wna, na_norm(raw[j] >> 16, nf.ma, yma));
                    tv[j] = raw[j] != 0xFFFFFFFFu ? tot + 1 : 0u;
                }
            } else if constexpr ((F & kFeatWide) == 0) {
                const DPodX px{};
#pragma unroll
                for (int j0 = 0; j0 < E; j0 += kSelB) {  // kSelB nodes' loads in flight, as above
                    constexpr int B = E < kSelB ? E : kSelB;
                    RowQ q[B];
#pragma unroll
                    for (int b = 0; b < B && j0 + b < E; ++b) q[b] = load_row_q<F>(rs, base + (j0 + b) * kWave);
#pragma unroll
                    for (int b = 0; b < B && j0 + b < E; ++b) {  // one node after another (bounded registers)
                        const int j = j0 + b;
                        tv[j] = 0;
                        if (base + j * kWave < end) {
                            RowX x;
                            const Row r = decode_row_q<F>(q[b], x);
                            const bool f = feasible<F>(r, x, p, px);
                            const uint32_t tot = node_total<F>(r, x, p, px, cv, 0, 0.0, 0, 0.0, nullptr);
                            tv[j] = f ? tot + 1 : 0;
                        }
                    }
                }
            } else {
                const DPodX px{};
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    const uint32_t idx = base + j * kWave;
                    tv[j] = 0;
                    if (idx < end) {
                        RowX x;
                        const RowT<F> r = load_row_coh<F>(t, rs, idx, x);
                        const bool f = feasible<F>(r, x, p, px);
                        const uint32_t tot = node_total<F>(r, x, p, px, cv, 0, 0.0, 0, 0.0, nullptr);
                        tv[j] = f ? tot + 1 : 0;
                    }
                }
            }
            if (rdiag && c.sel_diag) { __syncthreads(); ts1 = __builtin_amdgcn_s_memrealtime(); }
            block_topl<kResBS, E>(tv, L, lbuf, [&](int j) { return pack_key(tv[j], base + j * kWave); });
            __syncthreads();  // lbuf complete
            if (rdiag && c.sel_diag) ts2 = __builtin_amdgcn_s_memrealtime();
            uint64_t *out = lists + (size_t)k * 64;
            // NORM: the pod's NormInfo goes out with its list (written before the list's signal)
            auto put_norm = [&]() {
                if (NORM && tid == 0) {
                    NormInfo *no = norm0 + (size_t)b * 64 + k;
                    store_coh_u64(reinterpret_cast<uint64_t *>(no), (uint64_t)nf.mt | ((uint64_t)nf.ct << 32));
                    store_coh_u64(reinterpret_cast<uint64_t *>(no) + 1, (uint64_t)nf.ma | ((uint64_t)nf.ca << 32));
                }
            };
            // lbuf holds this rank's top-L of pod k: publish it (unsharded), or exchange it with
            // every rank and publish the top-L of the W shard lists (sharded)
            auto publish = [&]() {
                if (rsh.W > 1) {
                    if (!res_cross_merge(lbuf, L, k, w, rsh, hello_ok, okflag, c.werr, c.first_ticks)) return false;
                }
                uint32_t r0;
                if constexpr (NORM)
                    r0 = res_publish_list_norm(lbuf, L, out, &ctl->rdy[b][0], t, pods, podx, s0 + k, P,
                                               stat0 + ((size_t)b * K + k) * 128);
                else
                    r0 = res_publish_list(lbuf, L, out, &ctl->rdy[b][0]);
                if (rdiag && tid == 0 && w >= 2 && r0 + 1 == (w >> 1) * K + kw) {  // QS_RES_DIAG: the window's last list
                    const uint64_t dt_ = __builtin_amdgcn_s_memrealtime() - wstart_;
                    lastp_ += dt_;
                    ++nlast_;
                    late13_ += dt_ > 1300u;
                    late15_ += dt_ > 1500u;
                }
                return true;
            };
            if (G == 1) {
                put_norm();
                if (!publish()) return;
            } else {
                uint64_t *cl = clists + (size_t)k * G * L;
                if ((uint32_t)tid < L) store_coh_u64(cl + (size_t)g * L + tid, lbuf[tid]);
                drain_stores();
                __syncthreads();
                if (tid == 0) okflag = (res_add(&ctl->ticket[b][k]) + 1) % G == 0 ? 1u : 0u;
                __syncthreads();
                if (okflag) {  // this block delivered pod k's last chunk: merge (k_la_merge's routine)
                    const uint32_t M = G * L;
                    uint64_t e[E2];
                    uint32_t te[E2];
#pragma unroll
                    for (int j = 0; j < E2; ++j) {
                        const uint32_t pos = (uint32_t)w8 * E2 * kWave + (uint32_t)j * kWave + lane;
                        e[j] = pos < M ? load_coh_u64(cl + pos) : 0ull;
                        te[j] = (uint32_t)(e[j] >> 32);
                    }
                    __syncthreads();  // every wave is done reading lbuf
                    block_topl<kResBS, E2>(te, L, lbuf, [&](int j) { return e[j]; });
                    __syncthreads();
                    put_norm();
                    if (!publish()) return;
                    ++nmerge;
                }
            }
            __syncthreads();  // lbuf / okflag reused by the next task
            if (rdiag && c.sel_diag) {
                const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
                dsc += ts1 - ts0; dtl += ts2 - ts1; dpm += t3 - ts2; ++ntask;
            }
        }
        if (rdiag && tid == 0 && w >= 2) {  // QS_RES_DIAG: this selector's window timeline
            const uint64_t tp = __builtin_amdgcn_s_memrealtime();
            seen_ += tdone_ - wstart_;
            fin_ += tp - wstart_;
            ++nwt_;
        }
    }
    if (rdiag && sid == 0 && tid == 0) { rdiag[13] = seen_; rdiag[14] = fin_; rdiag[2] = nwt_; }
    if (rdiag && tid == 0 && sid < 64) rdiag[64 + sid] = nwt_ ? fin_ / nwt_ : 0ull;  // mean finish, per selector
    if (rdiag && tid == 0 && nlast_) {  // when each window's last list went out
        atomicAdd((unsigned long long *)&rdiag[32], (unsigned long long)lastp_);
        atomicAdd((unsigned long long *)&rdiag[33], (unsigned long long)nlast_);
        atomicAdd((unsigned long long *)&rdiag[34], (unsigned long long)late13_);
        atomicAdd((unsigned long long *)&rdiag[35], (unsigned long long)late15_);
    }
    if (rdiag && c.sel_diag && tid == 0) {
        atomicAdd((unsigned long long *)&rdiag[16], (unsigned long long)dsc);
        atomicAdd((unsigned long long *)&rdiag[17], (unsigned long long)dtl);
        atomicAdd((unsigned long long *)&rdiag[18], (unsigned long long)dpm);
        atomicAdd((unsigned long long *)&rdiag[19], (unsigned long long)ntask);
        atomicAdd((unsigned long long *)&rdiag[20], (unsigned long long)nmerge);
    }
}

// Resident four-wave resolver: la_resolve4_block's pipeline (one list entry per lane) run over every
// window of the stream without leaving the kernel.  Nothing crosses a window boundary through
// global memory: the slots won in window w (window w+1's inherited dirty set, §4.1 item 4) are
// compacted in place through LDS (rows stay on chip), dropped slots' dirty bits are cleared, wave D
// loads window w+1's pod records at the start of window w, and wave C polls window w+1's lists five
// pods before the end of window w and prefetches the entries of its first three pods and the
// candidate rows of its first pod.  Wave A stores the rows won in window w write-through and, at
// window w+1's first pod (drained there; round 6: from the third pod, so the next selections start
// two pod steps earlier: configs 2 / 3 / 4 -2 % / -5 % / -1 %), signals done = w + 1.
// Per window and wave: one prologue barrier, one barrier per pod, two boundary barriers.
//
// Normalizing profiles (NORM: TaintToleration / NodeAffinity, config 4): list keys
// and slot keys are normalized with the selection-time maxima of each pod (NormInfo, published by
// the selectors with the lists), and waves A/B/C return two "lost holder" flags per key (infeasible
// now and raw score = the maximum), which wave D counts before its argmax, exactly as
// la_resolve4_block does.  When a maximum may be lost at pod i, D publishes STOP; after that step's
// barrier ALL EIGHT waves of the workgroup (the four pipeline waves and the four that otherwise
// only keep the barrier count) rescan the table exactly for pod i (slot rows from LDS, every other
// row from HBM), D publishes the winner as an ordinary result — a new slot always with source lane 0,
// whose staged row, key and flags for pod i+1 wave C writes there — and the pipeline continues with
// pod i+1, whose precomputed keys cover every outcome of pod i.  Per window one more prologue
// barrier (B0: the window's NormInfo in LDS before wave A's first keys), four per rescan.  The four
// extra waves also stage the next window's pod extension records (176 B each) in LDS.
constexpr uint32_t kResNormK = 32;  // window pods whose NORM records are staged per parity (K <= 32)
// Fit + Balanced (+ext) profiles: stream pods whose list entries / candidate rows sit in the LDS
// rings of waves 4 (entries) and 5 (rows), indexed by stream pod modulo kResRing
constexpr uint32_t kResRing = 4;
constexpr uint32_t kResTStride = 65;
constexpr size_t kResLdsMax = 96 * 1024;
constexpr uint32_t kResSgprMax = 112;  // bound on the resident kernels' sgpr_count (checked: tools/kres.sh)  // dynamic LDS of the resident launch (gfx950: up to 160 KiB per workgroup)  // slot statics [pod][lane] rows, padded: both access patterns conflict-free
template <uint32_t F>
constexpr size_t res_stream_lds_bytes(uint32_t n) {
    size_t b = ((((size_t)n + 31) / 32 + 3) & ~(size_t)3) * 4 + 4 * 2 * 64 * 8 + 2 * 64 * (sizeof(RowT<F>) + sizeof(int4)) +
               2 * sizeof(ResPub) + 3 * 64 * 4 + 64 * (sizeof(RowT<F>) + sizeof(int4)) + 2 * 64 * sizeof(PodT<F>);
    if ((F & kFeatNorm) == 0)  // the entry / candidate-row rings (kResRing pods) and the late flag
        b += kResRing * 64 * (8 + sizeof(RowT<F>) + sizeof(int4)) + 16;
    if ((F & kFeatNorm) != 0)
        b += 2 * kResNormK * (sizeof(DPodX) + sizeof(NormInfo) + sizeof(double2)) + 2 * 64 * sizeof(RowX) +
             64 * sizeof(RowX) + 64 * (sizeof(RowT<F>) + sizeof(RowX)) + 2 * 64 * 4 + 64 * 4 + 16 * 4 + 8 * 8 + 16 +
             2 * kResNormK * kResTStride * 4 + 2 * 64 * 4 + 2 * kResNormK * 4 + 64 * sizeof(DMask);
    return b;
}
// QS_RES_DIAG_BLOCK build (experiments): per-role busy shader cycles per pod step, barrier exit
// to barrier entry, into rdiag[8 + role] (D, A, B, C) with the step count in rdiag[12].
#ifdef QS_RES_DIAG_BLOCK
constexpr bool kResDiag = true;
#else
constexpr bool kResDiag = false;
#endif
#define QS_RSTAMP_BEGIN() if (kResDiag && rdiag) ts_ = diag_stamp();
#define QS_RSTAMP_END() if (kResDiag && rdiag) busy_ += diag_stamp() - ts_;
// cycles from the step's start to point k of a role's step (rdiag[21 + k], summed)
#define QS_RSTAMP_MARK(k) if (kResDiag && rdiag) sub_[k] += diag_stamp() - ts_;
// NORM: exact rescan of one window pod p at the current state by the resident resolver
// workgroup's four parked waves (4-7; wave D has staged its slot nodes in sidx / snd and wave A the
// slot rows in srow / sxr before R1).  Rows of dirty nodes come from the slots, every other row
// from HBM, where it is current (only slots change during a window).  Returns the pod's packed key
// (0 = unschedulable); red_k[0..3] hold the four waves' partial keys after R3, which is how the
// pipeline waves (res_rescan_wait: the same three barriers) read it.  Only the parked waves run it:
// inlined into the pipeline roles, its row batches pushed their hot loops into scratch.
template <uint32_t F>
__device__ __forceinline__ uint64_t res_rescan_pass(const DevTable &t, const PodT<F> &p, const DPodX &pxi,
                                                    const uint32_t *dirty, const uint32_t *sidx, const RowT<F> *srow,
                                                    const RowX *sxr, const DMask *smask, uint32_t *red_m,
                                                    uint64_t *red_k, const uint32_t *snd, const DevCfg &cv) {
    __syncthreads();  // R1: slots staged
    const int lane = threadIdx.x & 63;
    const uint32_t wid = (threadIdx.x >> 6) - 4;
    const uint32_t n = t.n, nds = *snd;
    constexpr uint32_t U = 2;  // (rows per lane in flight: 4 put the normalizing kernels over 256 VGPRs)
    auto rows_at = [&](uint32_t b0, RowT<F>(&r)[U], RowX(&x)[U]) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t idx = b0 + 64 * u < n ? b0 + 64 * u : 0u;
            r[u] = load_row<F>(t, idx);
            x[u] = load_rowx<F>(t, idx);
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t idx = b0 + 64 * u;
            if (idx < n && ((dirty[idx >> 5] >> (idx & 31)) & 1u)) {
                uint32_t j = 0;
                while (j + 1 < nds && sidx[j] != idx) ++j;  // dirty <=> held by a slot
                r[u] = srow[j];
                x[u] = sxr[j];
                const DMask m = smask[j];
                x[u].th = m.th; x[u].ts = m.ts; x[u].lb0 = m.lb0; x[u].lb1 = m.lb1;
            }
        }
    };
    uint32_t mt = 0, ma = 0;
    for (uint32_t b0 = wid * 64 * U + lane; b0 < n; b0 += 4 * 64 * U) {
        RowT<F> r[U];
        RowX x[U];
        rows_at(b0, r, x);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (b0 + 64 * u < n && feasible<F>(r[u], x[u], p, pxi)) {
                const uint32_t a = (F & kFeatTaint) ? taint_raw(x[u], pxi) : 0u;
                const uint32_t b2 = (F & kFeatAffinity) ? affinity_raw(x[u], p, pxi) : 0u;
                mt = a > mt ? a : mt;
                ma = b2 > ma ? b2 : ma;
            }
        }
    }
    mt = wave_max_u32(mt);
    ma = wave_max_u32(ma);
    if (lane == 0) { red_m[2 * wid] = mt; red_m[2 * wid + 1] = ma; }
    __syncthreads();  // R2
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        mt = red_m[2 * q] > mt ? red_m[2 * q] : mt;
        ma = red_m[2 * q + 1] > ma ? red_m[2 * q + 1] : ma;
    }
    const double ymt = rcp_exact(mt), yma = rcp_exact(ma);
    uint64_t best = 0;
    for (uint32_t b0 = wid * 64 * U + lane; b0 < n; b0 += 4 * 64 * U) {
        RowT<F> r[U];
        RowX x[U];
        rows_at(b0, r, x);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t idx = b0 + 64 * u;
            const uint32_t tv = node_total<F>(r[u], x[u], p, pxi, cv, mt, ymt, ma, yma, nullptr);
            const uint64_t key = (idx < n && feasible<F>(r[u], x[u], p, pxi)) ? pack_key(tv + 1, idx) : 0ull;
            best = key > best ? key : best;
        }
    }
    uint64_t ks = wave_max_u64(best);
    if (lane == 0) red_k[wid] = ks;
    __syncthreads();  // R3
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) ks = red_k[q] > ks ? red_k[q] : ks;
    return ks;
}
// The pipeline waves' side of a rescan: R1, R2, R3, then the parked waves' key.
__device__ __forceinline__ uint64_t res_rescan_wait(const uint64_t *red_k) {
    __syncthreads();  // R1
    __syncthreads();  // R2
    __syncthreads();  // R3
    uint64_t ks = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) ks = red_k[q] > ks ? red_k[q] : ks;
    return ks;
}

template <uint32_t F, bool K32>
__device__ __forceinline__ void la_resolve4_stream(uint32_t *lds, const DevTable &t, const PodT<F> *__restrict__ pods,
                                                   const DevCfg &c, uint32_t P, uint32_t K, uint32_t nwin,
                                                   const uint64_t *lists0, uint32_t lwords,
                                                   int32_t *__restrict__ out_node, uint64_t *__restrict__ out_key,
                                                   uint64_t *__restrict__ stamps, ResCtl *ctl, uint64_t *rdiag,
                                                   const DPodX *__restrict__ podx, const NormInfo *norm0,
                                                   const uint32_t *stat0, unsigned long long *nfall) {
    constexpr bool NORM = (F & kFeatNorm) != 0;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nwords = (t.n + 31) / 32;
    uint32_t *dirty = lds;
    char *base = (char *)(lds + ((nwords + 3) & ~3u));
    uint64_t(*keyA)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*keyB)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*keyC)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    uint64_t(*C1)[64] = (uint64_t(*)[64])base; base += 2 * 64 * 8;
    RowT<F>(*stage)[64] = (RowT<F>(*)[64])base; base += 2 * 64 * sizeof(RowT<F>);
    int4(*stagex)[64] = (int4(*)[64])base; base += 2 * 64 * sizeof(int4);
    ResPub *pub = (ResPub *)base; base += 2 * sizeof(ResPub);
    uint32_t *xrank = (uint32_t *)base; base += 64 * 4;  // slot lane -> rank among the window's won slots, or ~0
    uint32_t *xnode = (uint32_t *)base; base += 64 * 4;  // slot lane -> node
    uint32_t *dnode = (uint32_t *)base; base += 64 * 4;  // rank -> node
    RowT<F> *carry = (RowT<F> *)base; base += 64 * sizeof(RowT<F>);
    int4 *carryx = (int4 *)base; base += 64 * sizeof(int4);
    PodT<F>(*wpods2)[64] = (PodT<F>(*)[64])base; base += 2 * 64 * sizeof(PodT<F>);  // window pod records, by window parity
    // NORM only (the host sizes the LDS accordingly)
    DPodX(*wpodx2)[kResNormK] = (DPodX(*)[kResNormK])base; base += 2 * kResNormK * sizeof(DPodX);
    NormInfo(*wnorm2)[kResNormK] = (NormInfo(*)[kResNormK])base; base += 2 * kResNormK * sizeof(NormInfo);
    double2(*wrcp2)[kResNormK] = (double2(*)[kResNormK])base; base += 2 * kResNormK * sizeof(double2);
    RowX(*stagexN)[64] = (RowX(*)[64])base; base += 2 * 64 * sizeof(RowX);  // full candidate RowX (masks)
    RowX *carryxN = (RowX *)base; base += 64 * sizeof(RowX);
    RowT<F> *srow = (RowT<F> *)base; base += 64 * sizeof(RowT<F>);  // rescan: slot rows
    RowX *sxr = (RowX *)base; base += 64 * sizeof(RowX);
    uint32_t(*flagC)[64] = (uint32_t(*)[64])base; base += 2 * 64 * 4;  // C's lost-holder flags
    uint32_t *sidx = (uint32_t *)base; base += 64 * 4;                // rescan: slot lane -> node
    uint32_t *red_m = (uint32_t *)base; base += 16 * 4;
    uint64_t *red_k = (uint64_t *)base; base += 8 * 8;
    uint32_t *snd = (uint32_t *)base; base += 16;                      // rescan: slot count
    // slot statics (static_raw) by [window pod][slot lane]: this window's, and the next window's
    // for the slots alive now (rank-compacted into Tcur at the boundary); stS: the statics of wave
    // C's staged candidates against the pod two later (a new slot's first key in waves A/B);
    // nflag2: the next window's pod flags
    uint32_t *Tcur = (uint32_t *)base; base += kResNormK * kResTStride * 4;
    uint32_t *Tnext = (uint32_t *)base; base += kResNormK * kResTStride * 4;
    uint32_t(*stS)[64] = (uint32_t(*)[64])base; base += 2 * 64 * 4;
    uint32_t(*nflag2)[kResNormK] = (uint32_t(*)[kResNormK])base; base += 2 * kResNormK * 4;
    // NORM: the taint / label masks of the current slots by slot lane (waves A / B carry only a
    // slot's extended resources: the masks are written by wave 4 when a slot is created, by wave A
    // at a window boundary for the inherited ones, and read by rescans and the boundary)
    DMask *smask = (DMask *)base;
    // RING (Fit + Balanced (+ext); the NORM arrays above are not allocated then, so the rings start
    // right after nflag2's slot): stream pod g's list entry per lane (ringE[g % kResRing]), the rows
    // of those entries (ringR / ringX: extended resources), and wave 4's "next window's lists were
    // not there in time" flag for C's boundary fallback
    char *rbase = (char *)(wpodx2);
    uint64_t(*ringE)[64] = (uint64_t(*)[64])rbase; rbase += kResRing * 64 * 8;
    RowT<F>(*ringR)[64] = (RowT<F>(*)[64])rbase; rbase += kResRing * 64 * sizeof(RowT<F>);
    int4(*ringX)[64] = (int4(*)[64])rbase; rbase += kResRing * 64 * sizeof(int4);
    uint32_t *late = (uint32_t *)rbase;
    const ResPub none{0, 0xFFFFFFFFu, -1, -1, 0, {0, 0}};
    const DPodX px{};
    // the LeastAllocated weights and weight-sum reciprocals held in VGPRs: the score's per-lane
    // selects then read them directly (gfx950 VALU takes one scalar operand: from SGPRs every
    // select needed a v_mov first, on every wave's critical path)
    DevCfg cv = c;
    asm volatile("" : "+v"(cv.yd_both), "+v"(cv.yd_c), "+v"(cv.yd_m), "+v"(cv.wc), "+v"(cv.wm));
    uint64_t ts_ = 0, busy_ = 0, steps_ = 0, sub_[3] = {0, 0, 0};
    // QS_RES_DIAG: wave D's window-boundary segments (s_memrealtime ticks summed over the windows):
    // [0] last step's barrier -> bookkeeping done, [1] -> B2, [2] -> B3, [3] -> B1, [4] -> pod 0 decided
    // [5] B3 -> B1 without the B1 wait (waves A and C: their [0])
    uint64_t bseg_[6] = {0, 0, 0, 0, 0, 0}, bt_ = 0;
    auto bmark = [&](int k) {
        if (rdiag) {
            const uint64_t t_ = __builtin_amdgcn_s_memrealtime();
            if (k >= 0 && bt_) bseg_[k] += t_ - bt_;
            bt_ = t_;
        }
    };
    // the pipeline waves (0-3) win VALU issue arbitration against the parked waves sharing their
    // SIMDs (MI355X_MICROARCH.md, two waves per SIMD: priority, then age)
    if (wv < 4) __builtin_amdgcn_s_setprio(3);

    for (uint32_t i = threadIdx.x; i < nwords; i += 256) dirty[i] = 0;
    if (threadIdx.x < min(K, P)) wpods2[0][threadIdx.x] = pods[threadIdx.x];
    if (threadIdx.x == 0) pub[1] = none;
    if constexpr (!NORM) {  // RING: no entry yet (wave 5 may read a slot before its first write)
        for (uint32_t j = threadIdx.x; j < kResRing * 64; j += 256) (&ringE[0][0])[j] = 0ull;
        if (threadIdx.x == 0) *late = 1u;  // window 0: C fetches its first entries and row
    }
    if constexpr (NORM) {  // window 0's pod extension records
        constexpr uint32_t q = sizeof(DPodX) / 16;
        for (uint32_t j = threadIdx.x; j < min(K, P) * q; j += kResBS)
            reinterpret_cast<int4 *>(&wpodx2[0][0])[j] = reinterpret_cast<const int4 *>(podx)[j];
    }
    __syncthreads();

    // NORM: exact rescan of window pod i by the parked waves (res_rescan_pass); the pipeline waves
    // keep the barrier count (res_rescan_wait) and read its key
    auto rescan_pass = [&](uint32_t i, uint32_t wb) -> uint64_t {
        return res_rescan_pass<F>(t, wpods2[wb][i], wpodx2[wb][i], dirty, sidx, srow, sxr, smask, red_m, red_k, snd,
                                  cv);
    };

    if (wv == 0) {
        // ---- D: pod i's winner from the precomputed keys (la_resolve4_block's wave D) -----------
        uint32_t nd = 0, didx = 0xFFFFFFFFu;
        bool won = false;  // slot won a pod of the current window (it stays a slot in the next one)
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const uint32_t knext = w + 1 < nwin ? min(K, P - s0 - K) : 0u;
            // next window's pod records (to LDS at the end; loaded unconditionally, clamped, so the
            // loads stay in flight through the window instead of being waited for at a branch join)
            // (three named registers, not an int4[PQ] array: the array stayed a private-memory
            // alloca, so the loads were waited for right away and spilled to scratch before B1,
            // ≈ 0.6 µs of every window boundary)
            constexpr int PQ = (int)(sizeof(PodT<F>) / 16);  // 16-byte quads per pod record (2, wide 3)
            static_assert(PQ == 2 || PQ == 3, "pod record of two or three 16-byte quads");
            const int4 *pq = reinterpret_cast<const int4 *>(pods + min(s0 + K + (uint32_t)lane, P - 1));
            const int4 npq0 = pq[0], npq1 = pq[1];
            const int4 npq2 = PQ > 2 ? pq[PQ - 1] : make_int4(0, 0, 0, 0);
            uint64_t res_key = 0, res_stamp = 0;
            ResPub pv = none;
            bool stopped = false;  // NORM: a rescan ran in this window
            if (NORM) __syncthreads();  // B0
            if (w > 0) bmark(5);
            __syncthreads();  // B1
            if (w > 0) bmark(3);
            if (rdiag && lane == 0) store_coh_u64(&rdiag[15], __builtin_amdgcn_s_memrealtime());
            for (uint32_t i = 0; i < kend; ++i) {
                QS_RSTAMP_BEGIN()
                const int par = i & 1, pp = par ^ 1;
                const uint64_t a = keyA[pp][lane], b = keyB[pp][lane], cl = keyC[pp][lane];
                const uint64_t e1 = C1[pp][lane];
                uint32_t fcl = 0;
                NormInfo nf{0, 0, 0, 0};
                if (NORM) {
                    fcl = flagC[pp][lane];
                    nf = wnorm2[w & 1][i];
                }
                const bool pnew = pv.ks != 0 && pv.slot < 0;
                uint64_t sc = (lane == pv.slot) ? b : a;
                uint32_t fl = 0;  // NORM: lost-holder flags of this slot (bit 0 taint, bit 1 affinity)
                if (NORM) {
                    fl = (uint32_t)sc & 3u;
                    sc &= ~3ull;
                }
                uint64_t fk = ((uint32_t)lane < nd && sc) ? (sc | (uint64_t)(0xFFFFFFFFu - didx)) : 0ull;
                // the new slot's key, read unconditionally (under a branch the compiler sank the
                // keyC load into it: a second, dependent LDS round trip on D's chain)
                const int srcl = pv.src >= 0 ? pv.src : 0;
                const uint64_t cw = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(cl >> 32), srcl) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cl, srcl);
                if (pnew && (uint32_t)lane == pv.nd_old) fk = cw;
                bool unsafe = false;
                if (NORM) {
                    const uint32_t fc = (uint32_t)__builtin_amdgcn_readlane((int)fcl, srcl);
                    if (pnew && (uint32_t)lane == pv.nd_old) fl = fc;
                    // do the selection-time maxima still hold for pod i?  A maximum is lost only
                    // when every node attaining it is dirty and infeasible now
                    if (F & kFeatTaint)
                        unsafe |= nf.mt > 0 && (uint32_t)__popcll(__ballot((uint32_t)lane < nd && (fl & 1u))) >= nf.ct;
                    if (F & kFeatAffinity)
                        unsafe |= nf.ma > 0 && (uint32_t)__popcll(__ballot((uint32_t)lane < nd && (fl & 2u))) >= nf.ca;
                }
                if (NORM && unsafe) {
                    if (lane == 0) pub[par] = ResPub{0, 0xFFFFFFFFu, -2, -1, nd, {0, 0}};  // STOP
                } else {
                    const uint64_t cand = (pv.ks != 0 && e1 != 0 && key_node(e1) == pv.w) ? 0ull : e1;
                    const uint64_t best = fk > cand ? fk : cand;
                    uint64_t ks;
                    if (K32) {  // (score+1) < 2^10 and n <= 2^22: one 32-bit reduction
                        const uint32_t tv = (uint32_t)(best >> 32);
                        const uint32_t k32 = tv ? (tv << 22) | (0x3FFFFFu - key_node(best)) : 0u;
                        const uint32_t m = wave_max_u32_dpp(k32);
                        ks = m ? (((uint64_t)(m >> 22) << 32) | (uint64_t)(0xFFFFFFFFu - (0x3FFFFFu - (m & 0x3FFFFFu)))) : 0ull;
                    } else {
                        ks = wave_max_u64(best);
                    }
                    ResPub np{ks, ks ? key_node(ks) : 0xFFFFFFFFu, -1, -1, nd, {0, 0}};
                    if (ks) {
                        const uint64_t own = __ballot((uint32_t)lane < nd && didx == np.w);
                        if (own) {
                            np.slot = (int32_t)__builtin_ctzll(own);
                            won |= lane == np.slot;
                        } else {
                            np.src = (int32_t)__builtin_ctzll(__ballot(cand == ks));
                            if ((uint32_t)lane == nd) { didx = np.w; won = true; }
                            ++nd;
                            if (lane == 0)  // dirty from now on: wave C's next dirty-word reads see it
                                __hip_atomic_fetch_or(&dirty[np.w >> 5], 1u << (np.w & 31), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    }
                    pv = np;
                    if (lane == 0) pub[par] = np;
                    if ((uint32_t)lane == i) {
                        res_key = ks;
                        if (stamps) res_stamp = __builtin_amdgcn_s_memrealtime();
                    }
                    if (i == 0 && w > 0) bmark(4);
                }
                QS_RSTAMP_MARK(0)
                QS_RSTAMP_END()
                __syncthreads();
                if (NORM && unsafe) {
                    // the exact rescan of pod i (every wave), then pod i's result as usual; a new
                    // slot takes source lane 0, whose staged row / key / flags wave C rewrites
                    if ((uint32_t)lane < nd) sidx[lane] = didx;
                    if (lane == 0) *snd = nd;
                    const uint64_t ks = res_rescan_wait(red_k);
                    ResPub np{ks, ks ? key_node(ks) : 0xFFFFFFFFu, -1, -1, nd, {0, 0}};
                    if (ks) {
                        const uint64_t own = __ballot((uint32_t)lane < nd && didx == np.w);
                        if (own) {
                            np.slot = (int32_t)__builtin_ctzll(own);
                            won |= lane == np.slot;
                        } else {
                            np.src = 0;
                            if ((uint32_t)lane == nd) { didx = np.w; won = true; }
                            ++nd;
                            if (lane == 0)
                                __hip_atomic_fetch_or(&dirty[np.w >> 5], 1u << (np.w & 31), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    }
                    pv = np;
                    if (lane == 0) {
                        pub[par] = np;
                        if (nfall) atomicAdd(nfall, 1ull);  // pods resolved by an exact rescan
                    }
                    if ((uint32_t)lane == i) {
                        res_key = ks;
                        if (stamps) res_stamp = __builtin_amdgcn_s_memrealtime();
                    }
                    stopped = true;
                    __syncthreads();  // R5
                }
            }
            steps_ += kend;
            bmark(-1);
            if (NORM && stopped && lane == 0 && nfall) atomicAdd(nfall + 1, 1ull);  // windows with a rescan
            if ((uint32_t)lane < kend) {
                out_node[s0 + lane] = res_key ? (int32_t)key_node(res_key) : -1;
                if (out_key) out_key[s0 + lane] = res_key;
                if (stamps) stamps[s0 + lane] = res_stamp;
            }
            // boundary: the won slots become the next window's inherited slots (rank order), the
            // others are clean again for the next window's lists (selected after this window's
            // predecessor was resolved)
            const bool act = (uint32_t)lane < nd;
            const uint64_t wm = __ballot(act && won);
            const uint32_t rk = (uint32_t)__popcll(wm & ((1ull << lane) - 1ull));
            xrank[lane] = (act && won) ? rk : 0xFFFFFFFFu;
            xnode[lane] = didx;
            if (act && won) {
                dnode[rk] = didx;
                // (already marked when created; kept as the boundary invariant: dirty == live slots)
                __hip_atomic_fetch_or(&dirty[didx >> 5], 1u << (didx & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (act && !won)
                __hip_atomic_fetch_and(&dirty[didx >> 5], ~(1u << (didx & 31)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((uint32_t)lane < knext) {
                int4 *dq = reinterpret_cast<int4 *>(&wpods2[(w + 1) & 1][lane]);
                dq[0] = npq0;
                dq[1] = npq1;
                if (PQ > 2) dq[PQ - 1] = npq2;
            }
            bmark(0);
            __syncthreads();  // B2
            bmark(1);
            __syncthreads();  // B3 (wave A stored and staged the won rows)
            bmark(2);
            nd = (uint32_t)__popcll(wm);
            didx = (uint32_t)lane < nd ? dnode[lane] : 0xFFFFFFFFu;
            won = false;
            if (lane == 0) pub[1] = none;
        }
    } else if (wv <= 2) {
        // ---- A / B: slot rows; apply pod i-1's winner, then the next pod's keys -----------------
        RowT<F> S = empty_row<F>();
        RowX SX{};
        uint32_t nd = 0;
        uint32_t pend = 0;  // wave A: windows whose rows are stored but not yet signalled (done value)
        const __amdgpu_buffer_rsrc_t rs = row_rsrc<F>(t);
        // NORM: pod k's maxima and reciprocals (LDS, read one step ahead)
        struct PodN {
            NormInfo nf;
            double2 yr;
        };
        // NORM: st = the slot's static_raw against pod q (Tcur, or stS for a slot created this step)
        auto slot_key = [&](const RowT<F> &r, const RowX &x, const PodT<F> &q, const PodN &pn, uint32_t st) -> uint64_t {
            const bool act = (uint32_t)lane < nd;
            if constexpr (QS_EXP_NORM_AB(NORM)) {
                const bool f = fits<F>(r, x, q) && (st & 1u) != 0u;
                const uint32_t tot = norm_total<F>(r, x, q, cv, st, pn.nf.mt, pn.yr.x, pn.nf.ma, pn.yr.y);
                uint32_t fl = 0;
                if (act && !f) fl = holder_flags<F>(st, pn.nf.mt, pn.nf.ma);
                return ((act && f) ? ((uint64_t)(tot + 1) << 32) : 0ull) | fl;
            }
            QS_EXP_SLOT_KEY(act, r, q)
            const bool f = feasible<F>(r, x, q, px);
            const uint32_t tot = node_total<F>(r, x, q, px, cv, 0, 0.0, 0, 0.0, nullptr);
            return (act && f) ? ((uint64_t)(tot + 1) << 32) : 0ull;
        };
        uint32_t snew = 0;  // NORM: the static of a slot created by the applied winner
        // (the new slot's row is read from LDS at pv.src: a per-lane readlane of the own-lane staged
        // rows instead was measured slower, A / B +90 busy cycles a step)
        // gi: the stream pod whose winner pv is (RING: its candidates' rows are ringR[gi % kResRing])
        auto apply = [&](const ResPub &pv, int pp, const PodT<F> &pprev, uint32_t gi) {
            if (pv.ks == 0) return;
            if (pv.slot >= 0) {
                if (lane == pv.slot) reserve(S, SX, pprev, +1);
            } else {
                if ((uint32_t)lane == pv.nd_old) {
                    if constexpr (!NORM) {
                        S = ringR[gi % kResRing][pv.src];
                        if (F & kFeatExt) {
                            const int4 e = ringX[gi % kResRing][pv.src];
                            SX.ae0 = e.x; SX.re0 = e.y; SX.ae1 = e.z; SX.re1 = e.w;
                        }
                    } else {
                        S = stage[pp][pv.src];
                    }
                    if constexpr (NORM) {  // (the extended resources only: masks in smask)
                        const int4 e = *reinterpret_cast<const int4 *>(&stagexN[pp][pv.src]);
                        SX.ae0 = e.x; SX.re0 = e.y; SX.ae1 = e.z; SX.re1 = e.w;
                        snew = stS[pp][pv.src];
                    }
                    reserve(S, SX, pprev, +1);
                }
                ++nd;
            }
        };
        // NORM: D stopped at window pod j: stage the slot rows (wave A), rescan with every wave
        auto rescan_ab = [&](uint32_t j, uint32_t wb) {
            if (wv == 1 && (uint32_t)lane < nd) {  // (the rescan takes the slot masks from smask)
                srow[lane] = S;
                *reinterpret_cast<int4 *>(&sxr[lane]) = make_int4(SX.ae0, SX.re0, SX.ae1, SX.re1);
            }
            (void)res_rescan_wait(red_k);
            (void)j;
            (void)wb;
            __syncthreads();  // R5
        };
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const PodT<F> *wp = wpods2[w & 1];
            auto podn = [&](uint32_t k) -> PodN {
                PodN r{};
                if constexpr (NORM)
                    if (k < kend) r = PodN{wnorm2[w & 1][k], wrcp2[w & 1][k]};
                return r;
            };
            if (NORM) __syncthreads();  // B0 (the window's NormInfo is in LDS)
            if (wv == 1 && nd > 0)  // pod 0, inherited slots
                keyA[1][lane] = slot_key(S, SX, wp[0], podn(0), NORM ? Tcur[lane] : 0u);
            if (w > 0) bmark(0);
            __syncthreads();  // B1
            const uint32_t isig = 0;  // the step that signals done for the previous window
            PodT<F> pprev = wp[0], pcur = wp[0];  // pods i-1 and i (pod i+1's record is read each step)
            PodN pnx = podn(1);                   // NORM: pod i+1's record at step i
            for (uint32_t i = 0; i < kend; ++i) {
                QS_RSTAMP_BEGIN()
                const int par = i & 1, pp = par ^ 1;
                ResPub pv = read_pub(&pub[pp]);
                const PodT<F> pn1 = wp[i + 1];
                const uint32_t tst = NORM ? Tcur[min(i + 1, kResNormK - 1) * kResTStride + lane] : 0u;
                PodN pnn{};
                if (NORM) pnn = podn(i + 2);  // next step's maxima: read with this step's LDS reads
                __builtin_amdgcn_sched_barrier(0);  // the LDS reads go out before the pub's wait
                if (NORM && i > 0 && pv.slot == -2) {  // D stopped at pod i-1
                    rescan_ab(i - 1, w & 1);
                    pv = read_pub(&pub[pp]);
                }
                const uint32_t nd0 = nd;
                QS_RSTAMP_MARK(0)
                if (i > 0) apply(pv, pp, pprev, s0 + i - 1);
                QS_RSTAMP_MARK(1)
                if (wv == 1 && pend && i == isig) {
                    // the previous window's rows went out write-through at the boundary (B2-B3)
                    drain_stores();
                    if (lane == 0) __hip_atomic_store((gu32 *)&ctl->done, pend, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    pend = 0;
                }
                if (i + 1 < kend) {
                    const PodN pnc = pnx;
                    pnx = pnn;
                    RowT<F> s2 = S;
                    RowX x2s = SX;
                    if (wv == 2) reserve(s2, x2s, pcur, +1);
                    // a slot created by pod i-1's winner has no Tcur entry yet: its static came with
                    // the candidate wave C staged
                    const uint32_t st = (nd != nd0 && (uint32_t)lane == nd0) ? snew : tst;
                    (wv == 1 ? keyA : keyB)[par][lane] = slot_key(s2, x2s, pn1, pnc, st);
                }

                pprev = pcur;
                pcur = pn1;
                QS_RSTAMP_END()
                __syncthreads();
            }
            if (NORM && read_pub(&pub[(kend - 1) & 1]).slot == -2) rescan_ab(kend - 1, w & 1);
            apply(read_pub(&pub[(kend - 1) & 1]), (kend - 1) & 1, pprev, s0 + kend - 1);
            __syncthreads();  // B2 (D's slot ranks and nodes)
            const uint32_t rk = xrank[lane];
            const bool keep = (uint32_t)lane < nd && rk != 0xFFFFFFFFu;
            if (wv == 1 && keep) {
                store_row_coh<F>(t, rs, xnode[lane], S, SX);
                carry[rk] = S;
                if constexpr (NORM) {
                    const DMask m = smask[lane];
                    carryxN[rk] = RowX{SX.ae0, SX.re0, SX.ae1, SX.re1, m.th, m.ts, m.lb0, m.lb1};
                } else {
                    carryx[rk] = make_int4(SX.ae0, SX.re0, SX.ae1, SX.re1);
                }
            }
            if (wv == 1) pend = w + 1;
            __syncthreads();  // B3
            nd = (uint32_t)__popcll(__ballot(keep));
            if ((uint32_t)lane < nd) {
                S = carry[lane];
                if constexpr (NORM) {
                    const RowX o = carryxN[lane];
                    SX = RowX{};
                    SX.ae0 = o.ae0; SX.re0 = o.re0; SX.ae1 = o.ae1; SX.re1 = o.re1;
                    if (wv == 1) smask[lane] = DMask{o.th, o.ts, o.lb0, o.lb1};
                } else {
                    const int4 e = carryx[lane];
                    SX.ae0 = e.x; SX.re0 = e.y; SX.ae1 = e.z; SX.re1 = e.w;
                }
            } else {
                S = empty_row<F>();
                SX = RowX{};
            }
            bmark(-1);
        }
        if (wv == 1 && pend) {
            drain_stores();
            if (lane == 0) __hip_atomic_store((gu32 *)&ctl->done, pend, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (NORM && wv == 3) {
        // ---- C: candidate rows, C keys, the next pod's best clean entry; next-window prefetch -----
        uint64_t eX = 0, eY = 0, eZ = 0, c1 = 0;
        // NORM: the statics of pod i's entries (this lane's) against pods i+1 and i+2, published by
        // the selectors with the lists; two register pairs by pod parity, each loaded two pods ahead
        // in place (a pair is reloaded right after its pod's step used it)
        uint32_t sA1 = 0, sA2 = 0, sB1 = 0, sB2 = 0;
        RowT<F> r1 = empty_row<F>();
        RowX x1{};
        bool pref = false;  // window w's first entries and first candidate rows already loaded
        uint64_t pe0 = 0, pe1 = 0, pe2 = 0;
        uint64_t pn0 = 0, pn1w = 0;  // NORM: the next window's NormInfo of this lane's pod (prefetched)
        uint32_t rdyv = 0, nfallback = 0;
        uint64_t cdef_ = 0, cmiss_ = 0;  // QS_RES_DIAG: lists missing at the prefetch check (sum, windows)
        auto dirty_bit = [&](uint64_t e) -> bool {
            const uint32_t nidx = e ? key_node(e) : 0u;
            return (dirty[nidx >> 5] >> (nidx & 31)) & 1u;
        };
        // NORM: NormInfo of lane `lane`'s pod into the window's LDS arrays (+ the reciprocals)
        auto put_norm = [&](uint32_t wb, uint64_t lo, uint64_t hi) {
            const NormInfo nf{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
            wnorm2[wb][lane] = nf;
            wrcp2[wb][lane] = make_double2(rcp_exact(nf.mt), rcp_exact(nf.ma));
        };
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const uint64_t *lists = lists0 + (size_t)(w & 1) * lwords;
            const uint32_t *stats = NORM ? stat0 + (size_t)(w & 1) * K * 128 : nullptr;
            const PodT<F> *wp = wpods2[w & 1];
            const bool hasnext = w + 1 < nwin;
            const uint32_t knext = hasnext ? min(K, P - s0 - K) : 0u;
            const uint64_t *listsn = lists0 + (size_t)((w + 1) & 1) * lwords;
            const uint32_t *statsn = NORM ? stat0 + (size_t)((w + 1) & 1) * K * 128 : nullptr;
            const uint32_t tnext = ((w + 1) >> 1) * K + knext;
            // an entry, loaded unconditionally from a clamped pod (a load under a branch made the
            // compiler wait for every load in flight at the next join); an entry of a pod beyond the
            // window is never consumed: every use is guarded by that pod's index
            auto ent = [&](const uint64_t *l, uint32_t pod, uint32_t kk) -> uint64_t {
                return load_coh_u64(l + (size_t)min(pod, kk - 1) * 64 + lane);
            };
            // NORM: the statics of pod `pod`'s entries (this lane's) into a register pair
            auto stat_load = [&](uint32_t &d1, uint32_t &d2, const uint32_t *sl, uint32_t pod, uint32_t kk) {
                if constexpr (NORM) {
                    const uint32_t *q = sl + (size_t)min(pod, kk - 1) * 128 + lane;
                    d1 = load_coh_u32(q);
                    d2 = load_coh_u32(q + 64);
                }
            };
            // NORM: D stopped at window pod j: the parked waves rescan it (and stage a new slot's
            // row, static, key and flags as source lane 0 of step j); C keeps the barrier count
            auto rescan_c = [&](uint32_t j) {
                (void)res_rescan_wait(red_k);
                (void)j;
                __syncthreads();  // R5
            };
            uint64_t e0;
            if (pref) {
                e0 = pe0; eX = pe1; eY = pe2;
            } else {
                ++nfallback;
                if (lane == 0) (void)res_wait_ge(&ctl->rdy[w & 1][0], (w >> 1) * K + kend, c.werr, res_bound(c, w));
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below)
                e0 = ent(lists, 0, kend);
                eX = ent(lists, 1, kend);
                eY = ent(lists, 2, kend);
                stat_load(sA1, sA2, stats, 0, kend);
                stat_load(sB1, sB2, stats, 1, kend);
                if constexpr (NORM) {
                    if ((uint32_t)lane < kend) {
                        const uint64_t *nq = reinterpret_cast<const uint64_t *>(norm0 + (size_t)(w & 1) * 64 + lane);
                        put_norm(w & 1, load_coh_u64(nq), load_coh_u64(nq + 1));
                    }
                }
            }
            c1 = (e0 != 0 && !dirty_bit(e0)) ? e0 : 0ull;
            C1[1][lane] = c1;
            if (!pref) {
                r1 = load_row<F>(t, c1 ? key_node(c1) : 0u);
                x1 = load_rowx<F>(t, c1 ? key_node(c1) : 0u);
            }  // else r1 / x1 hold e0's row (loaded at the previous window's last pod)
            pref = false;
            if (NORM) __syncthreads();  // B0
            if (w > 0) bmark(0);
            __syncthreads();  // B1
            const bool pfw = hasnext && kend >= 6;  // prefetch the next window during this one
            PodT<F> pcur = wp[0];  // pod i's record (pod i+1's is read each step)
            // HOOK: the step may carry the next-window prefetch (only the last steps of a window)
            // LM (entry loads): 0 pod i+3's entry into en; 1 pods i+3 and i+4 (into en and eZ); 2 none,
            // en takes eZ.  The plain pairs use 1 then 2, so no entry load is in flight at the loop's
            // back-edge (the compiler waits for every load in flight there, vmcnt(0)).
            auto step = [&](auto hook, auto lm, uint32_t i, uint64_t &en, uint32_t &c1s1, uint32_t &c1s2) {
                QS_RSTAMP_BEGIN()
                const int par = i & 1;
                // the step's LDS reads first, together: the dirty word of pod i+1's entry (the set
                // through pod i-1: wave D marks a new slot in the step that creates it) and pod i+1.
                // C never reads the published winner: a candidate taken by pod i-1's winner is
                // masked by D, which then never names that lane as a new slot's source.
                const uint32_t en_node = en ? key_node(en) : 0u;
                uint32_t dword = dirty[en_node >> 5];
                // pod i+1's candidate row, issued first: its address needs the entry only (a dirty
                // entry's row is loaded and never used), so the load has the whole step to arrive.
                // One unconditional load (the last pod: the next window's first candidate when
                // prefetched, else node 0's row, never used; a node dirtied from here on is masked
                // out at the boundary): issued at the step's end, or under a branch, the compiler's
                // wait tracking waited for the rows early in the next step (measured: config 2 +1.5 %,
                // config 3 +1 %, wide +3 %, config 4 +3.6 % against the late issue; -9 % / -16 % for
                // wide / config 4 with the load under a branch).
                const uint32_t ln = i + 1 < kend ? en_node : (pref && pe0 ? key_node(pe0) : 0u);
                const RowT<F> rn = load_row<F>(t, ln);
                const RowX xn = load_rowx<F>(t, ln);
                const PodT<F> pn1 = wp[i + 1];
                const uint32_t kn = min(i + 1, kend - 1);
                NormInfo nf{0, 0, 0, 0};
                double2 yr = make_double2(0.0, 0.0);
                int32_t stop = 0;
                if constexpr (NORM) {
                    nf = wnorm2[w & 1][kn];
                    yr = wrcp2[w & 1][kn];
                    stop = pub[par ^ 1].slot;  // NORM only: a STOP of pod i-1 is read here
                }
                __builtin_amdgcn_sched_barrier(0);  // the LDS reads go out before their waits
                if (NORM && i > 0 && stop == -2) {
                    rescan_c(i - 1);
                    dword = dirty[en_node >> 5];  // pod i-1's rescanned winner is dirty now
                }
                QS_RSTAMP_MARK(0)
                // keyC's score (candidate c1's row + pod i, scored for pod i+1) needs no pub
                RowT<F> cr = r1;
                RowX crx = x1;
                reserve(cr, crx, pcur, +1);
                bool f;
                uint32_t tot, fl = 0;
                if constexpr (NORM) {  // the candidate's static against pod i+1 came with its entry
                    f = fits<F>(cr, crx, pn1) && (c1s1 & 1u) != 0u;
                    tot = norm_total<F>(cr, crx, pn1, cv, c1s1, nf.mt, yr.x, nf.ma, yr.y);
                    if (!f) fl = holder_flags<F>(c1s1, nf.mt, nf.ma);
                } else {
                    f = feasible<F>(cr, crx, pn1, px);
                    tot = node_total<F>(cr, crx, pn1, px, cv, 0, 0.0, 0, 0.0, nullptr);
                    QS_EXP_CAND_KEY(f, tot, cr, pn1)
                }
                QS_RSTAMP_MARK(1)
                stage[par][lane] = r1;
                if constexpr (NORM) {
                    stagexN[par][lane] = x1;
                    stS[par][lane] = c1s2;
                } else if (F & kFeatExt) {
                    stagex[par][lane] = make_int4(x1.ae0, x1.re0, x1.ae1, x1.re1);
                }
                if (i + 1 < kend) {
                    keyC[par][lane] = (c1 != 0 && f) ? pack_key(tot + 1, key_node(c1)) : 0ull;
                    if (NORM) flagC[par][lane] = fl;
                    const bool dirt = ((dword >> (en_node & 31)) & 1u) != 0;
                    c1 = (en != 0 && !dirt) ? en : 0ull;  // pod i+1 against the dirty set through pod i-1
                    C1[par][lane] = c1;
                    if constexpr (decltype(lm)::value == 2) {
                        en = eZ;
                    } else {
                        en = ent(lists, i + 3, kend);
                        if constexpr (decltype(lm)::value == 1) eZ = ent(lists, i + 4, kend);
                    }
                }
                r1 = rn;
                x1 = xn;
                // NORM: this parity's pair now holds pod i+2's statics (the next window's pod
                // i+2-kend when prefetched)
                if (i + 2 < kend) stat_load(c1s1, c1s2, stats, i + 2, kend);
                else if (pref) stat_load(c1s1, c1s2, statsn, i + 2 - kend, knext);
                QS_RSTAMP_MARK(2)
                pcur = pn1;
                if (decltype(hook)::value && pfw) {
                    if (i == kend - 5) rdyv = load_coh_u32(&ctl->rdy[(w + 1) & 1][0]);
                    if (i == kend - 3) {
                        pref = __builtin_amdgcn_readfirstlane(rdyv) >= tnext;
                        if (rdiag && !pref) {  // QS_RES_DIAG: how many of the next window's lists were missing
                            cdef_ += tnext - (uint32_t)__builtin_amdgcn_readfirstlane(rdyv);
                            cmiss_ += 1;
                        }
                        if (pref) {
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                            pe0 = ent(listsn, 0, knext);
                            pe1 = ent(listsn, 1, knext);
                            pe2 = ent(listsn, 2, knext);
                            if constexpr (NORM) {
                                const uint64_t *nq =
                                    reinterpret_cast<const uint64_t *>(norm0 + (size_t)((w + 1) & 1) * 64 + lane);
                                pn0 = (uint32_t)lane < knext ? load_coh_u64(nq) : 0ull;
                                pn1w = (uint32_t)lane < knext ? load_coh_u64(nq + 1) : 0ull;
                            }
                        }
                    }
                }
                QS_RSTAMP_END()
                __syncthreads();
            };
            const std::integral_constant<bool, false> plain{};
            const std::integral_constant<bool, true> hooked{};
            const std::integral_constant<int, 0> l1{};
            const std::integral_constant<int, 1> l2{};
            const std::integral_constant<int, 2> l0{};
            const uint32_t ih = pfw ? ((kend - 5) & ~1u) : kend;  // first step with the hooks (even)
            uint32_t i = 0;
            for (; i + 1 < ih; i += 2) {
                step(plain, l2, i, eX, sA1, sA2);
                step(plain, l0, i + 1, eY, sB1, sB2);
            }
            for (; i + 1 < kend; i += 2) {
                step(hooked, l1, i, eX, sA1, sA2);
                step(hooked, l1, i + 1, eY, sB1, sB2);
            }
            if (i < kend) step(hooked, l1, i, eX, sA1, sA2);
            if (NORM && pref && (kend & 1)) {  // the next window's pods 0 / 1 went to the B / A pairs
                const uint32_t t1 = sA1, t2 = sA2;
                sA1 = sB1; sA2 = sB2;
                sB1 = t1; sB2 = t2;
            }
            if (NORM && pub[(kend - 1) & 1].slot == -2) rescan_c(kend - 1);
            if (NORM && pref && (uint32_t)lane < knext) put_norm((w + 1) & 1, pn0, pn1w);
            __syncthreads();  // B2
            __syncthreads();  // B3 (D cleared the dropped slots' dirty bits before B2)
            bmark(-1);
        }
        if (rdiag && lane == 0) { rdiag[4] = nfallback; rdiag[5] = cdef_; rdiag[6] = cmiss_; }
    } else if (!NORM && wv == 3) {
        // ---- C (RING, Fit + Balanced (+ext)): every lane's candidate key and the next pod's best
        // clean entry.  The entries come from ringE (wave 4) and the candidates' rows from ringR /
        // ringX (wave 5), so a step issues no global load: C's row no longer waits behind older
        // sc1 entry loads (vector loads complete in issue order).  A/B read a new slot's row from
        // ringR as well, so C stages nothing.
        uint64_t c1 = 0;
        uint32_t nfallback = 0;
        auto dirty_bit = [&](uint64_t e) -> bool {
            const uint32_t nidx = e ? key_node(e) : 0u;
            return (dirty[nidx >> 5] >> (nidx & 31)) & 1u;
        };
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const PodT<F> *wp = wpods2[w & 1];
            if (*late) {
                // the first window, or the lists of this one were not all published when wave 4
                // looked (three pods before the previous window's end): the entries of pods 0-2 and
                // the rows of pod 0's entries here, before B1 (wave 4 then continues from pod 3)
                ++nfallback;
                const uint64_t *lists = lists0 + (size_t)(w & 1) * lwords;
                if (lane == 0) (void)res_wait_ge(&ctl->rdy[w & 1][0], (w >> 1) * K + kend, c.werr, res_bound(c, w));
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below)
                uint64_t e[3];
#pragma unroll
                for (uint32_t j = 0; j < 3; ++j)
                    e[j] = j < kend ? load_coh_u64(lists + (size_t)j * 64 + lane) : 0ull;
#pragma unroll
                for (uint32_t j = 0; j < 3; ++j) ringE[(s0 + j) % kResRing][lane] = e[j];
                const uint32_t n0 = e[0] ? key_node(e[0]) : 0u;
                ringR[s0 % kResRing][lane] = load_row<F>(t, n0);
                if (F & kFeatExt) {
                    const RowX x = load_rowx<F>(t, n0);
                    ringX[s0 % kResRing][lane] = make_int4(x.ae0, x.re0, x.ae1, x.re1);
                }
            }
            // pod 0's candidates against the dirty set at the window start (the inherited slots)
            const uint64_t e0 = ringE[s0 % kResRing][lane];
            c1 = (e0 != 0 && !dirty_bit(e0)) ? e0 : 0ull;
            C1[1][lane] = c1;
            if (w > 0) bmark(0);
            __syncthreads();  // B1
            PodT<F> pcur = wp[0];  // pod i's record (pod i+1's is read each step)
            for (uint32_t i = 0; i < kend; ++i) {
                QS_RSTAMP_BEGIN()
                const uint32_t g = s0 + i;
                const int par = i & 1;
                // the step's LDS reads: pod i+1's entry (then its dirty word: the set through pod
                // i-1, wave D marks a new slot in the step that creates it), pod i's candidate row
                // (c1's), pod i+1's record.  C never reads the published winner: a candidate taken
                // by pod i-1's winner is masked by D, which then never names that lane as a source.
                const uint64_t en = ringE[(g + 1) % kResRing][lane];
                const RowT<F> r1 = ringR[g % kResRing][lane];
                RowX x1{};
                if (F & kFeatExt) {
                    const int4 e = ringX[g % kResRing][lane];
                    x1.ae0 = e.x; x1.re0 = e.y; x1.ae1 = e.z; x1.re1 = e.w;
                }
                const PodT<F> pn1 = wp[i + 1];
                const uint32_t en_node = en ? key_node(en) : 0u;
                const uint32_t dword = dirty[en_node >> 5];
                QS_RSTAMP_MARK(0)
                // keyC: candidate c1's row + pod i, scored for pod i+1 (needs no pub)
                RowT<F> cr = r1;
                RowX crx = x1;
                reserve(cr, crx, pcur, +1);
                const bool f = feasible<F>(cr, crx, pn1, px);
                const uint32_t tot = node_total<F>(cr, crx, pn1, px, cv, 0, 0.0, 0, 0.0, nullptr);
                QS_EXP_CAND_KEY(f, tot, cr, pn1)
                QS_RSTAMP_MARK(1)
                if (i + 1 < kend) {
                    keyC[par][lane] = (c1 != 0 && f) ? pack_key(tot + 1, key_node(c1)) : 0ull;
                    const bool dirt = ((dword >> (en_node & 31)) & 1u) != 0;
                    c1 = (en != 0 && !dirt) ? en : 0ull;  // pod i+1 against the dirty set through pod i-1
                    C1[par][lane] = c1;
                }
                QS_RSTAMP_MARK(2)
                pcur = pn1;
                QS_RSTAMP_END()
                __syncthreads();
            }
            __syncthreads();  // B2
            __syncthreads();  // B3 (D cleared the dropped slots' dirty bits before B2)
            bmark(-1);
        }
        if (rdiag && lane == 0) { rdiag[4] = nfallback; rdiag[5] = 0; rdiag[6] = 0; }
    } else if (!NORM && wv == 4) {
        // ---- wave 4 (RING): list entries three pods ahead.  Step i (stream pod g) writes E(g+2),
        // whose sc1 load it issued one step earlier (the wait sits at the loop's top, where the
        // compiler waits for every load in flight anyway), and issues E(g+3).  The next window's
        // entries need all its lists published: rdy is read at step kend-4 and decided at kend-3
        // (late = 0: prefetched; else C's fallback at the next window's start).  A wave of its own,
        // so its loads never sit in front of another wave's.
        uint64_t ein = 0;   // E(g+2), in flight at the start of step i
        bool skip = true;   // step 0: E(s0+2) came from C's fallback
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const bool hasnext = w + 1 < nwin;
            const uint32_t knext = hasnext ? min(K, P - s0 - K) : 0u;
            const uint64_t *lists = lists0 + (size_t)(w & 1) * lwords;
            const uint64_t *listsn = lists0 + (size_t)((w + 1) & 1) * lwords;
            const uint32_t tnext = ((w + 1) >> 1) * K + knext;
            const bool pfw = hasnext && kend >= 6;
            const uint32_t ic = pfw ? kend - 3 : kend - 1;  // the step that decides the next window's path
            bool lt = hasnext;
            uint32_t rdyv = 0;
            __syncthreads();  // B1
            for (uint32_t i = 0; i < kend; ++i) {
                const uint32_t g = s0 + i;
                if (!(skip && i == 0)) ringE[(g + 2) % kResRing][lane] = ein;
                if (i == ic) {
                    if (pfw) lt = !((uint32_t)__builtin_amdgcn_readfirstlane(rdyv) >= tnext);
                    if (lane == 0) *late = lt ? 1u : 0u;
                }
                // E(g+3): this window's pod i+3, or the next window's pod i+3-kend once its lists are in
                uint64_t v = 0;
                if (i + 3 < kend) {
                    v = load_coh_u64(lists + (size_t)(i + 3) * 64 + lane);
                } else if (i >= ic && !lt && hasnext) {
                    const uint32_t j = i + 3 - kend;
                    v = load_coh_u64(listsn + (size_t)min(j, knext - 1) * 64 + lane);
                    v = j < knext ? v : 0ull;
                }
                ein = v;
                if (pfw && i + 4 == kend) rdyv = load_coh_u32(&ctl->rdy[(w + 1) & 1][0]);
                __syncthreads();
            }
            skip = lt;
            __syncthreads();  // B2
            __syncthreads();  // B3
        }
    } else if (!NORM && wv == 5) {
        // ---- wave 5 (RING): the rows of pod g+1's entries (plain loads, issued and waited within
        // step i) into ringR / ringX for C's step i+1 and A/B's step i+2; the next window's pod 0
        // only when wave 4 prefetched its entries (late == 0)
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const bool hasnext = w + 1 < nwin;
            const bool pfw = hasnext && kend >= 6;
            __syncthreads();  // B1
            for (uint32_t i = 0; i < kend; ++i) {
                const uint32_t g = s0 + i;
                const bool go = i + 1 < kend || (pfw ? *late == 0u : !hasnext);
                if (go) {
                    const uint64_t e = ringE[(g + 1) % kResRing][lane];
                    const uint32_t nd = e ? key_node(e) : 0u;
                    const RowT<F> r = load_row<F>(t, nd);
                    ringR[(g + 1) % kResRing][lane] = r;
                    if (F & kFeatExt) {
                        const RowX x = load_rowx<F>(t, nd);
                        ringX[(g + 1) % kResRing][lane] = make_int4(x.ae0, x.re0, x.ae1, x.re1);
                    }
                }
                __syncthreads();
            }
            __syncthreads();  // B2
            __syncthreads();  // B3
        }
    } else if constexpr (NORM) {
        // ---- waves 4-7: slot statics, the rescans' extra hands, the next window's pod records ------
        // Per step (work(i), before the step's barrier; a STOP's rescan of pod i-1 already done):
        //  wave 4: a slot created by pod i-1's winner: its static against this window's pods from
        //          i+2 on (Tcur; waves A/B take pod i+1's from stS) and against the next window's
        //          pods (Tnext) — on wave D's SIMD, the least busy pipeline wave's (round 6: from
        //          wave 6, which shares wave B's: config 4 147.0 -> 145.1 ms);
        //  wave 7: one share of the inherited slots' statics against the next window's pods (Tnext);
        //  step 0: the next window's pod extension records and flags into LDS.
        // Between B2 and B3, Tnext is rank-compacted into Tcur for the next window's inherited slots.
        constexpr uint32_t q = sizeof(DPodX) / 16;
        const uint32_t pw = (uint32_t)(wv - 4);
        uint32_t ndi = 0;  // this window's inherited slots
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t s0 = w * K, kend = min(K, P - s0);
            const uint32_t knext = w + 1 < nwin ? min(K, P - s0 - K) : 0u;
            const uint32_t wb = w & 1, nb = (w + 1) & 1;
            const PodT<F> *wp = wpods2[wb];
            const uint32_t id0 = pw * 64 + lane, id1 = id0 + 256;
            const bool h0 = id0 < knext * q, h1 = id1 < knext * q;
            const int4 *src = reinterpret_cast<const int4 *>(podx + (size_t)s0 + K);
            int4 q0 = make_int4(0, 0, 0, 0), q1 = make_int4(0, 0, 0, 0);
            if (h0) q0 = src[id0];
            if (h1) q1 = src[id1];
            uint32_t nfl = 0;
            if (pw == 0 && (uint32_t)lane < knext) nfl = pods[s0 + K + lane].flags;
            // Waves 4 and 7 keep one pod's extension record and flags per lane in registers for the
            // window (read from LDS once, at step 1): wave 4 lanes 0-31 this window's pod `lane`,
            // lanes 32-63 and every wave-7 lane the next window's pod `lane & 31`.  Reading a record
            // per lane and step from LDS held the pipeline waves' reads up by ~850 cycles a step.
            const uint32_t qq = (uint32_t)lane & 31u;
            const bool mycur = wv == 4 && lane < 32;
            DPodX myx{};
            uint32_t myf = 0;
            auto load_mine = [&]() {
                myx = mycur ? wpodx2[wb][qq] : wpodx2[nb][qq];
                myf = mycur ? wp[qq].flags : nflag2[nb][qq];
            };
            // new slot of pod j's winner (j = i - 1): statics against pods >= j + 3 of this window
            // (cur) and every next-window pod
            auto new_slot = [&](uint32_t j, bool cur) {
                QS_EXP_PARK_RETURN()
                const ResPub pv = read_pub(&pub[j & 1]);
                if (pv.ks == 0 || pv.slot >= 0) return;
                const RowX sx = stagexN[j & 1][pv.src];
                const uint32_t l = pv.nd_old;
                if (lane == 0) smask[l] = DMask{sx.th, sx.ts, sx.lb0, sx.lb1};
                const uint32_t st = static_raw(sx.th, sx.ts, sx.lb0, sx.lb1, myf, myx);
                if (lane < 32) {
                    if (cur && qq >= j + 3 && qq < kend) Tcur[qq * kResTStride + l] = st;
                } else if (qq < knext) {
                    Tnext[qq * kResTStride + l] = st;
                }
            };
            // inherited slots x next-window pods: slots 2j (lanes 0-31) and 2j + 1 (lanes 32-63)
            auto inherited = [&](uint32_t j) {
                QS_EXP_PARK_RETURN()
                const uint32_t l = 2 * j + (lane < 32 ? 0u : 1u);
                if (l < ndi && qq < knext) {
                    const RowX sx = carryxN[l];
                    Tnext[qq * kResTStride + l] = static_raw(sx.th, sx.ts, sx.lb0, sx.lb1, myf, myx);
                }
            };
            // a rescan of pod j found winner ks: if it is a new slot, stage it as source lane 0 of
            // step j (wave C's staging): its row before pod j, its static against pod j+2, and its
            // key and lost-holder flags for pod j+1 after pod j (wave 4, before R5)
            auto rescan_tail = [&](uint32_t j, uint64_t ks) {
                const uint32_t W = ks ? key_node(ks) : 0u;
                const bool slot = __ballot((uint32_t)lane < *snd && sidx[lane] == W) != 0;
                if (!ks || slot) return;
                // the staged row is needed even at the window's last pod (waves A/B apply it after
                // the loop); the key and flags only when pod j+1 is in this window
                const int pj = j & 1;
                const RowT<F> rw = load_row<F>(t, W);
                const RowX xw = load_rowx<F>(t, W);
                uint32_t st2 = 0;
                if (j + 2 < kend) st2 = static_raw(xw.th, xw.ts, xw.lb0, xw.lb1, wp[j + 2].flags, wpodx2[wb][j + 2]);
                if (lane == 0) {
                    stage[pj][0] = rw;
                    stagexN[pj][0] = xw;
                    stS[pj][0] = st2;
                }
                if (j + 1 < kend) {
                    RowT<F> cr = rw;
                    RowX crx = xw;
                    reserve(cr, crx, wp[j], +1);
                    const PodT<F> q1 = wp[j + 1];
                    const DPodX qx = wpodx2[wb][j + 1];
                    const NormInfo nf = wnorm2[wb][j + 1];
                    const double2 yr = wrcp2[wb][j + 1];
                    const bool f = feasible<F>(cr, crx, q1, qx);
                    const uint32_t tot = node_total<F>(cr, crx, q1, qx, cv, nf.mt, yr.x, nf.ma, yr.y, nullptr);
                    uint32_t fl = 0;
                    if (!f) {
                        if (F & kFeatTaint) fl |= taint_raw(crx, qx) == nf.mt ? 1u : 0u;
                        if (F & kFeatAffinity) fl |= affinity_raw(crx, q1, qx) == nf.ma ? 2u : 0u;
                    }
                    if (lane == 0) {
                        keyC[pj][0] = f ? pack_key(tot + 1, W) : 0ull;
                        flagC[pj][0] = fl;
                    }
                }
            };
            __syncthreads();  // B0
            __syncthreads();  // B1
            for (uint32_t i = 0; i < kend; ++i) {
                if (i == 0) {
                    int4 *dst = reinterpret_cast<int4 *>(&wpodx2[nb][0]);
                    if (h0) dst[id0] = q0;
                    if (h1) dst[id1] = q1;
                    if (pw == 0 && (uint32_t)lane < knext) nflag2[nb][lane] = nfl;
                } else if (wv == 4 || wv == 7) {
                    if (i == 1) load_mine();
                    if (wv == 4) new_slot(i - 1, true);
                    else inherited(i - 1);
                }
                __syncthreads();
                if (pub[i & 1].slot == -2) {
                    const uint64_t ks = rescan_pass(i, wb);
                    if (wv == 4) rescan_tail(i, ks);
                    __syncthreads();  // R5
                }
            }
            if ((wv == 4 || wv == 7) && kend == 1) load_mine();
            if (wv == 4) new_slot(kend - 1, false);
            if (wv == 7)
                for (uint32_t j = kend - 1; 2 * j < ndi; ++j) inherited(j);  // (short windows: the rest)
            __syncthreads();  // B2 (D's slot ranks)
            for (uint32_t idx = id0; idx < knext * 64; idx += 256) {
                const uint32_t qq = idx >> 6, l = idx & 63u, r = xrank[l];
                if (r != 0xFFFFFFFFu) Tcur[qq * kResTStride + r] = Tnext[qq * kResTStride + l];
            }
            ndi = (uint32_t)__popcll(__ballot(xrank[lane] != 0xFFFFFFFFu));
            __syncthreads();  // B3
        }
    }
    if (kResDiag && rdiag && lane == 0 && wv < 4) {
        rdiag[8 + wv] = busy_;
        if (wv == 1) { rdiag[21] = sub_[0]; rdiag[22] = sub_[1]; }
        if (wv == 3) { rdiag[23] = sub_[0]; rdiag[24] = sub_[1]; rdiag[25] = sub_[2]; }
        if (wv == 0) rdiag[26] = sub_[0];
        if (wv == 0) rdiag[12] = steps_;
    }
    if (rdiag && lane == 0 && wv == 0)
        for (int k = 0; k < 5; ++k) rdiag[27 + k] = bseg_[k];
    if (rdiag && lane == 0 && wv == 0) rdiag[38] = bseg_[5];
    if (rdiag && lane == 0 && (wv == 1 || wv == 3)) rdiag[wv == 1 ? 37 : 36] = bseg_[0];
}
#undef QS_RSTAMP_BEGIN
#undef QS_RSTAMP_END

template <uint32_t F, int E, int E2, bool K32>
__global__ __launch_bounds__(kResBS) void k_la_stream_res(DevTable t, const PodT<F> *__restrict__ pods, DevCfg c,
                                                       uint32_t P, uint32_t K, uint32_t G, uint32_t L,
                                                       uint32_t chunk, uint32_t nwin, uint64_t *lists0,
                                                       uint64_t *clists0, uint32_t lwords, uint32_t cwords,
                                                       int32_t *__restrict__ out_node,
                                                       uint64_t *__restrict__ out_key,
                                                       uint64_t *__restrict__ stamps, ResCtl *ctl,
                                                       uint64_t *__restrict__ rdiag, const DPodX *__restrict__ podx,
                                                       uint4 *npart0, NormInfo *norm0, uint32_t *stat0,
                                                       unsigned long long *nfall, ResShard rsh) {
    if (blockIdx.x != 0) {
        res_selector<E, E2, F>(t, pods, c, P, K, G, L, chunk, nwin, lists0, clists0, lwords, cwords, ctl,
                               blockIdx.x - 1, gridDim.x - 1, rdiag, podx, npart0, norm0, stat0, rsh);
        return;
    }
    if (rsh.W > 1 && threadIdx.x == 0)  // this rank is in its new run: peers may write its mailbox
        for (uint32_t r = 0; r < rsh.W; ++r)
            __hip_atomic_store(reinterpret_cast<uint64_t *>(rsh.peers[r] + rsh.hello) + rsh.rank, rsh.seq,
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if ((F & kFeatNorm) == 0 && threadIdx.x >= 384) {
        // waves 6-7 (waves 4-5 fill the entry / row rings): the same barrier count (1 + per window kend + 3)
        __syncthreads();
        for (uint32_t w = 0; w < nwin; ++w)
            for (uint32_t j = 0, nb = min(K, P - w * K) + 3; j < nb; ++j) __syncthreads();
        return;
    }
    const uint64_t t0 = rdiag ? __builtin_amdgcn_s_memrealtime() : 0ull;
    la_resolve4_stream<F, K32>(lds, t, pods, c, P, K, nwin, lists0, lwords, out_node, out_key, stamps, ctl, rdiag,
                               podx, norm0, stat0, nfall);
    if (rdiag && threadIdx.x == 0) { rdiag[1] = __builtin_amdgcn_s_memrealtime() - t0; rdiag[3] = nwin; }
}

// Dynamic LDS above 64 KiB (the normalizing resident stream's statics) needs the per-kernel limit
// raised before the launch and before the occupancy query.
static hipError_t res_lds_attr(const void *fn, size_t lds4) {
    if (lds4 <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds4);
}
template <uint32_t F>
static hipError_t la_stream_res_f(const DevTable &t, const void *pods, const DPodX *podx, const DevCfg &c, uint32_t P,
                                  const LaGeom &geo, uint64_t *lists0, uint64_t *clists0, uint32_t lwords,
                                  uint32_t cwords, uint4 *npart0, NormInfo *norm0, uint32_t *stat0,
                                  unsigned long long *nfall, int32_t *on, uint64_t *ok, uint64_t *st, void *ctl,
                                  uint32_t sel_blocks, uint64_t *rdiag, const ResShard &rsh, hipStream_t stream) {
    const uint32_t K = geo.K, G = geo.G, L = geo.L, nwin = (P + K - 1) / K;
    // sharded: W * L <= 512 keys per cross merge, K <= 32 pods per slot
    if (rsh.W > 1 && (rsh.W * L > (uint32_t)kResBS || K > 32 || rsh.W > 16 || !rsh.peers))
        return hipErrorInvalidValue;
    const uint32_t E2 = geo.e2;  // a pod's G*L <= 512 * E2 chunk keys, E2 per merging thread
    if (G * L > E2 * (uint32_t)kResBS || (E2 == 2 && (F & kFeatNorm))) return hipErrorInvalidValue;
    const size_t lds4 = res_stream_lds_bytes<F>(t.n);
    if (lds4 > kResLdsMax) return hipErrorInvalidValue;
    // NORM: K <= kResNormK staged records per window, and a task per workgroup (the G chunks of a
    // pod wait for each other's partial maxima)
    if ((F & kFeatNorm) && (K > kResNormK || sel_blocks < K * G || !podx || !npart0 || !norm0 || !stat0))
        return hipErrorInvalidValue;
    const dim3 grid(1 + sel_blocks);
    const PodT<F> *pp = (const PodT<F> *)pods;
    ResCtl *rc = (ResCtl *)ctl;
#define QS_RESK(EE, EE2, KK)                                                                                          \
    do {                                                                                                              \
    if (hipError_t ea = res_lds_attr((const void *)k_la_stream_res<F, EE, EE2, KK>, lds4); ea != hipSuccess) return ea; \
    hipLaunchKernelGGL((k_la_stream_res<F, EE, EE2, KK>), grid, dim3(kResBS), lds4, stream, t, pp, c, P, K, G, L,       \
                       geo.chunk, nwin, lists0, clists0, lwords, cwords, on, ok, st, rc, rdiag, podx, npart0, norm0,   \
                       stat0, nfall, rsh);                                                                       \
    } while (0)
#define QS_RESE(EE, EE2) \
    else if (geo.E == EE && E2 == EE2) { if (geo.k32) QS_RESK(EE, EE2, true); else QS_RESK(EE, EE2, false); }
// two keys per merging thread: Fit + Balanced (+ext) instantiations only (normalizing profiles keep G <= 8)
#define QS_RESE2(EE) \
    else if (geo.E == EE && E2 == 2 && (F & kFeatNorm) == 0) { \
        if constexpr ((F & kFeatNorm) == 0) { if (geo.k32) QS_RESK(EE, 2, true); else QS_RESK(EE, 2, false); } }
    if (false) {
    }
    QS_RESE(3, 1) QS_RESE(5, 1) QS_RESE(7, 1) QS_RESE(8, 1) QS_RESE(16, 1)
    QS_RESE2(5) QS_RESE2(7) QS_RESE2(8) QS_RESE2(16)
    else return hipErrorInvalidValue;
#undef QS_RESE
#undef QS_RESE2
#undef QS_RESK
    return hipGetLastError();
}
constexpr size_t kResCtlBytes = sizeof(ResCtl);

// Workgroups of the instantiation la_stream_res_f would launch that the occupancy API admits per
// CU (every workgroup of the launch carries the resolver's dynamic LDS); 0 if not instantiated.
template <uint32_t F>
static int la_stream_res_per_cu(const LaGeom &geo, uint32_t n) {
    const size_t lds4 = res_stream_lds_bytes<F>(n);
    const void *fn = nullptr;
#define QS_RESP(EE, KK) \
    if (geo.E == EE && geo.e2 == 1 && (geo.k32 != 0) == KK) fn = (const void *)k_la_stream_res<F, EE, 1, KK>;
    QS_RESP(3, true) QS_RESP(3, false) QS_RESP(5, true) QS_RESP(5, false) QS_RESP(7, true) QS_RESP(7, false)
    QS_RESP(8, true) QS_RESP(8, false) QS_RESP(16, true) QS_RESP(16, false)
#undef QS_RESP
    if constexpr ((F & kFeatNorm) == 0) {
#define QS_RESP2(EE, KK) \
        if (geo.E == EE && geo.e2 == 2 && (geo.k32 != 0) == KK) fn = (const void *)k_la_stream_res<F, EE, 2, KK>;
        QS_RESP2(5, true) QS_RESP2(5, false) QS_RESP2(7, true) QS_RESP2(7, false) QS_RESP2(8, true) QS_RESP2(8, false) QS_RESP2(16, true) QS_RESP2(16, false)
#undef QS_RESP2
    }
    int per = 0;
    if (!fn || res_lds_attr(fn, lds4) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kResBS, lds4) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return per;
}

// =============================================================================================
// BATCHED mode (spec S11): per batch of B <= 64 pods, k_la_select + k_la_merge give each pod its
// 64 best keys against the batch-start table; k_batch_claim walks the batch in queue order, each
// pod claiming its best key whose node (and, for zone anti-affinity, whose (app, zone)) no earlier
// pod of the batch claimed, then applies every claim (Reserve + anti-affinity state) and builds
// the next batch: the pods that found no free candidate first, then fresh pods from the stream.
// ctrl = {pods in the batch, stream cursor}.
// =============================================================================================
#ifdef QS_CLAIM_DIAG
static __device__ uint64_t g_claim_diag[5];
#define CLAIM_STAMP0() uint64_t cds[4] = {0, 0, 0, 0}; uint64_t ctp = diag_stamp();
#define CLAIM_STAMP(q) { const uint64_t t_ = diag_stamp(); cds[q] += t_ - ctp; ctp = t_; }
#else
#define CLAIM_STAMP0()
#define CLAIM_STAMP(q)
#endif
constexpr int kClaimWaves = 16;
constexpr uint32_t kClaimNonEmpty = 1u << 31;  // staged pod flag: the pod's list holds a feasible node
constexpr uint32_t kClaimCarried = 64, kClaimNone = 65;  // walk outcomes beside a source lane 0..63
// LDS layout of k_batch_claim (bytes): the fixed-size arrays first, so that every address the walk
// forms is a lane offset plus a compile-time immediate; the node bitmap (one extra all-ones word
// that invalid entries point at) last.
constexpr uint32_t kClLkey = 0, kClLnode = kClLkey + 64 * 64 * 8, kClLazb = kClLnode + 64 * 64 * 4,
                   kClAz = kClLazb + 64 * 64 * 4, kClPend = kClAz + kMaxApps * kMaxZones / 8, kClSrc = kClPend + 256,
                   kClPod = kClSrc + 256, kClNodes = kClPod + 512;
__host__ __device__ constexpr size_t batch_claim_lds_bytes(uint32_t n) {
    return kClNodes + (((size_t)n + 31) / 32 + 1 + 3) / 4 * 16;
}

template <uint32_t F>
__global__ __launch_bounds__(64 * kClaimWaves) void k_batch_claim(
    DevTable t, const PodT<F> *__restrict__ pods, const uint64_t *__restrict__ lists, uint32_t GLp,
    uint32_t *ctrl, uint32_t *bidx, uint32_t P, uint32_t B, int32_t *__restrict__ out_node,
    uint64_t *__restrict__ out_key) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    CLAIM_STAMP0();
    const uint32_t nwords = (t.n + 31) / 32, sent = nwords * 32;  // sent: the all-ones bitmap word
    uint8_t *lb = reinterpret_cast<uint8_t *>(lds);
    uint64_t *lkey = reinterpret_cast<uint64_t *>(lb + kClLkey);  // [64 pods][64] keys, best first
    uint32_t *lnode = reinterpret_cast<uint32_t *>(lb + kClLnode);  // their nodes (sent: no entry)
    uint32_t *lazb = reinterpret_cast<uint32_t *>(lb + kClLazb);    // app * kMaxZones + zone
    uint32_t *claimed_az = reinterpret_cast<uint32_t *>(lb + kClAz);  // (app, zone) bitmap
    uint32_t *pend = reinterpret_cast<uint32_t *>(lb + kClPend);    // carried pods (<= 64)
    uint32_t *rsrc = reinterpret_cast<uint32_t *>(lb + kClSrc);     // [64] walk outcomes
    uint32_t *lpod = reinterpret_cast<uint32_t *>(lb + kClPod);     // [64] stream positions, [64] flags
    uint32_t *claimed = reinterpret_cast<uint32_t *>(lb + kClNodes);  // node bitmap
    const uint32_t nb = ctrl[0], cursor = ctrl[1];
    for (uint32_t i = tid; i < nwords; i += 64 * kClaimWaves) claimed[i] = 0;
    if (tid == 0) claimed[nwords] = 0xFFFFFFFFu;
    for (uint32_t i = tid; i < kMaxApps * kMaxZones / 32; i += 64 * kClaimWaves) claimed_az[i] = 0;
    // Staging, all waves: each pod's list, sorted best-first by the merge (so that a pod's claim is
    // the first still-available lane) as keys, nodes and, for zone-anti-affinity pods, the (app, zone)
    // bit of every candidate.  Wave wv takes pods wv + 16q (q < 4, all 64 rows written: rows past the
    // batch hold no entry): all loads of a round are issued before any is used.
    {
        constexpr int Q = 64 / kClaimWaves;
        uint64_t ev[Q];
        uint32_t fv[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t i = (uint32_t)wv + kClaimWaves * q;
            ev[q] = i < nb ? lists[(size_t)i * GLp + lane] : 0ull;
            fv[q] = i < nb ? bidx[i] : 0u;
        }
        uint32_t sv[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            sv[q] = fv[q];
            fv[q] = (uint32_t)wv + kClaimWaves * q < nb ? pods[sv[q]].flags : 0u;
        }
        uint32_t zv[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q)
            zv[q] = (ev[q] && pod_aa(fv[q]) == 2u) ? (uint32_t)t.zone[key_node(ev[q])] : 0u;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t i = (uint32_t)wv + kClaimWaves * q;
            const bool ok = ev[q] != 0ull;
            lkey[i * 64 + lane] = ev[q];
            lnode[i * 64 + lane] = ok ? key_node(ev[q]) : sent;
            lazb[i * 64 + lane] = pod_app(fv[q]) * kMaxZones + (zv[q] & (kMaxZones - 1));
            const uint32_t ne = __ballot(ok) ? kClaimNonEmpty : 0u;
            if (lane == 0) { lpod[i] = sv[q]; lpod[64 + i] = fv[q] | ne; }
        }
    }
    __syncthreads();
    if (wv != 0) return;
    CLAIM_STAMP(0);  // the claim walk and the apply step are one wave's work
    uint32_t npend = 0;
    // lane i holds batch pod i's stream position and flags (read with readlane in the walk)
    const uint32_t my_s = (uint32_t)lane < nb ? lpod[lane] : 0u;
    const uint32_t my_flags = lpod[64 + lane];
    CLAIM_STAMP(1);
    // Software-pipelined walk, one pod per step.  Entering step i: pod i's entries (node, (app, zone)
    // per lane) and its exact availability mask am (claims of pods < i), pod i+1's entries.  Pod
    // i+1's bitmap words are read before pod i's claim is written (they see the claims of pods < i)
    // and then patched with pod i's claim, so the LDS round trip overlaps pod i's scalar chain.
    // Invalid entries point at the all-ones word (always taken); a step records only pod i's source
    // lane (or carried / none), the keys are gathered after the walk.  Three entry register sets
    // rotate over an unrolled-by-3 loop (a copy at the back-edge would wait for the next load).
    struct Ents {
        uint32_t node, azb;
    };
    auto ents = [&](uint32_t j) -> Ents {
        const uint32_t o = min(j, 63u) * 64 + (uint32_t)lane;
        return Ents{lnode[o], lazb[o]};
    };
    Ents sa = ents(0), sb = ents(1), sc{sent, 0u};
    uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)my_flags, 0);
    uint64_t am;
    {
        uint32_t tk = (claimed[sa.node >> 5] >> (sa.node & 31)) & 1u;
        am = __ballot(tk == 0u);  // no claims yet: only the invalid entries are taken
    }
    auto step = [&](uint32_t i, const Ents &cur, const Ents &nxt, Ents &n2) {
        const uint32_t fl1 = (uint32_t)__builtin_amdgcn_readlane((int)my_flags, (int)min(i + 1, 63u));
        const bool aa = pod_aa(fl) == 2u, aa1 = pod_aa(fl1) == 2u;
        // pod i+1: bitmap words (claims of pods < i) and pod i+2's entries, all in flight now
        const uint32_t cw1 = claimed[nxt.node >> 5];
        const uint32_t aw1 = aa1 ? claimed_az[nxt.azb >> 5] : 0u;
        n2 = ents(i + 2);
        // pod i
        uint32_t w = 0xFFFFFFFFu, bw = 0xFFFFFFFFu;
        if (am) {
            const int src = __builtin_ctzll(am);
            w = (uint32_t)__builtin_amdgcn_readlane((int)cur.node, src);
            if (aa) bw = (uint32_t)__builtin_amdgcn_readlane((int)cur.azb, src);
            if (lane == 0) {
                __hip_atomic_fetch_or(&claimed[w >> 5], 1u << (w & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                if (aa)
                    __hip_atomic_fetch_or(&claimed_az[bw >> 5], 1u << (bw & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                rsrc[i] = (uint32_t)src;
            }
        } else if (fl & kClaimNonEmpty) {  // every candidate taken by an earlier pod: carried
            if (lane == 0) {
                pend[npend] = (uint32_t)__builtin_amdgcn_readlane((int)my_s, (int)i);
                rsrc[i] = kClaimCarried;
            }
            ++npend;
        } else if (lane == 0) {
            rsrc[i] = kClaimNone;  // no feasible node at all (spec S7: unschedulable)
        }
        // pod i+1's exact mask: bitmap words patched with pod i's claim
        uint32_t tk = (cw1 >> (nxt.node & 31)) & 1u;
        if (aa1) tk |= ((aw1 >> (nxt.azb & 31)) & 1u) | ((aa && nxt.azb == bw) ? 1u : 0u);
        am = __ballot(tk == 0u && nxt.node != w);
        fl = fl1;
    };
    uint32_t i = 0;
    for (; i + 2 < nb; i += 3) {
        step(i, sa, sb, sc);
        step(i + 1, sb, sc, sa);
        step(i + 2, sc, sa, sb);
    }
    if (i < nb) step(i, sa, sb, sc);
    if (i + 1 < nb) step(i + 1, sb, sc, sa);
    CLAIM_STAMP(2);
    // lane i: batch pod i's outcome (-2 carried, -1 unschedulable) and its key
    int32_t my_node = -2;
    uint64_t my_key = 0;
    if ((uint32_t)lane < nb) {
        const uint32_t r = rsrc[lane];
        if (r < 64u) {
            my_key = lkey[(uint32_t)lane * 64 + r];
            my_node = (int32_t)key_node(my_key);
        } else {
            my_node = r == kClaimCarried ? -2 : -1;
        }
    }
    // apply every claim (distinct nodes; counts of one (app, zone) may be shared: atomics)
    if ((uint32_t)lane < nb && my_node != -2) {
        const uint32_t s = my_s;
        if (my_node >= 0) {
            const PodT<F> p = pods[s];
            const uint32_t w = (uint32_t)my_node;
            RowT<F> r = load_row<F>(t, w);
            RowX x = load_rowx<F>(t, w);
            reserve(r, x, p, +1);
            store_dyn<F>(t, w, r);
            store_dynx<F>(t, w, x);
            if (t.apps) {
                const uint32_t app = pod_app(p.flags);
                atomicOr(&t.apps[(size_t)(app >> 5) * t.cap + w], 1u << (app & 31));
                atomicAdd(&t.zcount[app * kMaxZones + (uint32_t)t.zone[w]], 1);
            }
        }
        out_node[s] = my_node;
        if (out_key) out_key[s] = my_key;
    }
    // next batch: carried pods first (queue order), then fresh pods from the stream.  bidx is
    // rewritten only after every lane has read its entry above (single wave, program order).
    const uint32_t take = min(B - npend, P - cursor);
    if ((uint32_t)lane < npend) bidx[lane] = pend[lane];
    else if ((uint32_t)lane < npend + take) bidx[lane] = cursor + (uint32_t)lane - npend;
    if (lane == 0) { ctrl[0] = npend + take; ctrl[1] = cursor + take; }
    CLAIM_STAMP(3);
#ifdef QS_CLAIM_DIAG
    if (lane == 0) {
        for (int q = 0; q < 4; ++q) atomicAdd((unsigned long long *)&g_claim_diag[q], (unsigned long long)cds[q]);
        const unsigned long long nbt = atomicAdd((unsigned long long *)&g_claim_diag[4], 1ull);
        if (npend + take == 0)
            printf("claim diag: batches %llu  stage %llu  setup %llu  walk %llu  apply %llu (clocks, totals)\n",
                   nbt + 1, (unsigned long long)g_claim_diag[0], (unsigned long long)g_claim_diag[1],
                   (unsigned long long)g_claim_diag[2], (unsigned long long)g_claim_diag[3]);
    }
#endif
}


// =============================================================================================
// templated launchers (one set of instantiations per layout translation unit)
// =============================================================================================
#define QS_RET(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

template <int NPT, int BS, uint32_t F>
static hipError_t persistent_t(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P,
                               const DevCfg &c, int32_t *on, uint64_t *ok, uint64_t *st,
                               hipStream_t stream) {
    hipLaunchKernelGGL((k_persistent<NPT, BS, F>), dim3(1), dim3(BS), 0, stream, t,
                       (const PodT<F> *)pods, podx, P, c, on, ok, st);
    return hipGetLastError();
}

// Largest node count per feature set for the register-resident rows (1024 threads, 4 waves/SIMD;
// the largest NPT of each set spills a few dwords to scratch: correct, slower — the LOOKAHEAD
// engine is the fast path at these sizes).  Wide rows carry three f64 memory columns.
template <uint32_t F>
static constexpr uint32_t persistent_cap() {
    if (F & kFeatWide) return (F & kFeatNorm) ? 2048u : 5120u;
    return F == 0 ? 6144u : (F == kFeatExt ? 5120u : 2048u);
}

template <uint32_t F>
static hipError_t persistent_f(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P,
                               const DevCfg &c, int32_t *on, uint64_t *ok, uint64_t *st,
                               hipStream_t stream) {
    const uint32_t n = t.n;
    if (n > persistent_cap<F>()) return hipErrorInvalidValue;
    if (n <= 64) return persistent_t<1, 64, F>(t, pods, podx, P, c, on, ok, st, stream);
    if (n <= 128) return persistent_t<1, 128, F>(t, pods, podx, P, c, on, ok, st, stream);
    if (n <= 256) return persistent_t<1, 256, F>(t, pods, podx, P, c, on, ok, st, stream);
    if (n <= 512) return persistent_t<1, 512, F>(t, pods, podx, P, c, on, ok, st, stream);
    if (n <= 1024) return persistent_t<1, 1024, F>(t, pods, podx, P, c, on, ok, st, stream);
    if (n <= 2048) return persistent_t<2, 1024, F>(t, pods, podx, P, c, on, ok, st, stream);
    if constexpr (persistent_cap<F>() > 2048) {
        if (n <= 3072) return persistent_t<3, 1024, F>(t, pods, podx, P, c, on, ok, st, stream);
        if (n <= 4096) return persistent_t<4, 1024, F>(t, pods, podx, P, c, on, ok, st, stream);
    }
    if constexpr (persistent_cap<F>() > 4096) {
        if (n <= 5120) return persistent_t<5, 1024, F>(t, pods, podx, P, c, on, ok, st, stream);
    }
    if constexpr (persistent_cap<F>() > 5120) {
        if (n <= 6144) return persistent_t<6, 1024, F>(t, pods, podx, P, c, on, ok, st, stream);
    }
    return hipErrorInvalidValue;
}

template <uint32_t F>
static hipError_t scan_pod_f(const DevTable &t, const void *pods_, const DPodX *podx, uint32_t s,
                             const DevCfg &c, void *scratch, int32_t *on, uint64_t *ok,
                             uint64_t *st, uint8_t *feas, int32_t *score, int32_t *total,
                             int part, hipStream_t stream) {
    const PodT<F> *pods = (const PodT<F> *)pods_;
    ScanScratch *sc = (ScanScratch *)scratch;
    // the column-major copy exists for compact-layout tables only
    constexpr bool kSoaOk = (F & (kFeatNorm | kFeatWide)) == 0;
    const bool soa = kSoaOk && t.soa.c[0];
    // one partial key per block; a grid of <= 2048 blocks (8 four-wave blocks per CU) strides
    const uint32_t units = soa ? (t.n + 3) / 4 : t.n;
    uint32_t blocks = min(kScanBlocksMax, max(1u, (units + 255) / 256));
    if (part & 1) {
        if constexpr (kSoaOk) {
            if (soa) {
                // SoA scan: exactly one resident wave of blocks (CUs x blocks per CU at this
                // kernel's occupancy), so no CU runs a second, partial round at the end of the scan
                static const uint32_t resident = [] {
                    int dev = 0, cus = 0, per = 0;
                    if (hipGetDevice(&dev) != hipSuccess ||
                        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)k_scan_soa<F>, 256, 0) != hipSuccess)
                        return kScanBlocksMax;
                    const char *env = getenv("QS_SCAN_BLOCKS");
                    if (env && atoi(env) > 0) return (uint32_t)atoi(env);
                    return (uint32_t)std::max(1, std::min((int)kScanBlocksMax, cus * per));
                }();
                blocks = min(blocks, min(kScanBlocksMax, resident));
                hipLaunchKernelGGL((k_scan_soa<F>), dim3(blocks), dim3(256), 0, stream, t, pods, s, c, sc,
                                   feas, score, total);
            }
        }
        if (!soa) {
            if (F & kFeatNorm)
                hipLaunchKernelGGL((k_scan_norm<F>), dim3(blocks), dim3(256), 0, stream, t, pods, podx, s, sc);
            hipLaunchKernelGGL((k_scan_key<F>), dim3(blocks), dim3(256), 0, stream, t, pods, podx, s, c, sc,
                               feas, score, total);
        }
    }
    if (part & 2)
        hipLaunchKernelGGL((k_scan_commit<F>), dim3(1), dim3(256), 0, stream, t, pods, s, blocks, sc,
                           on, ok, st);
    // the per-pod all-reduce engine (rows over the scratch's node range, no SoA): 8 the normalize
    // maxima, 16 the keys, 32 their reduction into sc->best, 64 the commit of sc->best
    if (!soa) {
        if ((part & 8) && (F & kFeatNorm))
            hipLaunchKernelGGL((k_scan_norm<F>), dim3(blocks), dim3(256), 0, stream, t, pods, podx, s, sc);
        if (part & 16)
            hipLaunchKernelGGL((k_scan_key<F>), dim3(blocks), dim3(256), 0, stream, t, pods, podx, s, c, sc,
                               nullptr, nullptr, nullptr);
        if (part & 32)
            hipLaunchKernelGGL((k_scan_commit<F>), dim3(1), dim3(256), 0, stream, t, pods, s, blocks, sc,
                               nullptr, nullptr, nullptr);
        if (part & 64)
            hipLaunchKernelGGL((k_scan_commit<F>), dim3(1), dim3(256), 0, stream, t, pods, s, 0u, sc, on, ok, st);
    }
    return hipGetLastError();
}

template <uint32_t F>
static hipError_t score_pod1_f(const DevTable &t, const void *pod, const DPodX *podx, const DevCfg &c, uint8_t *hout,
                               uint64_t *gs, uint64_t seq, uint32_t pidx, const HostRow &prow, hipStream_t stream) {
    if (!gs && t.n > kScorePod1Max) return hipErrorInvalidValue;
    PodT<F> p;
    std::memcpy(&p, pod, sizeof p);
    DPodX px{};
    if ((F & kFeatNorm) && podx) px = *podx;
    if (gs && t.n > 0) {
        const uint32_t g = (t.n + kScorePodGT - 1) / kScorePodGT;
        if constexpr ((F & kFeatNorm) != 0)
            hipLaunchKernelGGL((k_score_podg_max<F>), dim3(g), dim3(kScorePodGT), 0, stream, t, p, px, gs, pidx,
                               prow);
        hipLaunchKernelGGL((k_score_podg<F>), dim3(g), dim3(kScorePodGT), 0, stream, t, p, px, c, hout, gs, seq,
                           pidx, prow);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_score_pod1<F>), dim3(1), dim3(1024), 0, stream, t, p, px, c, hout, seq, pidx, prow);
    return hipGetLastError();
}

template <uint32_t F>
static hipError_t la_window_f(const DevTable &t, const void *pods_, const DPodX *podx, uint32_t s0,
                              uint32_t P, const DevCfg &c, const LaGeom &geo, const LaBufs &bf,
                              int32_t *on, uint64_t *ok, uint64_t *st, uint64_t *diag,
                              hipStream_t stream, int part) {
    const PodT<F> *pods = (const PodT<F> *)pods_;
    const uint32_t K = geo.K, G = geo.G, L = geo.L, GLp = geo.eplr * 64;
    const uint32_t kw = min(K, P - s0);
    LaShard sh{geo.W, geo.v0, kw, 0u, (uint64_t)K * GLp};
    const dim3 grid(geo.nv * kw * G);
    if ((part & 4) && (F & kFeatNorm)) {
        switch (geo.E) {
#define QS_NRM(EE) case EE: hipLaunchKernelGGL((k_la_norm<256, EE, F>), grid, dim3(256), 0, stream, t, pods, podx, s0, P, sh, G, K, geo.chunk, bf.npart); break;
            QS_NRM(1) QS_NRM(2) QS_NRM(3) QS_NRM(4) QS_NRM(5) QS_NRM(6) QS_NRM(8) QS_NRM(10) QS_NRM(12) QS_NRM(16)
#undef QS_NRM
            default: return hipErrorInvalidValue;
        }
        QS_RET(hipGetLastError());
    }
    if (part & 1) {
        // batched mode: the merge inside the select launch (its G * L keys: two per thread)
        uint32_t *tickets = (bf.tickets && G > 1 && G * L <= 512) ? bf.tickets : nullptr;
        switch (geo.E) {
#define QS_SEL(EE) case EE: hipLaunchKernelGGL((k_la_select<256, EE, F>), grid, dim3(256), 0, stream, t, pods, podx, c, s0, P, sh, G, L, geo.chunk, GLp, bf.lists, bf.clists, bf.npart, K, bf.norm, bf.pidx, bf.pcount, tickets); break;
            QS_SEL(1) QS_SEL(2) QS_SEL(3) QS_SEL(4) QS_SEL(5) QS_SEL(6) QS_SEL(8) QS_SEL(10) QS_SEL(12) QS_SEL(16)
#undef QS_SEL
            default: return hipErrorInvalidValue;
        }
        QS_RET(hipGetLastError());
        if (G > 1 && !tickets) {
            const uint32_t M = G * L, e2 = (M + 255) / 256;
            const dim3 mgrid(geo.nv * kw);
            switch (e2) {
#define QS_MRG(EE) case EE: hipLaunchKernelGGL((k_la_merge<EE, (F & kFeatWide) != 0>), mgrid, dim3(256), 0, stream, bf.clists, M, L, sh, GLp, bf.lists); break;
                QS_MRG(1) QS_MRG(2) QS_MRG(3) QS_MRG(4) QS_MRG(5) QS_MRG(6) QS_MRG(7) QS_MRG(8)
#undef QS_MRG
                default: return hipErrorInvalidValue;
            }
            QS_RET(hipGetLastError());
        }
    }
    if (part & 2) {
        const size_t bm = (((t.n + 31) / 32 + 3) & ~3u) * 4;
        if constexpr ((F & kFeatNorm) != 0) {
            const size_t ldsn = bm + 64 * (sizeof(RowT<F>) + sizeof(RowX)) + sizeof(RowT<F>) + sizeof(RowX) + 64 * 4;
            if (geo.waves == 4) {
                // four-wave resolver with the maxima test; on a lost maximum it stops and the
                // single-wave kernel resumes the window from that pod (rescan included)
                if (geo.epl != 1 || !bf.rec) return hipErrorInvalidValue;
                const size_t lds4n = bm + 5 * 2 * 64 * 8 + 2 * 64 * (sizeof(RowT<F>) + sizeof(int4)) + 2 * sizeof(ResPub) +
                                     64 * 4 + 64 * sizeof(PodT<F>) + 64 * sizeof(DPodX) + 64 * sizeof(NormInfo) +
                                     64 * sizeof(double2) + 2 * 64 * 4 + 2 * 64 * sizeof(RowX);
                // (the resume of a stopped window runs inside the same launch: LDS for both)
                const size_t ldsr = std::max(lds4n, ldsn);
                if (diag)
                    hipLaunchKernelGGL((k_la_resolve4<F, 1, true, false>), dim3(1), dim3(256), ldsr, stream, t, pods, c, s0, P,
                                       K, GLp, geo.lr, sh, bf.lists, on, ok, st, diag, bf.dprev, bf.dcur, podx, bf.norm, bf.rec, bf.nfall);
                else if (geo.k32)
                    hipLaunchKernelGGL((k_la_resolve4<F, 1, false, true>), dim3(1), dim3(256), ldsr, stream, t, pods, c, s0, P,
                                       K, GLp, geo.lr, sh, bf.lists, on, ok, st, diag, bf.dprev, bf.dcur, podx, bf.norm, bf.rec, bf.nfall);
                else
                    hipLaunchKernelGGL((k_la_resolve4<F, 1, false, false>), dim3(1), dim3(256), ldsr, stream, t, pods, c, s0, P,
                                       K, GLp, geo.lr, sh, bf.lists, on, ok, st, diag, bf.dprev, bf.dcur, podx, bf.norm, bf.rec, bf.nfall);
                return hipGetLastError();
            }
            switch (geo.epl) {
#define QS_RESN(EP) case EP: hipLaunchKernelGGL((k_la_resolve_norm<F, EP>), dim3(1), dim3(64 * kResNormWaves), ldsn, stream, t, pods, podx, c, s0, P, K, GLp, geo.lr, sh, bf.lists, bf.norm, on, ok, st, bf.dprev, bf.dcur, bf.nfall, nullptr); break;
                QS_RESN(1) QS_RESN(2) QS_RESN(4) QS_RESN(8) QS_RESN(16)
#undef QS_RESN
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
        const uint64_t *lists = bf.lists;
        const uint32_t *dprev = bf.dprev;
        uint32_t *dcur = bf.dcur;
        const size_t lds = bm + sizeof(RowT<F>) + sizeof(RowX);
        const size_t lds4 = bm + 5 * 2 * 64 * 8 + 2 * 64 * (sizeof(RowT<F>) + sizeof(int4)) + 2 * sizeof(ResPub) + 64 * 4 + 64 * sizeof(PodT<F>);
        switch (geo.epl) {
#define QS_RES(EP) case EP: \
            if (geo.waves == 1) { \
                if (diag) hipLaunchKernelGGL((k_la_resolve<F, EP, true>), dim3(1), dim3(64), lds, stream, t, pods, c, s0, P, K, GLp, geo.lr, sh, lists, on, ok, st, diag); \
                else hipLaunchKernelGGL((k_la_resolve<F, EP, false>), dim3(1), dim3(64), lds, stream, t, pods, c, s0, P, K, GLp, geo.lr, sh, lists, on, ok, st, diag); \
            } else { \
                if (diag) hipLaunchKernelGGL((k_la_resolve4<F, EP, true, false>), dim3(1), dim3(256), lds4, stream, t, pods, c, s0, P, K, GLp, geo.lr, sh, lists, on, ok, st, diag, dprev, dcur, nullptr, nullptr, nullptr, nullptr); \
                else if (geo.k32) hipLaunchKernelGGL((k_la_resolve4<F, EP, false, true>), dim3(1), dim3(256), lds4, stream, t, pods, c, s0, P, K, GLp, geo.lr, sh, lists, on, ok, st, diag, dprev, dcur, nullptr, nullptr, nullptr, nullptr); \
                else hipLaunchKernelGGL((k_la_resolve4<F, EP, false, false>), dim3(1), dim3(256), lds4, stream, t, pods, c, s0, P, K, GLp, geo.lr, sh, lists, on, ok, st, diag, dprev, dcur, nullptr, nullptr, nullptr, nullptr); \
            } break;
            QS_RES(1) QS_RES(2) QS_RES(4) QS_RES(8) QS_RES(16)
#undef QS_RES
            default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}


template <uint32_t F>
static hipError_t batch_claim_prepare_f() {
    // raises the claim kernel's dynamic-LDS limit to the CU's 160 KB; called once, outside capture
    static const hipError_t attr = hipFuncSetAttribute((const void *)k_batch_claim<F>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return attr;
}

template <uint32_t F>
static hipError_t batch_claim_f(const DevTable &t, const void *pods, const uint64_t *lists, uint32_t *ctrl,
                                uint32_t *bidx, uint32_t P, uint32_t B, int32_t *on, uint64_t *ok,
                                size_t lds, hipStream_t stream) {
    hipLaunchKernelGGL((k_batch_claim<F>), dim3(1), dim3(64 * kClaimWaves), lds, stream, t, (const PodT<F> *)pods,
                       lists, 64u, ctrl, bidx, P, B, on, ok);
    return hipGetLastError();
}

// Wide-layout entry points (qs_kernels_wide.hip); the compact dispatchers in qs_kernels.hip call
// them when the table is wide (DevTable::wrows != nullptr).
hipError_t wide_persistent(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P,
                           const DevCfg &c, int32_t *on, uint64_t *ok, uint64_t *st, hipStream_t stream);
uint32_t wide_persistent_max_nodes(uint32_t feat);
hipError_t wide_scan_pod(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s,
                         const DevCfg &c, void *scratch, int32_t *on, uint64_t *ok, uint64_t *st,
                         uint8_t *feas, int32_t *score, int32_t *total, int part, hipStream_t stream);
hipError_t wide_la_window(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s0,
                          uint32_t P, const DevCfg &c, const LaGeom &geo, const LaBufs &bf,
                          int32_t *on, uint64_t *ok, uint64_t *st, uint64_t *diag,
                          hipStream_t stream, int part);
hipError_t wide_batch_claim_prepare();
hipError_t wide_score_pod1(const DevTable &t, const void *pod, const DPodX *podx, const DevCfg &c, uint8_t *hout,
                           uint64_t *gs, uint64_t seq, uint32_t pidx, const HostRow &prow, hipStream_t stream);
hipError_t wide_batch_claim(const DevTable &t, const void *pods, const uint64_t *lists, uint32_t *ctrl,
                            uint32_t *bidx, uint32_t P, uint32_t B, int32_t *on, uint64_t *ok,
                            size_t lds, hipStream_t stream);
hipError_t wide_la_stream_res(const DevTable &t, const void *pods, const DPodX *podx, const DevCfg &c, uint32_t P,
                              const LaGeom &geo, uint64_t *lists0, uint64_t *clists0, uint32_t lwords, uint32_t cwords,
                              uint4 *npart, NormInfo *norm, uint32_t *stat, unsigned long long *nfall, int32_t *on,
                              uint64_t *ok, uint64_t *st, void *ctl, uint32_t sel_blocks, uint64_t *rdiag,
                              const ResShard &rsh, hipStream_t stream);
int wide_la_stream_res_per_cu(const LaGeom &geo, uint32_t feat, uint32_t n);

// Configurable-scoring-resource entry points (kFeatRes; qs_kernels_res.inc, one translation unit per
// row layout: res_compact_* and res_wide_*).
#define QS_DECL_RES(P)                                                                                        \
    hipError_t P##persistent(const DevTable &t, const void *pods, const DPodX *podx, uint32_t P_,            \
                             const DevCfg &c, int32_t *on, uint64_t *ok, uint64_t *st, hipStream_t stream);   \
    uint32_t P##persistent_max_nodes(uint32_t feat);                                                          \
    hipError_t P##scan_pod(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s,               \
                           const DevCfg &c, void *scratch, int32_t *on, uint64_t *ok, uint64_t *st,           \
                           uint8_t *feas, int32_t *score, int32_t *total, int part, hipStream_t stream);      \
    hipError_t P##score_pod1(const DevTable &t, const void *pod, const DPodX *podx, const DevCfg &c,         \
                             uint8_t *hout, uint64_t *gs, uint64_t seq, uint32_t pidx, const HostRow &prow,   \
                             hipStream_t stream);                                                             \
    hipError_t P##la_window(const DevTable &t, const void *pods, const DPodX *podx, uint32_t s0, uint32_t P_, \
                            const DevCfg &c, const LaGeom &geo, const LaBufs &bf, int32_t *on, uint64_t *ok,  \
                            uint64_t *st, uint64_t *diag, hipStream_t stream, int part);                     \
    hipError_t P##la_stream_res(const DevTable &t, const void *pods, const DPodX *podx, const DevCfg &c,     \
                                uint32_t P_, const LaGeom &geo, uint64_t *lists0, uint64_t *clists0,         \
                                uint32_t lwords, uint32_t cwords, uint4 *npart, NormInfo *norm,               \
                                uint32_t *stat, unsigned long long *nfall, int32_t *on, uint64_t *ok,         \
                                uint64_t *st, void *ctl, uint32_t sel_blocks, uint64_t *rdiag,                \
                                const ResShard &rsh, hipStream_t stream);                                     \
    int P##la_stream_res_per_cu(const LaGeom &geo, uint32_t feat, uint32_t n);
QS_DECL_RES(res_compact_)
QS_DECL_RES(res_wide_)
#undef QS_DECL_RES

}  // namespace qs
