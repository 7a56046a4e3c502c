// qs_device.hpp — device-side data layout and the per-(pod, node) evaluation shared by every
// gfx950 kernel of libqsched.  Semantics: spec/semantics.md (S4–S7); exactness arguments: S10.
//
// Layout in HBM: the node table is an array of 64-byte rows of int32 fields in
// compacted units (cpu millicores, memory 2^u bytes) plus per-node reciprocals RN_f64(1/alloc)
// precomputed at load time, and a parallel array of 32-byte taint/label mask rows.
// Everything here is compiled with -ffp-contract=off: the float64 path must round exactly like
// Go's float64 (spec S5, kat K7).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <type_traits>

namespace qs {

constexpr int kWave = 64;
#define QS_BAL_MAX 4  // entries of the BalancedAllocation resource list (QS_MAX_SCORE_RES)

// ---- device node table: one 64-byte row per node (+ a 32-byte mask row) -----------------------
// Row-major so that a lane gathering one node (the resolver's candidate / dirty rows) touches one
// cache line with four 16-byte loads; a 64-lane scan over consecutive nodes still uses whole lines.
struct alignas(16) DRow {
    int32_t ac, am;          // Allocatable cpu (m), memory (2^u B)
    int32_t rc, rm;          // Requested
    int32_t zc, zm;          // NonZeroRequested
    int32_t np, mp;          // pod count, AllowedPodNumber
    double yc, ym;           // RN_f64(1/alloc) (0 where alloc == 0)
    int32_t ae0, re0, ae1, re1;  // extended resources
};
// Wide layout (spec S10 fallback): used when the table's memory quantities cannot
// be stored exactly as int32 multiples of 2^u bytes below 2^24 (odd-Ki kubelet allocatable,
// decimal "100M" requests).  Memory columns are f64 integers in bytes (exact below 2^53); cpu,
// pod counts and extended resources stay int32 as in DRow.  80 bytes.
// The fields a Reserve changes sit in q0 / q1 (and q4): the resident stream hands exactly those
// quads off write-through, as it does q0 / q1 / q3 of a compact row.
struct alignas(16) DRowW {
    int32_t rc, zc, np, ac;      // q0  Requested / NonZeroRequested cpu, pod count; Allocatable cpu
    double rm, zm;               // q1  Requested / NonZeroRequested memory (bytes)
    double am, ym;               // q2  Allocatable memory, RN_f64(1/am)
    double yc;                   // q3  RN_f64(1/ac)
    int32_t mp, pad;
    int32_t ae0, re0, ae1, re1;  // q4  extended resources
};
struct alignas(16) DMask {
    uint64_t th, ts;         // taint_hard, taint_soft
    uint64_t lb0, lb1;       // label requirement bits
};
// Column-major (SoA) copy of the int32 fields for HBM-resident tables (n >= kSoaMinNodes): the
// SCAN engine and qs_score_pod stream 4 nodes per lane with one 16-byte load per column, so a
// scan moves exactly the 32 algorithmic bytes per node.  Reciprocals are
// recomputed in registers.  c[0] == nullptr: no SoA copy.
enum SoaCol : int { kSAc, kSAm, kSRc, kSRm, kSZc, kSZm, kSNp, kSMp, kSAe0, kSRe0, kSAe1, kSRe1, kSCols };
struct DevSoa {
    int32_t *c[kSCols];
};
// Anti-affinity state of batched mode (spec S11): per node its topology zone, per (app, node) a
// presence bit (word-major: word w of node i at apps[w * cap + i], so a wave over consecutive
// nodes reads consecutive words), per (app, zone) a pod count.  apps == nullptr: not kept.
constexpr uint32_t kMaxApps = 1024, kMaxZones = 64, kAppWords = kMaxApps / 32;
struct DevTable {
    DRow *rows;       // compact layout (nullptr in the wide layout)
    DRowW *wrows;     // wide layout (nullptr in the compact layout)
    DMask *masks;
    uint32_t n;
    DevSoa soa;
    int32_t *zone;
    uint32_t *apps;
    int32_t *zcount;  // [kMaxApps][kMaxZones]
    uint32_t cap;     // row capacity (stride of the app words)
};

// kFeatWide selects the wide row / pod layout (DRowW, DPodW); the host sets it with kFeatExt.
// kFeatRes selects the configurable scoring-resource form of LeastAllocated / BalancedAllocation
// (spec S5 "Scoring resources": extended resources in the lists, lists other than {cpu, memory});
// the host sets it with kFeatExt.
enum FeatBits : uint32_t { kFeatTaint = 1u, kFeatAffinity = 2u, kFeatExt = 4u, kFeatWide = 8u, kFeatRes = 16u };

// pod flags: bits 0-1 QoS, 4-6 required terms, 8-10 preferred terms, 12-13 anti-affinity kind,
// 16-25 app group (spec S11)
__device__ __forceinline__ uint32_t pod_aa(uint32_t flags) { return (flags >> 12) & 3u; }
__device__ __forceinline__ uint32_t pod_app(uint32_t flags) { return (flags >> 16) & 1023u; }
// Required anti-affinity of a batched-mode pod against node i (state at batch start).
__device__ __forceinline__ bool aa_ok(const DevTable &t, uint32_t flags, uint32_t i) {
    const uint32_t aa = pod_aa(flags), app = pod_app(flags);
    if (aa == 1u) return !((t.apps[(size_t)(app >> 5) * t.cap + i] >> (app & 31u)) & 1u);
    if (aa == 2u) return t.zcount[app * kMaxZones + (uint32_t)t.zone[i]] == 0;
    return true;
}

// Profile constants resolved on the host.
struct DevCfg {
    int32_t wc, wm;              // LeastAllocated resource weights
    double yd_both, yd_c, yd_m;  // RN_f64(1 / weight sums)
    int32_t wtt, wna;            // TaintToleration / NodeAffinity plugin weights
    uint32_t feat;               // kFeat* bits
    uint32_t ba_skip_be;         // balanced_skip_besteffort
    // kFeatRes only: LeastAllocated weights of the extended resources (0 = not in the list; wc / wm
    // likewise for cpu / memory) and the BalancedAllocation list in order, 4 bits per entry
    // (1 cpu, 2 memory, 3 ext0, 4 ext1; 0 ends the list)
    int32_t we0, we1;
    uint32_t bal;
    // Overlapped lookahead windows: the resolver of window w waits in-kernel for
    // ready >= (epoch << 32 | w + 1), published by k_ready_set after window w's select chain,
    // instead of a cross-stream event per window.  nullptr: no wait (the launch is ordered).
    const uint64_t *ready;
    uint64_t epoch;  // the run's sequence number (host counter)
    uint32_t *werr;  // set to 1 when a wait times out (the run returns QS_ETIMEOUT)
    // Test hook (QS_INJECT_FAULT=resident_stall, tests/test_gpu_recovery.py): 1 = the selectors of
    // the resident stream never deliver window 3's first task, so the resolver's wait times out
    // and the in-kernel werr drain runs for real.  0 in every normal run.
    uint32_t inject;
    // Bound (s_memrealtime ticks, 100 MHz) of the resident stream's waits in its first window, whose
    // producers may be a peer rank still in host-side prepare (sharded: 5 s, as the per-window
    // mailbox wait, qs_dist.cpp); 0 = the 0.5 s bound of every later wait.
    uint64_t first_ticks;
    // QS_RES_DIAG=1: the resident selectors time their phases too (extra barriers); =2: the
    // resolver's counters only, selectors untouched
    uint32_t sel_diag;
};

// Resolver prologue: thread 0 spins (s_sleep) until window s0/K's lists are published, then every
// thread proceeds.  Bounded: after 0.5 s (s_memrealtime, 100 MHz) it records a timeout; once one is
// recorded no later resolver of the run waits (a profiler that serialises dispatches across streams
// would otherwise cost the bound per window), and the run returns QS_ETIMEOUT.
__device__ __forceinline__ void wait_lists_ready(const DevCfg &c, uint32_t s0, uint32_t K) {
    if (c.ready == nullptr) return;
    if (threadIdx.x == 0 && __hip_atomic_load(c.werr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        const uint64_t want = (c.epoch << 32) | (uint64_t)(s0 / K + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(c.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {
                __hip_atomic_store(c.werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

// Pod record (32 B).  w_fit / w_bal already resolved from the pod's QoS class (spec S9).
struct alignas(16) DPod {
    int32_t rc, rm, zc, zm;   // Requested / NonZeroRequested cpu, memory (compacted)
    int32_t re0, re1;         // extended requests
    uint16_t wfit, wbal;
    uint32_t flags;           // bits 0-1 qos, 4-6 n_req_terms, 8-10 n_pref_terms
};
// Pod record of the wide layout (48 B): memory requests as f64 bytes.
struct alignas(16) DPodW {
    int32_t rc, zc, re0, re1;
    uint16_t wfit, wbal;
    uint32_t flags;
    uint32_t pad0, pad1;
    double rm, zm;
};
// Config-4 extension record (176 B), only read when kFeatTaint|kFeatAffinity.
struct alignas(16) DPodX {
    uint64_t tol_hard, tol_soft, sel0, sel1;
    uint64_t req[4][2];
    uint64_t pref[4][2];
    int32_t pw[4];
};

// Load a wave-uniform record through the vector path (VGPRs).  The pod extension record is 44
// dwords; read with scalar loads it pushed the normalizing kernels into SGPR spills.  The zero
// offset comes from an opaque VGPR so the compiler cannot prove uniformity.
template <class T>
__device__ __forceinline__ T load_vgpr(const T *p) {
    static_assert(sizeof(T) % 16 == 0, "16-byte granules");
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    const int4 *q = reinterpret_cast<const int4 *>(p) + z;
    T out;
    int4 *o = reinterpret_cast<int4 *>(&out);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 16); ++i) o[i] = q[i];
    return out;
}

// One node row in registers (compact layout).
struct Row {
    int32_t ac, am, rc, rm, zc, zm, np, mp;
    double yc, ym;
};
// One node row in registers (wide layout: memory as f64 bytes).
struct RowW {
    int32_t ac, rc, zc, np, mp;
    double am, rm, zm, yc, ym;
};
struct RowX {
    int32_t ae0, re0, ae1, re1;
    uint64_t th, ts, lb0, lb1;
};
// Register row / pod record types of a feature set (kFeatWide picks the wide layout).
template <uint32_t F>
using RowT = typename std::conditional<(F & kFeatWide) != 0, RowW, Row>::type;
template <uint32_t F>
using PodT = typename std::conditional<(F & kFeatWide) != 0, DPodW, DPod>::type;

template <uint32_t F>
__device__ __forceinline__ RowT<F> load_row(const DevTable &t, uint32_t i) {
    if constexpr ((F & kFeatWide) != 0) {
        const int4 *q = reinterpret_cast<const int4 *>(t.wrows + i);
        const int4 a = q[0], d = q[3];
        const double2 *y = reinterpret_cast<const double2 *>(t.wrows + i);
        const double2 b = y[1], c = y[2];
        RowW r;
        r.rc = a.x; r.zc = a.y; r.np = a.z; r.ac = a.w;
        r.rm = b.x; r.zm = b.y; r.am = c.x; r.ym = c.y;
        r.yc = __builtin_bit_cast(double, ((uint64_t)(uint32_t)d.y << 32) | (uint32_t)d.x);
        r.mp = d.z;
        return r;
    } else {
        const int4 *q = reinterpret_cast<const int4 *>(t.rows + i);
        const int4 a = q[0], b = q[1];
        const double2 y = reinterpret_cast<const double2 *>(t.rows + i)[2];
        Row r;
        r.ac = a.x; r.am = a.y; r.rc = a.z; r.rm = a.w;
        r.zc = b.x; r.zm = b.y; r.np = b.z; r.mp = b.w;
        r.yc = y.x; r.ym = y.y;
        return r;
    }
}
template <uint32_t F>
__device__ __forceinline__ RowT<F> empty_row() {
    RowT<F> r;
    r.ac = r.am = r.rc = r.rm = r.zc = r.zm = 0;
    r.np = 0; r.mp = 0;  // pods + 1 > max_pods -> never feasible
    r.yc = r.ym = 0.0;
    return r;
}
// Per-field select (a ternary on whole structs is lowered through scratch memory).
__device__ __forceinline__ Row sel_row(bool c, const Row &a, const Row &b) {
    Row r;
    r.ac = c ? a.ac : b.ac; r.am = c ? a.am : b.am; r.rc = c ? a.rc : b.rc; r.rm = c ? a.rm : b.rm;
    r.zc = c ? a.zc : b.zc; r.zm = c ? a.zm : b.zm; r.np = c ? a.np : b.np; r.mp = c ? a.mp : b.mp;
    r.yc = c ? a.yc : b.yc; r.ym = c ? a.ym : b.ym;
    return r;
}
__device__ __forceinline__ RowW sel_row(bool c, const RowW &a, const RowW &b) {
    RowW r;
    r.ac = c ? a.ac : b.ac; r.am = c ? a.am : b.am; r.rc = c ? a.rc : b.rc; r.rm = c ? a.rm : b.rm;
    r.zc = c ? a.zc : b.zc; r.zm = c ? a.zm : b.zm; r.np = c ? a.np : b.np; r.mp = c ? a.mp : b.mp;
    r.yc = c ? a.yc : b.yc; r.ym = c ? a.ym : b.ym;
    return r;
}
__device__ __forceinline__ RowX sel_rowx(bool c, const RowX &a, const RowX &b) {
    RowX r;
    r.ae0 = c ? a.ae0 : b.ae0; r.re0 = c ? a.re0 : b.re0; r.ae1 = c ? a.ae1 : b.ae1;
    r.re1 = c ? a.re1 : b.re1; r.th = c ? a.th : b.th; r.ts = c ? a.ts : b.ts;
    r.lb0 = c ? a.lb0 : b.lb0; r.lb1 = c ? a.lb1 : b.lb1;
    return r;
}
template <uint32_t F>
__device__ __forceinline__ RowX load_rowx(const DevTable &t, uint32_t i) {
    RowX x;
    x.ae0 = x.re0 = x.ae1 = x.re1 = 0;
    x.th = x.ts = x.lb0 = x.lb1 = 0;
    if (F & kFeatExt) {
        const int4 e = (F & kFeatWide) ? reinterpret_cast<const int4 *>(t.wrows + i)[4]
                                       : reinterpret_cast<const int4 *>(t.rows + i)[3];
        x.ae0 = e.x; x.re0 = e.y; x.ae1 = e.z; x.re1 = e.w;
    }
    if (F & (kFeatTaint | kFeatAffinity)) {
        const DMask m = t.masks[i];
        x.th = m.th; x.ts = m.ts; x.lb0 = m.lb0; x.lb1 = m.lb1;
    }
    return x;
}
template <uint32_t F>
__device__ __forceinline__ void store_dyn(const DevTable &t, uint32_t i, const RowT<F> &r) {
    if constexpr ((F & kFeatWide) != 0) {
        int32_t *w = reinterpret_cast<int32_t *>(t.wrows + i);
        w[0] = r.rc; w[1] = r.zc; w[2] = r.np;
        *reinterpret_cast<double2 *>(w + 4) = make_double2(r.rm, r.zm);  // q1
    } else {
        int32_t *w = reinterpret_cast<int32_t *>(t.rows + i);
        *reinterpret_cast<int2 *>(w + 2) = make_int2(r.rc, r.rm);
        *reinterpret_cast<int2 *>(w + 4) = make_int2(r.zc, r.zm);
        w[6] = r.np;
    }
}
template <uint32_t F>
__device__ __forceinline__ void store_dynx(const DevTable &t, uint32_t i, const RowX &x) {
    if (F & kFeatExt) {
        int32_t *w = (F & kFeatWide) ? reinterpret_cast<int32_t *>(t.wrows + i) + 16
                                     : reinterpret_cast<int32_t *>(t.rows + i) + 12;
        w[1] = x.re0;
        w[3] = x.re1;
    }
}
// ---- in-launch hand-off forms of the resident stream -------------------------
// Per MI355X_MICROARCH.md § inter-workgroup visibility (valid forms, row 1): every handed-off byte
// is stored write-through (sc1) and read with sc1 loads to registers, so neither side needs an L2
// write-back or an L1 invalidate.  Both row layouts: the quads a Reserve changes (compact q0 q1
// q3, wide q0 q1 q4) go through sc1, the static ones (reciprocals, wide allocatable memory) are
// read plainly.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
template <uint32_t F>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const DevTable &t) {
    if constexpr ((F & kFeatWide) != 0)
        return __builtin_amdgcn_make_buffer_rsrc((void *)t.wrows, (short)0, (int)(t.n * sizeof(DRowW)), 0x00020000);
    else
        return __builtin_amdgcn_make_buffer_rsrc((void *)t.rows, (short)0, (int)(t.n * sizeof(DRow)), 0x00020000);
}
__device__ __forceinline__ uint64_t load_coh_u64(const uint64_t *p) {
    return __hip_atomic_load((gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_coh_u64(uint64_t *p, uint64_t v) {
    __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_coh_u32(const uint32_t *p) {
    return __hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Every storing wave drains its sc1 stores before the workgroup barrier that precedes a signal.
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ double u2d(uint32_t lo, uint32_t hi) {
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// A row whose dynamic quads another workgroup writes during the launch: those quads by sc1
// loads, the static ones plainly.
template <uint32_t F>
__device__ __forceinline__ RowT<F> load_row_coh(const DevTable &t, __amdgpu_buffer_rsrc_t rs, uint32_t i, RowX &x) {
    constexpr int RB = (int)((F & kFeatWide) ? sizeof(DRowW) : sizeof(DRow));
    constexpr int XQ = (F & kFeatWide) ? 64 : 48;  // byte offset of the extended-resource quad
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)i * RB, 0, 16);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)i * RB + 16, 0, 16);
    RowT<F> r;
    if constexpr ((F & kFeatWide) != 0) {
        const int4 *q = reinterpret_cast<const int4 *>(t.wrows + i);
        const double2 c = reinterpret_cast<const double2 *>(t.wrows + i)[2];
        const int4 d = q[3];
        r.rc = (int32_t)a.x; r.zc = (int32_t)a.y; r.np = (int32_t)a.z; r.ac = (int32_t)a.w;
        r.rm = u2d(b.x, b.y); r.zm = u2d(b.z, b.w);
        r.am = c.x; r.ym = c.y;
        r.yc = u2d((uint32_t)d.x, (uint32_t)d.y);
        r.mp = d.z;
    } else {
        const double2 y = reinterpret_cast<const double2 *>(t.rows + i)[2];
        r.ac = (int32_t)a.x; r.am = (int32_t)a.y; r.rc = (int32_t)a.z; r.rm = (int32_t)a.w;
        r.zc = (int32_t)b.x; r.zm = (int32_t)b.y; r.np = (int32_t)b.z; r.mp = (int32_t)b.w;
        r.yc = y.x; r.ym = y.y;
    }
    x = RowX{};
    if (F & kFeatExt) {
        const u32x4 e = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)i * RB + XQ, 0, 16);
        x.ae0 = (int32_t)e.x; x.re0 = (int32_t)e.y; x.ae1 = (int32_t)e.z; x.re1 = (int32_t)e.w;
    }
    return r;
}
template <uint32_t F>
__device__ __forceinline__ void store_row_coh(const DevTable &t, __amdgpu_buffer_rsrc_t rs, uint32_t i,
                                              const RowT<F> &r, const RowX &x) {
    (void)t;
    constexpr int RB = (int)((F & kFeatWide) ? sizeof(DRowW) : sizeof(DRow));
    constexpr int XQ = (F & kFeatWide) ? 64 : 48;
    u32x4 a, b;
    if constexpr ((F & kFeatWide) != 0) {
        const uint64_t rm = __builtin_bit_cast(uint64_t, r.rm), zm = __builtin_bit_cast(uint64_t, r.zm);
        a = u32x4{(uint32_t)r.rc, (uint32_t)r.zc, (uint32_t)r.np, (uint32_t)r.ac};
        b = u32x4{(uint32_t)rm, (uint32_t)(rm >> 32), (uint32_t)zm, (uint32_t)(zm >> 32)};
    } else {
        a = u32x4{(uint32_t)r.ac, (uint32_t)r.am, (uint32_t)r.rc, (uint32_t)r.rm};
        b = u32x4{(uint32_t)r.zc, (uint32_t)r.zm, (uint32_t)r.np, (uint32_t)r.mp};
    }
    __builtin_amdgcn_raw_buffer_store_b128(a, rs, (int)i * RB, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(b, rs, (int)i * RB + 16, 0, 16);
    if (F & kFeatExt) {
        const u32x4 e = {(uint32_t)x.ae0, (uint32_t)x.re0, (uint32_t)x.ae1, (uint32_t)x.re1};
        __builtin_amdgcn_raw_buffer_store_b128(e, rs, (int)i * RB + XQ, 0, 16);
    }
}

// The selectors' reads of compact rows, split so that a lane issues the loads of several nodes
// before it decodes any (res_selector: one memory round trip for a group of nodes instead of one
// per node): the dynamic quads q0 / q1 (and q3 with extended resources) by sc1 buffer loads (an
// index past the table reads zeros), and the reciprocals recomputed in registers (rcp_int below:
// RN(1/a) exactly, for a < 2^24) instead of loaded.
struct RowQ {
    u32x4 a, b, e;
};
template <uint32_t F>
__device__ __forceinline__ RowQ load_row_q(__amdgpu_buffer_rsrc_t rs, uint32_t i) {
    static_assert((F & kFeatWide) == 0, "compact rows only");
    // aux: sc1, and volatile (bit 31) so the compiler neither drops nor sinks a load into the
    // conditional block that consumes it: the group's loads stay issued back to back
    constexpr int kAux = 16 | (int)(1u << 31);
    RowQ q;
    q.a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * sizeof(DRow)), 0, kAux);
    q.b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * sizeof(DRow) + 16), 0, kAux);
    q.e = u32x4{0u, 0u, 0u, 0u};
    if (F & kFeatExt) q.e = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * sizeof(DRow) + 48), 0, kAux);
    return q;
}
__device__ __forceinline__ double rcp_int(int32_t a);
template <uint32_t F>
__device__ __forceinline__ Row decode_row_q(const RowQ &q, RowX &x) {
    Row r;
    r.ac = (int32_t)q.a.x; r.am = (int32_t)q.a.y; r.rc = (int32_t)q.a.z; r.rm = (int32_t)q.a.w;
    r.zc = (int32_t)q.b.x; r.zm = (int32_t)q.b.y; r.np = (int32_t)q.b.z; r.mp = (int32_t)q.b.w;
    r.yc = r.ac ? rcp_int(r.ac) : 0.0;  // (as the host's RN(1/alloc), 0 where alloc == 0)
    r.ym = r.am ? rcp_int(r.am) : 0.0;
    x = RowX{};
    if (F & kFeatExt) { x.ae0 = (int32_t)q.e.x; x.re0 = (int32_t)q.e.y; x.ae1 = (int32_t)q.e.z; x.re1 = (int32_t)q.e.w; }
    return r;
}

// Reserve (spec S7; UP framework/types.go#NodeInfo.update(+1))
template <class R, class P>
__device__ __forceinline__ void reserve(R &r, RowX &x, const P &p, int sign) {
    r.rc += sign * p.rc; r.rm += sign * p.rm;
    r.zc += sign * p.zc; r.zm += sign * p.zm;
    r.np += sign;
    x.re0 += sign * p.re0; x.re1 += sign * p.re1;
}

// ---- spec S4: NodeResourcesFit.Filter (UP noderesources/fit.go#fitsRequest) ------------------
// Per-resource checks are skipped for zero requests, which also covers the all-zero early return.
template <uint32_t F, class R, class P>
__device__ __forceinline__ bool fits(const R &r, const RowX &x, const P &p) {
    bool ok = r.np < r.mp;
    ok &= (p.rc <= 0) | (p.rc <= r.ac - r.rc);
    ok &= (p.rm <= 0) | (p.rm <= r.am - r.rm);
    if (F & kFeatExt) {
        ok &= (p.re0 == 0) | (p.re0 <= x.ae0 - x.re0);
        ok &= (p.re1 == 0) | (p.re1 <= x.ae1 - x.re1);
    }
    return ok;
}
__device__ __forceinline__ bool subset128(uint64_t m0, uint64_t m1, uint64_t b0, uint64_t b1) {
    return ((m0 & ~b0) | (m1 & ~b1)) == 0;
}
// Every caller evaluates ONE pod per wave (the pod record is wave-uniform), so the pod's term counts
// and its nodeSelector are read into scalars and the terms a pod does not have are skipped by
// scalar branches instead of being evaluated under a select (config 4: at most one required and
// two preferred terms per pod, most pods none).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
template <uint32_t F, class R, class P>
__device__ __forceinline__ bool feasible(const R &r, const RowX &x, const P &p, const DPodX &px) {
    bool ok = fits<F>(r, x, p);
    if (F & kFeatTaint) ok &= (x.th & ~px.tol_hard) == 0;  // UP tainttoleration#Filter
    if (F & kFeatAffinity) {                                 // UP nodeaffinity#Filter
        const uint64_t s0 = uniform64(px.sel0), s1 = uniform64(px.sel1);
        if (s0 | s1) ok &= subset128(s0, s1, x.lb0, x.lb1);
        const uint32_t nt = (uint32_t)__builtin_amdgcn_readfirstlane((int)((p.flags >> 4) & 7u));
        if (nt != 0) {
            bool any = false;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
                if (k < nt) any |= subset128(px.req[k][0], px.req[k][1], x.lb0, x.lb1);
            ok &= any;
        }
    }
    return ok;
}
// raw TaintToleration score: intolerable PreferNoSchedule taints (UP tainttoleration#Score)
__device__ __forceinline__ uint32_t taint_raw(const RowX &x, const DPodX &px) {
    return (uint32_t)__popcll(x.ts & ~px.tol_soft);
}
// raw NodeAffinity score: weights of matching preferred terms (UP nodeaffinity#Score)
template <class P>
__device__ __forceinline__ uint32_t affinity_raw(const RowX &x, const P &p, const DPodX &px) {
    const uint32_t nt = (uint32_t)__builtin_amdgcn_readfirstlane((int)((p.flags >> 8) & 7u));
    uint32_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        if (k < nt) s += subset128(px.pref[k][0], px.pref[k][1], x.lb0, x.lb1) ? (uint32_t)px.pw[k] : 0u;
    return s;
}

// The state-independent part of one (node, pod) evaluation of the normalizing plugins, packed in
// 32 bits (resident config-4 stream): bit 0 = the taint / nodeSelector /
// required-term filters pass, bits 1-7 = taint_raw (<= 64), bits 8-31 = affinity_raw.  Node masks
// and pod records never change during a stream, so it can be computed anywhere ahead of use; the
// resolver's slot and candidate keys then only add fits / LeastAllocated / BalancedAllocation and
// the two normalizations.  Same predicates as feasible / taint_raw / affinity_raw, with per-lane
// term counts (one pod per lane is allowed here).
__device__ __forceinline__ uint32_t static_raw(uint64_t th, uint64_t ts, uint64_t lb0, uint64_t lb1, uint32_t flags,
                                               const DPodX &px) {
    // branch-free (the callers run one pod per lane: per-lane branches cost exec-mask juggling)
    const uint32_t nr = (flags >> 4) & 7u, np = (flags >> 8) & 7u;
    uint32_t ok = (uint32_t)((th & ~px.tol_hard) == 0) & (uint32_t)(((px.sel0 | px.sel1) == 0) | subset128(px.sel0, px.sel1, lb0, lb1));
    uint32_t any = (uint32_t)(nr == 0), ra = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        any |= (uint32_t)(k < nr) & (uint32_t)subset128(px.req[k][0], px.req[k][1], lb0, lb1);
        const uint32_t hit = (uint32_t)(k < np) & (uint32_t)subset128(px.pref[k][0], px.pref[k][1], lb0, lb1);
        ra += (0u - hit) & (uint32_t)px.pw[k];
    }
    const uint32_t rt = (uint32_t)__popcll(ts & ~px.tol_soft);
    return (ok & any) | (rt << 1) | (ra << 8);
}

// ---- exact small divisions (spec S10) -------------------------------------------------------
// floor(n / d) for n < 2^32, 1 <= d < 2^29 and n / d <= ~1000, given y = RN_f64(1/d):
// n*y is within 2^-52 relative of n/d, whose fractional part is 0 or in [1/d, 1 - 1/d]; a 2^-30
// bias lifts exact integers clear of the truncation edge and can never carry a fraction over it.
__device__ __forceinline__ uint32_t floor_div(uint32_t n, double y) {
    return (uint32_t)__builtin_fma((double)n, y, 0x1p-30);
}
// UP least_allocated.go#leastRequestedScore: ((a - reqd) * 100) / a, 0 if reqd > a (a >= 0)
__device__ __forceinline__ uint32_t least_requested(int32_t a, int32_t reqd, double ya) {
    const int32_t rq = reqd < a ? reqd : a;                       // keep the discarded branch in range
    const uint32_t n = __umul24((uint32_t)(a - rq), 100u);        // a < 2^24 (compaction limit)
    const uint32_t q = floor_div(n, ya);
    return reqd > a ? 0u : q;
}
// min(RN(r / a), 1) for a > 0, r >= 0 — Markstein quotient, exact here (spec S10)
__device__ __forceinline__ double fraction(int32_t a, int32_t r, double y) {
    const double R = (double)r, A = (double)a;
    const double q0 = R * y;
    const double rem = __builtin_fma(-q0, A, R);
    const double q = __builtin_fma(rem, y, q0);
    return r >= a ? 1.0 : q;
}

// Wide layout (memory in f64 bytes, every value < 2^46, so (a - r) * 100 is exact):
// floor((a - reqd) * 100 / a) from the f64 quotient (within one of the floor: n * RN(1/a) is within
// 100 * 2^-52 of n / a) and one integer correction from the remainder n - q * a, which fma gives
// exactly (an integer below 2a in magnitude).  Branch-free; tests/native/exact_arith.c mode 4.
__device__ __forceinline__ uint32_t least_requested_w(double a, double reqd, double ya) {
    const double rq = reqd < a ? reqd : a;
    const double n = (a - rq) * 100.0;
    double q = __builtin_trunc(n * ya);
    const double r = __builtin_fma(-q, a, n);
    q = r < 0.0 ? q - 1.0 : q;
    q = (r >= a && a > 0.0) ? q + 1.0 : q;  // (a = 0: score 0, as upstream's capacity == 0 case)
    return reqd > a ? 0u : (uint32_t)q;
}
// min(RN(r / a), 1) for the wide layout: the Markstein quotient of `fraction` with y = RN(1/a) (the
// row's ym).  Exact for integers r < a <= 2^46: q0 = RN(r y) lies within 1.5 ulp of r / a, so the
// remainder r - q0 a is a multiple of ulp(q0) below 2^48 of them (exact in the fma), and q0 + rem y
// is within 2^-52 ulp of r / a, which lies at least ulp / 2a from every rounding midpoint
// (spec/semantics.md S10; tests/native/exact_arith.c mode 4).
__device__ __forceinline__ double fraction_w(double a, double r, double y) {
    const double q0 = r * y;
    const double rem = __builtin_fma(-q0, a, r);
    const double q = __builtin_fma(rem, y, q0);
    return r >= a ? 1.0 : q;
}

// ---- spec S5/S6: QoS-weighted total of one feasible node ------------------------------------
// floor(num / den) of a weighted mean of scores 0..100 (num = sum of score x weight < 2^24, den = the
// weight sum < 2^18, num / den <= 100): the f32 estimate is within 100 * 2^-22 < 1 of num / den, so it
// truncates to the floor or a neighbour; the exact remainder num - q den (|.| < 2^25) moves it by
// one.  den == 0 (no resource counted) scores 0, as upstream's weightSum == 0.
__device__ __forceinline__ uint32_t div_small(uint32_t num, uint32_t den) {
    const float d = (float)(den | (uint32_t)(den == 0u));
    int32_t q = (int32_t)((float)num * __builtin_amdgcn_rcpf(d));
    const int32_t r = (int32_t)num - q * (int32_t)den;
    q = r < 0 ? q - 1 : q;
    q = r >= (int32_t)den ? q + 1 : q;
    return den ? (uint32_t)q : 0u;
}
// RN(x / c) for the resource count c in {3, 4} of BalancedAllocation's >= 3-resource path (x >= 0,
// normal or zero: a sum of fractions or of squared deviations): c = 4 an exact scaling; c = 3
// Markstein's correction of q0 = RN(x RN(1/3)) (the remainder fma(-q0, 3, x) is exact and one fma with
// the correctly rounded reciprocal rounds the quotient correctly), in place of the IEEE division's
// scale / rcp / Newton / fixup sequence on the key chain.  Checked against IEEE division on 80 M
// cases (tests/native/exact_arith.c mode 5) and by every configurable-resource parity test.
__device__ __forceinline__ double div_count(double x, uint32_t c) {
    const double y3 = 0x1.5555555555555p-2;  // RN(1/3)
    const double q0 = x * y3;
    const double r = __builtin_fma(-q0, 3.0, x);
    const double q3 = __builtin_fma(r, y3, q0);
    return c == 4u ? x * 0.25 : q3;
}
// Correctly rounded f64 square root (Go math.Sqrt, SQRTSD): LLVM's gfx950 expansion of llvm.sqrt.f64
// (scaling, v_rsq_f64, two Newton steps, the fma residual correction), checked bit for bit against
// the host's sqrt on 33 M inputs by tests/native/sqrt_sweep.hip (tests/test_gpu_sqrt.py).
__device__ __forceinline__ double sqrt_rn(double v) { return __builtin_sqrt(v); }

// Extended-resource terms of the configurable lists (UP resource_allocation.go#
// calculateResourceAllocatableRequest): an extended resource counts only where the node has it and
// the pod requests it (scalar resource with podRequest == 0 -> (0, 0)); it is Requested (not
// NonZeroRequested) + the request in both plugins.  RN(1/alloc) from rcp_int (alloc < 2^24).
struct ExtTerms {
    bool h0, h1;
    double y0, y1;
};
template <class P>
__device__ __forceinline__ ExtTerms ext_terms(const RowX &x, const P &p) {
    ExtTerms e;
    e.h0 = (x.ae0 != 0) & (p.re0 != 0);
    e.h1 = (x.ae1 != 0) & (p.re1 != 0);
    e.y0 = rcp_int(x.ae0 | (int32_t)(x.ae0 == 0));
    e.y1 = rcp_int(x.ae1 | (int32_t)(x.ae1 == 0));
    return e;
}

// LeastAllocated (UP least_allocated.go#leastResourceScorer), NonZeroRequested + pod nz.
// Branch-free: a resource with alloc == 0 contributes weight 0 (its score is 0 as well).
template <uint32_t F, class R, class P>
__device__ __forceinline__ uint32_t la_score(const R &r, const RowX &x, const P &p, const DevCfg &c) {
    const bool hc = r.ac != 0, hm = r.am != 0;
    const uint32_t sc_c = least_requested(r.ac, r.zc + p.zc, r.yc);
    uint32_t sc_m;
    if constexpr (std::is_same<R, RowW>::value) sc_m = least_requested_w(r.am, r.zm + p.zm, r.ym);
    else sc_m = least_requested(r.am, r.zm + p.zm, r.ym);
    const uint32_t wce = hc ? (uint32_t)c.wc : 0u, wme = hm ? (uint32_t)c.wm : 0u;
    const uint32_t num = __umul24(sc_c, wce) + __umul24(sc_m, wme);
    if constexpr ((F & kFeatRes) != 0) {
        // the configured list (spec S5 "Scoring resources"): cpu / memory weights 0 when absent,
        // the extended columns' terms where counted, then the weighted mean
        const ExtTerms e = ext_terms(x, p);
        const uint32_t s0 = least_requested(x.ae0, x.re0 + p.re0, e.y0);
        const uint32_t s1 = least_requested(x.ae1, x.re1 + p.re1, e.y1);
        const uint32_t w0 = e.h0 ? (uint32_t)c.we0 : 0u, w1 = e.h1 ? (uint32_t)c.we1 : 0u;
        return div_small(num + __umul24(s0, w0) + __umul24(s1, w1), wce + wme + w0 + w1);
    } else {
        (void)x;
        // select the weight-sum reciprocal with bit masks (a ternary on the kernel-argument doubles
        // was lowered to a per-lane load from the kernarg segment, stalling on vmcnt(0))
        const uint64_t mb = 0ull - (uint64_t)(hc & hm), mc = 0ull - (uint64_t)(hc & !hm),
                       mm = 0ull - (uint64_t)(!hc & hm);
        const double yd = __builtin_bit_cast(
            double, (__builtin_bit_cast(uint64_t, c.yd_both) & mb) |
                        (__builtin_bit_cast(uint64_t, c.yd_c) & mc) | (__builtin_bit_cast(uint64_t, c.yd_m) & mm));
        // den == 0 means num == 0 and yd == 0.0: floor_div gives 0 without a branch
        return floor_div(num, yd);
    }
}
// BalancedAllocation (UP balanced_allocation.go#balancedResourceScorer), Requested + pod req
template <uint32_t F, class R, class P>
__device__ __forceinline__ uint32_t ba_score(const R &r, const RowX &x, const P &p, const DevCfg &c) {
    const bool hc = r.ac != 0, hm = r.am != 0;
    const double f0 = fraction(r.ac, r.rc + p.rc, r.yc);
    double f1;
    if constexpr (std::is_same<R, RowW>::value) f1 = fraction_w(r.am, r.rm + p.rm, r.ym);
    else f1 = fraction(r.am, r.rm + p.rm, r.ym);
    double sd = 0.0;
    if constexpr ((F & kFeatRes) != 0) {
        // the configured list in its order (c.bal, 4 bits per entry; the ids are wave-uniform):
        // included fractions summed in list order, a skipped entry adds an exact +0.0
        const ExtTerms e = ext_terms(x, p);
        const double fe0 = fraction(x.ae0, x.re0 + p.re0, e.y0), fe1 = fraction(x.ae1, x.re1 + p.re1, e.y1);
        double fj[QS_BAL_MAX], fa = 0.0, fb = 0.0, tot = 0.0;
        bool ij[QS_BAL_MAX];
        uint32_t cnt = 0;
#pragma unroll
        for (int j = 0; j < QS_BAL_MAX; ++j) {
            const uint32_t id = (c.bal >> (4 * j)) & 7u;
            fj[j] = id == 1u ? f0 : id == 2u ? f1 : id == 3u ? fe0 : fe1;
            ij[j] = id == 1u ? hc : id == 2u ? hm : id == 3u ? e.h0 : id == 4u ? e.h1 : false;
            fa = (ij[j] & (cnt == 0u)) ? fj[j] : fa;
            fb = (ij[j] & (cnt == 1u)) ? fj[j] : fb;
            tot = tot + (ij[j] ? fj[j] : 0.0);
            cnt += ij[j] ? 1u : 0u;
        }
        if (cnt == 2u) {
            sd = __builtin_fabs((fa - fb) / 2);
        } else if (cnt > 2u) {
            const double mean = div_count(tot, cnt);  // = RN(tot / cnt), the IEEE quotient
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < QS_BAL_MAX; ++j) {
                const double d = fj[j] - mean;
                const double sq = d * d;
                s = s + (ij[j] ? sq : 0.0);
            }
            sd = sqrt_rn(div_count(s, cnt));
        }
    } else {
        (void)x;
        if (hc & hm) sd = __builtin_fabs((f0 - f1) / 2);
    }
    const double scaled = (1 - sd) * 100.0;
    uint32_t ba = (uint32_t)(int32_t)scaled;  // int64() truncation toward zero
    if (c.ba_skip_be && (p.flags & 3u) == 0) ba = 0;
    return ba;
}

// Normalized TaintToleration score: reverse DefaultNormalizeScore (UP helper/normalize_score.go)
// of the raw count given the pod's maximum mt over feasible nodes and ymt = RN(1/mt).
__device__ __forceinline__ uint32_t tt_norm(uint32_t raw, uint32_t mt, double ymt) {
    return mt == 0 ? 100u : 100u - floor_div(100u * raw, ymt);
}
// Normalized NodeAffinity score: DefaultNormalizeScore (not reversed).
__device__ __forceinline__ uint32_t na_norm(uint32_t raw, uint32_t ma, double yma) {
    return ma == 0 ? raw : floor_div(100u * raw, yma);
}

template <uint32_t F, class R, class P>
__device__ __forceinline__ uint32_t node_total(const R &r, const RowX &x, const P &p,
                                               const DPodX &px, const DevCfg &c, uint32_t mt,
                                               double ymt, uint32_t ma, double yma, uint32_t *sc) {
    const uint32_t la = la_score<F>(r, x, p, c), ba = ba_score<F>(r, x, p, c);
    uint32_t total = __umul24((uint32_t)p.wfit, la) + __umul24((uint32_t)p.wbal, ba);
    uint32_t tt = 0, na = 0;
    if (F & kFeatTaint) {
        tt = tt_norm(taint_raw(x, px), mt, ymt);
        total += __umul24((uint32_t)c.wtt, tt);
    }
    if (F & kFeatAffinity) {
        na = na_norm(affinity_raw(x, p, px), ma, yma);
        total += __umul24((uint32_t)c.wna, na);
    }
    if (sc) { sc[0] = la; sc[1] = ba; sc[2] = tt; sc[3] = na; }
    return total;
}

// node_total of a normalizing profile with the node's static part given as static_raw (resident
// stream's waves A/B/C): the same sums in the same order.
template <uint32_t F, class R, class P>
__device__ __forceinline__ uint32_t norm_total(const R &r, const RowX &x, const P &p, const DevCfg &c, uint32_t st,
                                               uint32_t mt, double ymt, uint32_t ma, double yma) {
    uint32_t total = __umul24((uint32_t)p.wfit, la_score<F>(r, x, p, c)) +
                     __umul24((uint32_t)p.wbal, ba_score<F>(r, x, p, c));
    if (F & kFeatTaint) total += __umul24((uint32_t)c.wtt, tt_norm((st >> 1) & 127u, mt, ymt));
    if (F & kFeatAffinity) total += __umul24((uint32_t)c.wna, na_norm(st >> 8, ma, yma));
    return total;
}
// The resolver's lost-holder flags of an infeasible node (bit 0: its taint raw score is the pod's
// selection-time maximum, bit 1: its affinity raw score is), from static_raw.
template <uint32_t F>
__device__ __forceinline__ uint32_t holder_flags(uint32_t st, uint32_t mt, uint32_t ma) {
    uint32_t fl = 0;
    if (F & kFeatTaint) fl |= ((st >> 1) & 127u) == mt ? 1u : 0u;
    if (F & kFeatAffinity) fl |= (st >> 8) == ma ? 2u : 0u;
    return fl;
}

// Normalization facts of one pod at selection time (LOOKAHEAD with TaintToleration /
// NodeAffinity): the maxima of the raw scores over the nodes feasible then, and how many nodes
// attain each maximum (the resolver's proof that a maximum still holds).
struct alignas(16) NormInfo {
    uint32_t mt, ct, ma, ca;
};

// spec S7 packed key: ((total + 1) << 32) | (0xFFFFFFFF - idx); 0 = infeasible
__device__ __forceinline__ uint64_t pack_key(uint32_t tv, uint32_t idx) {
    return ((uint64_t)tv << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}
__device__ __forceinline__ uint32_t key_node(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }

// ---- 64-lane reductions with DPP (no LDS round trip) -----------------------------------------
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint64_t dpp_max64(uint64_t v) {
    const uint32_t lo = dpp32<CTRL, ROW_MASK>((uint32_t)v);
    const uint32_t hi = dpp32<CTRL, ROW_MASK>((uint32_t)(v >> 32));
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    return o > v ? o : v;
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp_max32(uint32_t v) {
    const uint32_t o = dpp32<CTRL, ROW_MASK>(v);
    return o > v ? o : v;
}
// Full-wave max; every lane must be active.  Result is wave-uniform.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = dpp_max32<0xB1>(v);        // quad_perm [1,0,3,2]
    v = dpp_max32<0x4E>(v);        // quad_perm [2,3,0,1]
    v = dpp_max32<0x141>(v);       // row_half_mirror
    v = dpp_max32<0x140>(v);       // row_mirror: each row of 16 holds its max
    v = dpp_max32<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v = dpp_max32<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// The same reduction with the DPP moves folded into the max (v_max_u32_dpp: 6 instead of 12 VALU
// instructions on the resolver's critical path); the s_nop 1 before each step covers the DPP
// read-after-VALU-write hazard that the compiler cannot see inside the asm.
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
    uint32_t r;
    asm volatile(
        "s_nop 1\n\t"
        "v_max_u32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_readlane_b32 %0, %1, 63"
        : "=s"(r), "+v"(v));
    return r;
}
// Max of packed keys as two 32-bit reductions: the score half first, then the index half among
// the lanes holding that score (keys are unique, so this is the u64 max).
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    const uint32_t hi = wave_max_u32((uint32_t)(v >> 32));
    const uint32_t lo = wave_max_u32((uint32_t)(v >> 32) == hi ? (uint32_t)v : 0u);
    return ((uint64_t)hi << 32) | lo;
}

// RN_f64(1/a) for 1 <= a < 2^24 without the IEEE division sequence: v_rcp_f32's estimate (within
// 1 ulp) refined by two fma Newton steps.  The second step leaves an error near 2^-92 relative,
// while 1/a lies at least 2^-77 (relative) from every rounding midpoint, so the final rounding is
// RN(1/a); tests/native/exact_arith.c mode 3 checks every a and every estimate within 2 ulps.
__device__ __forceinline__ double rcp_int(int32_t a) {
    const double A = (double)a;
    double y = (double)__builtin_amdgcn_rcpf((float)a);
    double e = __builtin_fma(-A, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-A, y, 1.0);
    return __builtin_fma(y, e, y);
}

// RN_f64(1/d) of a per-pod normalize maximum (IEEE division; once per pod, off the node loop).
__device__ __forceinline__ double rcp_exact(uint32_t d) { return d ? 1.0 / (double)d : 0.0; }

}  // namespace qs
