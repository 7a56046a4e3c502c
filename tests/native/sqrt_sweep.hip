// sqrt_sweep.hip — device check of the f64 arithmetic of configurable BalancedAllocation lists
// (spec/semantics.md S10 "Configurable scoring resources"; run by tests/test_gpu_sqrt.py on the GPU box).
//  1. qs::sqrt_rn (the device sqrt ba_score uses) against the host's correctly rounded sqrt, bit for
//     bit, on 32 M inputs: random bit patterns over every binade of [2^-120, 4], the tiny sums the
//     K12 sentinel produces, exact squares and their neighbours.
//  2. qs::ba_score<kFeatExt | kFeatRes> (the kernels' scorer) against the oracle's or_balanced_v on
//     2 M random (node, pod, list) cases with 2-4 counted resources, random list order and
//     skipped entries.
// Prints "sqrt mismatches M of N" and "balanced mismatches M of N"; exit 1 on any mismatch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../custom-k8s-scheduler_amd/csrc/qs_device.hpp"
extern "C" {
#include "../../oracle/qs_oracle.h"
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 2;                                                              \
        }                                                                          \
    } while (0)

__global__ void k_sqrt(const double *in, double *out, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = qs::sqrt_rn(in[i]);
}

struct BaCase {
    int32_t ac, rc, am, rm, ae0, re0, ae1, re1;  // node alloc / requested (before the pod)
    int32_t prc, prm, pre0, pre1;                // pod requests
    uint32_t bal;                                // list ids, 4 bits each
};

__global__ void k_ba(const BaCase *cs, uint32_t *out, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const BaCase c = cs[i];
    qs::Row r{};
    r.ac = c.ac; r.rc = c.rc; r.am = c.am; r.rm = c.rm; r.mp = 110;
    r.yc = c.ac ? qs::rcp_int(c.ac) : 0.0;
    r.ym = c.am ? qs::rcp_int(c.am) : 0.0;
    qs::RowX x{};
    x.ae0 = c.ae0; x.re0 = c.re0; x.ae1 = c.ae1; x.re1 = c.re1;
    qs::DPod p{};
    p.rc = c.prc; p.rm = c.prm; p.re0 = c.pre0; p.re1 = c.pre1; p.flags = 1;
    qs::DevCfg cfg{};
    cfg.bal = c.bal;
    out[i] = qs::ba_score<qs::kFeatExt | qs::kFeatRes>(r, x, p, cfg);
}

int main() {
    std::mt19937_64 rng(0x5EED5EEDull);
    // ---- 1. sqrt ----
    const size_t N = (size_t)32 << 20;
    std::vector<double> in(N);
    for (size_t i = 0; i < N; ++i) {
        const uint64_t b = rng();
        double v;
        switch (i % 4) {
            case 0: {  // random mantissa, exponent in [-120, 1]
                const uint64_t e = 1023 - 120 + (b >> 52) % 122;
                v = __builtin_bit_cast(double, (e << 52) | (b & ((1ull << 52) - 1)));
                break;
            }
            case 1: {  // (0, 1): the variance of fractions in [0, 1]
                v = (double)(b >> 11) * 0x1p-53;
                break;
            }
            case 2: {  // tiny sums of squared rounding errors (sentinel K12: ~2^-104)
                const uint64_t e = 1023 - 110 + (b >> 52) % 12;
                v = __builtin_bit_cast(double, (e << 52) | (b & ((1ull << 52) - 1)));
                break;
            }
            default: {  // exact squares and their neighbours
                const double y = (double)(b >> 40) * 0x1p-12 + 0x1p-30;
                const double sq = y * y;
                const int k = (int)(b & 3) - 1;
                v = k < 0 ? std::nextafter(sq, 0.0) : (k > 0 ? std::nextafter(sq, 4.0) : sq);
                break;
            }
        }
        in[i] = v;
    }
    double *din = nullptr, *dout = nullptr;
    CK(hipMalloc(&din, N * 8));
    CK(hipMalloc(&dout, N * 8));
    CK(hipMemcpy(din, in.data(), N * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_sqrt, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, 0, din, dout, N);
    CK(hipGetLastError());
    std::vector<double> out(N);
    CK(hipMemcpy(out.data(), dout, N * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < N; ++i) {
        const double ref = std::sqrt(in[i]);
        if (std::memcmp(&ref, &out[i], 8) != 0) {
            if (bad < 5) std::printf("  sqrt(%a): device %a host %a\n", in[i], out[i], ref);
            ++bad;
        }
    }
    std::printf("sqrt mismatches %zu of %zu\n", bad, N);
    CK(hipFree(din));
    CK(hipFree(dout));

    // ---- 2. the BalancedAllocation scorer over configurable lists ----
    const size_t M = (size_t)2 << 20;
    std::vector<BaCase> cs(M);
    auto pick = [&](uint64_t k) { return (int32_t)(rng() % k); };
    for (auto &c : cs) {
        const int32_t smalls[] = {1, 2, 3, 4, 5, 8, 10, 16, 25, 100, 1000, 4000, 65536, 1 << 20, (1 << 24) - 1};
        auto val = [&]() { return pick(4) == 0 ? smalls[pick(15)] : 1 + pick((1 << 24) - 1); };
        c.ac = pick(10) == 0 ? 0 : val();
        c.am = pick(10) == 0 ? 0 : val();
        c.ae0 = pick(3) == 0 ? 0 : val();
        c.ae1 = pick(3) == 0 ? 0 : val();
        auto used = [&](int32_t a) { return a ? pick(a + 1) : 0; };
        c.rc = used(c.ac); c.rm = used(c.am); c.re0 = used(c.ae0); c.re1 = used(c.ae1);
        auto req = [&](int32_t a, int32_t u) { return pick(4) == 0 ? 0 : (a ? pick(a - u + 2) : pick(8)); };
        c.prc = req(c.ac, c.rc); c.prm = req(c.am, c.rm); c.pre0 = req(c.ae0, c.re0); c.pre1 = req(c.ae1, c.re1);
        int ids[4] = {1, 2, 3, 4};
        std::shuffle(ids, ids + 4, rng);
        const int len = 1 + pick(4);
        c.bal = 0;
        for (int k = 0; k < len; ++k) c.bal |= (uint32_t)ids[k] << (4 * k);
    }
    BaCase *dcs = nullptr;
    uint32_t *dba = nullptr;
    CK(hipMalloc(&dcs, M * sizeof(BaCase)));
    CK(hipMalloc(&dba, M * 4));
    CK(hipMemcpy(dcs, cs.data(), M * sizeof(BaCase), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_ba, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, 0, dcs, dba, M);
    CK(hipGetLastError());
    std::vector<uint32_t> ba(M);
    CK(hipMemcpy(ba.data(), dba, M * 4, hipMemcpyDeviceToHost));
    size_t bad2 = 0, three = 0;
    for (size_t i = 0; i < M; ++i) {
        const BaCase &c = cs[i];
        int64_t alloc[4], reqd[4];
        int cnt = 0, counted = 0;
        for (int k = 0; k < 4; ++k) {
            const uint32_t id = (c.bal >> (4 * k)) & 15u;
            if (!id) break;
            int64_t a = 0, r = 0;
            if (id == 1) { a = c.ac; r = (int64_t)c.rc + c.prc; }
            if (id == 2) { a = c.am; r = (int64_t)c.rm + c.prm; }
            if (id == 3 && c.pre0) { a = c.ae0; r = (int64_t)c.re0 + c.pre0; }
            if (id == 4 && c.pre1) { a = c.ae1; r = (int64_t)c.re1 + c.pre1; }
            alloc[cnt] = a; reqd[cnt] = r; ++cnt;
            counted += a != 0;
        }
        three += counted > 2;
        const int64_t ref = or_balanced_v(cnt, alloc, reqd);
        if ((int64_t)ba[i] != ref) {
            if (bad2 < 5) std::printf("  case %zu: device %u oracle %lld\n", i, ba[i], (long long)ref);
            ++bad2;
        }
    }
    std::printf("balanced mismatches %zu of %zu (%zu with three or more counted resources)\n", bad2, M, three);
    CK(hipFree(dcs));
    CK(hipFree(dba));
    return (bad || bad2) ? 1 : 0;
}
