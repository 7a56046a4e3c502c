// Micro-benchmark of the HBM-resident scoring scan variants (not part of the library).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../custom-k8s-scheduler_amd/csrc scan_micro.hip -o scan_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "qs_device.hpp"
using namespace qs;

struct Cols { int32_t *c[8]; double *y[2]; };

// V: 0 = reciprocals by IEEE division, 1 = load-only (sum), 2 = reciprocal columns, 3 = rcp from f32 estimate
template <int V>
__global__ __launch_bounds__(256) void k(Cols t, uint32_t n, DPod p, DevCfg c, unsigned long long *out) {
    const DPodX px{};
    const uint32_t nq = n / 4;
    uint64_t best = 0;
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < nq; q += gridDim.x * 256) {
        int4 col[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) col[k] = reinterpret_cast<const int4 *>(t.c[k])[q];
        double2 ya0, ya1, yb0, yb1;
        if (V == 2) {
            ya0 = reinterpret_cast<const double2 *>(t.y[0])[2 * q]; ya1 = reinterpret_cast<const double2 *>(t.y[0])[2 * q + 1];
            yb0 = reinterpret_cast<const double2 *>(t.y[1])[2 * q]; yb1 = reinterpret_cast<const double2 *>(t.y[1])[2 * q + 1];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            auto el = [&](int k) { return e == 0 ? col[k].x : e == 1 ? col[k].y : e == 2 ? col[k].z : col[k].w; };
            if (V == 1) { best += (uint32_t)(el(0) ^ el(1) ^ el(2) ^ el(3) ^ el(4) ^ el(5) ^ el(6) ^ el(7)); continue; }
            Row r;
            r.ac = el(0); r.am = el(1); r.rc = el(2); r.rm = el(3); r.zc = el(4); r.zm = el(5); r.np = el(6); r.mp = el(7);
            if (V == 0) { r.yc = r.ac ? 1.0 / (double)r.ac : 0.0; r.ym = r.am ? 1.0 / (double)r.am : 0.0; }
            if (V == 2) { r.yc = e == 0 ? ya0.x : e == 1 ? ya0.y : e == 2 ? ya1.x : ya1.y; r.ym = e == 0 ? yb0.x : e == 1 ? yb0.y : e == 2 ? yb1.x : yb1.y; }
            if (V == 3) { r.yc = (double)(1.0f / (float)r.ac); r.ym = (double)(1.0f / (float)r.am); }
            RowX x{};
            const bool f = feasible<0>(r, x, p, px);
            const uint32_t tot = node_total<0>(r, x, p, px, c, 0, 0.0, 0, 0.0, nullptr);
            const uint64_t key = f ? pack_key(tot + 1, 4 * q + e) : 0ull;
            best = key > best ? key : best;
        }
    }
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0 && best) atomicMax(out, (unsigned long long)best);
}

template <int V>
float run(Cols t, uint32_t n, DPod p, DevCfg c, unsigned long long *out, int blocks) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, t, n, p, c, out);
    hipEventRecord(a);
    const int R = 10;
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, t, n, p, c, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / R;
}

int main() {
    const uint32_t n = 1u << 24;
    std::vector<int32_t> h(n);
    Cols t;
    const int32_t cpus[6] = {4000, 8000, 16000, 32000, 64000, 96000};
    for (int k = 0; k < 8; ++k) {
        for (uint32_t i = 0; i < n; ++i) {
            const int32_t ac = cpus[i % 6];
            h[i] = k == 0 ? ac : k == 1 ? ac / 1000 * 4096 : k == 2 ? (int32_t)(i * 7919 % ac) / 2 : k == 3 ? (int32_t)(i % 5000) : k == 4 ? (int32_t)(i * 7919 % ac) / 2 + 100 : k == 5 ? (int32_t)(i % 5000) + 200 : k == 6 ? (int32_t)(i % 50) : 110;
        }
        hipMalloc(&t.c[k], 4ull * n);
        hipMemcpy(t.c[k], h.data(), 4ull * n, hipMemcpyHostToDevice);
    }
    for (int k = 0; k < 2; ++k) {
        std::vector<double> y(n);
        for (uint32_t i = 0; i < n; ++i) { const int32_t ac = cpus[i % 6]; y[i] = 1.0 / (double)(k == 0 ? ac : ac / 1000 * 4096); }
        hipMalloc(&t.y[k], 8ull * n);
        hipMemcpy(t.y[k], y.data(), 8ull * n, hipMemcpyHostToDevice);
    }
    unsigned long long *out; hipMalloc(&out, 8);
    DPod p{}; p.rc = 1000; p.rm = 2048; p.zc = 1000; p.zm = 2048; p.wfit = 2; p.wbal = 1; p.flags = 1;
    DevCfg c{}; c.wc = 1; c.wm = 1; c.yd_both = 0.5; c.yd_c = 1.0; c.yd_m = 1.0;
    for (int blocks : {2048, 4096, 8192, 16384}) {
        const double bytes = 32.0 * n;
        float m0 = run<0>(t, n, p, c, out, blocks), m1 = run<1>(t, n, p, c, out, blocks);
        float m2 = run<2>(t, n, p, c, out, blocks), m3 = run<3>(t, n, p, c, out, blocks);
        printf("blocks %5d: div %.1f us (%.0f GB/s)  load-only %.1f us (%.0f GB/s)  ycols %.1f us (%.0f GB/s alg, %.0f actual)  f32rcp %.1f us (%.0f GB/s)\n",
               blocks, m0 * 1e3, bytes / m0 / 1e6, m1 * 1e3, bytes / m1 / 1e6, m2 * 1e3, bytes / m2 / 1e6, 1.5 * bytes / m2 / 1e6, m3 * 1e3, bytes / m3 / 1e6);
    }
    return 0;
}
