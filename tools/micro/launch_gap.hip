// Back-to-back launch overhead on one stream: 2000 single-workgroup kernels that each busy-wait a
// fixed number of s_memrealtime ticks (100 MHz), wall time vs the busy time; then the same
// through a HIP graph; then with 128 workgroups of a second stream running beside them.
// Build: hipcc --offload-arch=gfx950 -O3 launch_gap.hip -o launch_gap
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <stdint.h>

__global__ void k_busy(uint64_t ticks, uint32_t *sink) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0xdeadbeef) sink[0] = x;
}

static double run(hipStream_t s, int n, uint64_t ticks, uint32_t *sink, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, ticks, sink);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3 / n;  // us per launch
}

int main() {
    uint32_t *sink;
    (void)hipMalloc(&sink, 64);
    hipStream_t s1, s2;
    (void)hipStreamCreate(&s1);
    (void)hipStreamCreate(&s2);
    const int N = 2000;
    for (uint64_t ticks : {0ull, 500ull, 2000ull}) {  // 0, 5, 20 us of busy time
        run(s1, 100, ticks, sink, 1);
        const double us = run(s1, N, ticks, sink, 1);
        printf("busy %5.1f us: %7.2f us per launch (overhead %.2f us)\n", ticks / 100.0, us, us - ticks / 100.0);
    }
    // graph of N launches
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_busy, dim3(1), dim3(256), 0, s1, 2000ull, sink);
    (void)hipStreamEndCapture(s1, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(ge, s1);
    (void)hipStreamSynchronize(s1);
    auto t0 = std::chrono::steady_clock::now();
    (void)hipGraphLaunch(ge, s1);
    (void)hipStreamSynchronize(s1);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
    printf("graph, busy 20.0 us: %7.2f us per launch (overhead %.2f us)\n", us, us - 20.0);
    // a second stream keeps 128 workgroups busy beside the single-workgroup chain
    run(s2, 10, 2000, sink, 128);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_busy, dim3(128), dim3(256), 0, s2, 1000ull, sink);
    const double us2 = run(s1, 200, 2000ull, sink, 1);
    (void)hipDeviceSynchronize();
    printf("with a busy second stream, busy 20.0 us: %7.2f us per launch (overhead %.2f us)\n", us2, us2 - 20.0);
    return 0;
}
