// Latency microbenchmarks for the resolver's building blocks on gfx950 (one workgroup, shader
// clocks from s_memtime): dependent ballot->ff1->readlane chain, LDS read round trip, s_barrier
// with 8 waves, VALU dependent add, f64 fma chain, global load (L2) round trip.
// Build: hipcc --offload-arch=gfx950 -O3 lat_micro.hip -o lat_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

constexpr int IT = 1024;

__global__ __launch_bounds__(512) void k_lat(uint64_t *out, const uint32_t *gsrc, uint32_t seed) {
    __shared__ uint32_t lds[4096];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4096; i += 512) lds[i] = (i * 7 + 1) & 4095;
    __syncthreads();
    uint64_t t0, t1;
    // 0: stamp overhead
    t0 = stamp();
    t1 = stamp();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    // 1: ballot -> ff1 -> readlane chain (wave 0)
    if (threadIdx.x < 64) {
        uint32_t v = (lane * 13 + seed) & 63, x = seed & 63;
        t0 = stamp();
        for (int i = 0; i < IT; ++i) {
            const uint64_t m = __ballot(v >= x);
            const int l = m ? (int)__builtin_ctzll(m) : 0;
            x = (uint32_t)__builtin_amdgcn_readlane((int)v, l) ^ (uint32_t)i & 31u;
        }
        t1 = stamp();
        if (lane == 0) { out[1] = t1 - t0; out[15] = x; }
    }
    __syncthreads();
    // 2: LDS dependent read chain (wave 0)
    if (threadIdx.x < 64) {
        uint32_t idx = lane;
        t0 = stamp();
        for (int i = 0; i < IT; ++i) idx = lds[idx];
        t1 = stamp();
        if (lane == 0) { out[2] = t1 - t0; out[14] = idx; }
    }
    __syncthreads();
    // 3: barrier with 8 waves
    t0 = stamp();
    for (int i = 0; i < IT; ++i) __syncthreads();
    t1 = stamp();
    if (threadIdx.x == 0) out[3] = t1 - t0;
    // 4: VALU dependent add chain
    if (threadIdx.x < 64) {
        uint32_t a = lane;
        t0 = stamp();
        for (int i = 0; i < IT; ++i) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(a));
        }
        t1 = stamp();
        if (lane == 0) { out[4] = t1 - t0; out[13] = a; }
    }
    // 5: f64 fma chain
    if (threadIdx.x < 64) {
        double d = lane * 0.5;
        t0 = stamp();
        for (int i = 0; i < IT; ++i) d = __builtin_fma(d, 0.999, 0.001);
        t1 = stamp();
        if (lane == 0) { out[5] = t1 - t0; out[12] = (uint64_t)d; }
    }
    // 6: global load dependent chain (pointer chase within a 64 KB buffer: L2)
    if (threadIdx.x < 64) {
        uint32_t idx = lane;
        t0 = stamp();
        for (int i = 0; i < IT / 8; ++i) idx = gsrc[idx];
        t1 = stamp();
        if (lane == 0) { out[6] = (t1 - t0) * 8; out[11] = idx; }
    }
    // 7: LDS write then read (same wave) round trip
    if (threadIdx.x < 64) {
        uint32_t v = lane;
        t0 = stamp();
        for (int i = 0; i < IT; ++i) {
            lds[2048 + lane] = v + 1;
            v = lds[2048 + ((lane + 1) & 63)];
        }
        t1 = stamp();
        if (lane == 0) { out[7] = t1 - t0; out[10] = v; }
    }
    __syncthreads();
    // 8: barrier + LDS flag hand-off between waves 0 and 1 (ping-pong through __syncthreads)
    {
        uint32_t v = 0;
        t0 = stamp();
        for (int i = 0; i < IT; ++i) {
            if (threadIdx.x == 64) lds[3000] = i;
            __syncthreads();
            v += lds[3000];
            __syncthreads();
        }
        t1 = stamp();
        if (threadIdx.x == 0) { out[8] = t1 - t0; out[9] = v; }
    }
}

int main() {
    uint64_t *d;
    uint32_t *g;
    hipMalloc(&d, 16 * 8);
    hipMalloc(&g, 65536 * 4);
    uint32_t *h = (uint32_t *)malloc(65536 * 4);
    for (int i = 0; i < 65536; ++i) h[i] = (uint32_t)((i * 40503u + 977u) & 16383u);
    hipMemcpy(g, h, 65536 * 4, hipMemcpyHostToDevice);
    uint64_t o[16];
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(512), 0, 0, d, g, 5u + r);
        hipMemcpy(o, d, 16 * 8, hipMemcpyDeviceToHost);
    }
    const char *nm[] = {"stamp pair", "ballot-ff1-readlane", "lds read", "barrier(8 waves)", "v_add dep",
                        "f64 fma dep", "global load (L2)", "lds write+read", "barrier+lds handoff (2 barriers)"};
    printf("cycles per op (s_memtime):\n");
    printf("  %-34s %8.1f\n", nm[0], (double)o[0]);
    for (int k = 1; k < 9; ++k) printf("  %-34s %8.1f\n", nm[k], (double)o[k] / IT);
    hipFree(d);
    hipFree(g);
    return 0;
}
