// Diagnostic only: per-call cycles of chol_inv16_p on a loaded chip (1,024 one-wave blocks,
// one per SIMD), plus its building blocks: dependent fp64 FMA latency, an LDS write->read
// round trip within a wave, v_rcp_f64 + refinement, readlane.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I <pkg>/csrc tools/ubench3/c16.hip -o tools/ubench3/c16
#include <hip/hip_runtime.h>
#include <cstdio>
#include "linalg.h"
using namespace dcfm;

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ __launch_bounds__(64) void bench(double *sink, unsigned long long *cyc, int reps) {
    constexpr int LD = 17;
    __shared__ double Sd[16 * LD], Ud[16 * LD], lds_l[32], lds_u[16], X[64];
    const int lane = threadIdx.x, r = lane >> 2, cg = lane & 3;
    double acc = 0.0;
    for (int e = lane; e < 16 * 16; e += 64) {
        const int i = e >> 4, c = e & 15;
        Sd[i * LD + c] = (i == c ? 20.0 : 0.0) + 1.0 / (1.0 + i + c);
    }
    __syncthreads();
    unsigned long long t0, t1;
    // (0) chol_inv16_p
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
        chol_inv16_p<LD>(Sd, 0, Ud, lds_l, lds_u, lane);
        __builtin_amdgcn_wave_barrier();
        acc += Ud[lane];
    }
    t1 = stamp();
    if (lane == 0) cyc[blockIdx.x * 8 + 0] = (t1 - t0) / reps;
    // (1) 100 dependent fp64 FMAs
    double x = 1.0 + lane * 1e-3;
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int u = 0; u < 100; ++u) x = fma(x, 0.999999, 1e-9);
    }
    t1 = stamp();
    acc += x;
    if (lane == 0) cyc[blockIdx.x * 8 + 1] = (t1 - t0) / reps;     // per 100
    // (2) LDS write -> wave barrier -> read of another lane's value, 100 dependent rounds
    double y = lane;
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int u = 0; u < 100; ++u) {
            X[lane] = y;
            __builtin_amdgcn_wave_barrier();
            y = X[(lane + 1) & 63] + 1.0;
            __builtin_amdgcn_wave_barrier();
        }
    }
    t1 = stamp();
    acc += y;
    if (lane == 0) cyc[blockIdx.x * 8 + 2] = (t1 - t0) / reps;     // per 100
    // (3) rcp_f64 chain, 100 dependent
    double z = 3.0 + lane;
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int u = 0; u < 100; ++u) z = rcp_f64(z) + 2.0;
    }
    t1 = stamp();
    acc += z;
    if (lane == 0) cyc[blockIdx.x * 8 + 3] = (t1 - t0) / reps;     // per 100
    // (4) rsqrt_f64 chain, 100 dependent
    double w = 3.0 + lane;
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int u = 0; u < 100; ++u) w = rsqrt_f64(w) + 2.0;
    }
    t1 = stamp();
    acc += w;
    if (lane == 0) cyc[blockIdx.x * 8 + 4] = (t1 - t0) / reps;     // per 100
    // (5) readlane of a freshly written VGPR, 100 dependent
    double v = lane;
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int u = 0; u < 100; ++u) v = readlane_d(v, u & 63) + 1.0;
    }
    t1 = stamp();
    acc += v;
    if (lane == 0) cyc[blockIdx.x * 8 + 5] = (t1 - t0) / reps;     // per 100
    sink[blockIdx.x * 64 + lane] = acc;
}

int main() {
    const int nb = 1024, reps = 50;
    double *sink; unsigned long long *cyc;
    hipMalloc(&sink, nb * 64 * sizeof(double));
    hipMalloc(&cyc, nb * 8 * sizeof(unsigned long long));
    for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL(bench, dim3(pass ? nb : 1), dim3(64), 0, 0, sink, cyc, reps);
        hipDeviceSynchronize();
        unsigned long long h[8 * 1024];
        const int n = pass ? nb : 1;
        hipMemcpy(h, cyc, n * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double s[6] = {0};
        for (int b = 0; b < n; ++b) for (int i = 0; i < 6; ++i) s[i] += h[b * 8 + i];
        printf("%s: chol_inv16 %.0f cyc | fma %.1f | lds rt %.1f | rcp_f64 %.1f | rsqrt_f64 %.1f | readlane+add %.1f (cycles per op)\n",
               pass ? "1024 waves" : "1 wave", s[0] / n, s[1] / n / 100, s[2] / n / 100, s[3] / n / 100, s[4] / n / 100, s[5] / n / 100);
    }
    return 0;
}
