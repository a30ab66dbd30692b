// Latency / throughput of the device building blocks of the sweep (diagnostic only).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I <pkg>/csrc tools/ubench_chol.hip -o tools/ubench_chol
#include <hip/hip_runtime.h>
#include <cstdio>
#include "linalg.h"
#include "philox.h"

using namespace dcfm;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// one wave: 2 SPD matrices (one per half-wave).  Records cycles of each stage.
__global__ __launch_bounds__(64) void lat(double *sink, unsigned long long *cyc, int reps) {
    __shared__ double Lt[KP][LS];
    __shared__ double Lp[2][PSTRIDE];
    const int lane = threadIdx.x, r = lane & 31;
    const bool upper = lane >= 32;
    double acc = 0.0;
    unsigned long long t0, t1;
    // (0) chol_rows
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
        double q[KP];
#pragma unroll
        for (int c = 0; c < KP; ++c) q[c] = (c == r ? 40.0 + it : 0.0) + 1.0 / (1.0 + r + c);
        chol_rows(q, Lt, r, upper);
        acc += q[r];
    }
    t1 = stamp();
    if (lane == 0) cyc[0] = (t1 - t0) / reps;
    // (1) chol_rows_fwd
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
        double q[KP];
#pragma unroll
        for (int c = 0; c < KP; ++c) q[c] = (c == r ? 40.0 + it : 0.0) + 1.0 / (1.0 + r + c);
        double vr = 0.0;
        chol_rows_fwd(q, Lp[upper], r, upper, 1.0 + r, vr);
        acc += vr;
    }
    t1 = stamp();
    if (lane == 0) cyc[1] = (t1 - t0) / reps;
    // (8) chol2_rows<true> (2-column blocked, fused forward solve)
    __shared__ __attribute__((aligned(16))) double P2[2][P2STRIDE];
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
        double q[KP];
#pragma unroll
        for (int c = 0; c < KP; ++c) q[c] = (c == r ? 40.0 + it : 0.0) + 1.0 / (1.0 + r + c);
        double vr = 0.0;
        chol2_rows<true>(q, P2[upper], r, upper, 1.0 + r, vr);
        acc += vr;
    }
    t1 = stamp();
    if (lane == 0) cyc[8] = (t1 - t0) / reps;
    // (2) readsel chain
    double x = 1.0 + lane;
    t0 = stamp();
    for (int it = 0; it < reps * 32; ++it) x = readsel(x, it & 31, upper) * 1.0000001 + 1e-9;
    t1 = stamp();
    acc += x;
    if (lane == 0) cyc[2] = (t1 - t0) / (reps * 32);
    // (3) rsqrt chain
    x = 2.0 + lane;
    t0 = stamp();
    for (int it = 0; it < reps * 32; ++it) x = rsqrt_f64(x) + 1.5;
    t1 = stamp();
    acc += x;
    if (lane == 0) cyc[3] = (t1 - t0) / (reps * 32);
    // (4) divide chain
    x = 2.0 + lane;
    t0 = stamp();
    for (int it = 0; it < reps * 32; ++it) x = 1.0 / x + 1.5;
    t1 = stamp();
    acc += x;
    if (lane == 0) cyc[4] = (t1 - t0) / (reps * 32);
    // (5) Philox normal pair
    const Rng rng(7);
    t0 = stamp();
    for (int it = 0; it < reps * 8; ++it) {
        double a, b;
        rng.normal2(1, lane, it, 0, 1, a, b);
        acc += a + b;
    }
    t1 = stamp();
    if (lane == 0) cyc[5] = (t1 - t0) / (reps * 8);
    // (6) gamma(501)
    t0 = stamp();
    for (int it = 0; it < reps * 8; ++it) acc += rng.gamma(501.0, 6, lane, it, 0, 1);
    t1 = stamp();
    if (lane == 0) cyc[6] = (t1 - t0) / (reps * 8);
    // (7) LDS write -> read round trip (same wave)
    double *buf = &Lt[0][0];
    x = lane;
    t0 = stamp();
    for (int it = 0; it < reps * 32; ++it) {
        buf[lane] = x;
        x = buf[(lane + 1) & 63] + 1.0;
    }
    t1 = stamp();
    acc += x;
    if (lane == 0) cyc[7] = (t1 - t0) / (reps * 32);
    sink[blockIdx.x * 64 + lane] = acc;
}

// throughput: many waves each factoring 2 matrices with chol_rows_fwd + back-solve
__global__ __launch_bounds__(256) void thr(double *sink, int reps) {
    __shared__ double LP[8][PSTRIDE];
    const int lane = threadIdx.x & 63, r = lane & 31, hw = threadIdx.x >> 5;
    const bool upper = lane >= 32;
    double acc = 0.0;
    for (int it = 0; it < reps; ++it) {
        double q[KP];
#pragma unroll
        for (int c = 0; c < KP; ++c) q[c] = (c == r ? 40.0 + it : 0.0) + 1.0 / (1.0 + r + c + blockIdx.x);
        double vr = 0.0;
        chol_rows_fwd(q, LP[hw], r, upper, 1.0 + r, vr);
        acc += vr;
    }
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    double *sink;
    unsigned long long *cyc;
    CHECK(hipMalloc(&sink, 1 << 24));
    CHECK(hipMalloc(&cyc, 64 * 8));
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, sink, cyc, 4);
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, sink, cyc, 16);
    unsigned long long h[9];
    CHECK(hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost));
    const char *names[9] = {"chol_rows (32x32, 2/wave)", "chol_rows_fwd", "readsel", "rsqrt_f64",
                            "fp64 1/x", "philox normal2", "gamma(501)", "LDS write->read", "chol2_rows<fwd>"};
    for (int i = 0; i < 9; ++i) printf("%-28s %8llu cycles (s_memtime)\n", names[i], h[i]);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int blocks : {256, 768, 2496}) {
        hipLaunchKernelGGL(thr, dim3(blocks), dim3(256), 0, 0, sink, 2);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(thr, dim3(blocks), dim3(256), 0, 0, sink, 4);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("chol_rows_fwd throughput: %d blocks x 8 rows x 4 reps = %d factorisations in %.1f us (%.2f ns each)\n",
               blocks, blocks * 32, ms * 1e3, ms * 1e6 / (blocks * 32));
    }
    return 0;
}
