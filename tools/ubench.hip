// Microbenchmarks for the roofline peaks used in DESIGN.md / bench.py:
//  (1) fp64 MFMA v_mfma_f64_16x16x4_f64 issue rate (independent accumulators);
//  (2) fp64 VALU FMA rate;
//  (3) HBM streaming read bandwidth (16 B per lane, grid-stride).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench.hip -o tools/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void mfma_peak(double *out, int iters, double a0) {
    double a = a0 + threadIdx.x * 1e-3, b = a0 - threadIdx.x * 1e-3;
    d4 c[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) c[u] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[u], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += c[u][0] + c[u][1] + c[u][2] + c[u][3];
    if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void valu_peak(double *out, int iters, double a0) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = a0 + u + threadIdx.x;
    const double m = 0.999999, ad = 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = fma(x[u], m, ad);
    }
    double s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
    if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void stream_read(const d2 *__restrict__ in, size_t n, double *out) {
    d2 acc = {0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += in[i];
    if (acc.x + acc.y == 12345.0) out[0] = acc.x;
}

int main() {
    double *out;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float ms;
    const int iters = 4000;
    for (int wpb : {1, 2, 4}) {  // waves per SIMD
        const int grid = 256 * wpb;
        hipLaunchKernelGGL(mfma_peak, dim3(grid), dim3(256), 0, 0, out, 10, 1.0);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(mfma_peak, dim3(grid), dim3(256), 0, 0, out, iters, 1.0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double flops = (double)grid * 4 * iters * 8 * 2048.0;
        printf("fp64 MFMA 16x16x4: %d waves/SIMD  %.1f TFLOP/s\n", wpb, flops / (ms * 1e-3) / 1e12);
    }
    for (int wpb : {1, 2, 4}) {
        const int grid = 256 * wpb;
        hipLaunchKernelGGL(valu_peak, dim3(grid), dim3(256), 0, 0, out, 10, 1.0);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(valu_peak, dim3(grid), dim3(256), 0, 0, out, iters, 1.0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double flops = (double)grid * 256 * iters * 8 * 2.0;
        printf("fp64 VALU fma:     %d waves/SIMD  %.1f TFLOP/s\n", wpb, flops / (ms * 1e-3) / 1e12);
    }
    const size_t bytes = (size_t)2 << 30;   // 2 GiB (past the 256 MiB Infinity Cache)
    d2 *buf;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0, bytes));
    const size_t n = bytes / sizeof(d2);
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(stream_read, dim3(256 * 16), dim3(256), 0, 0, buf, n, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("HBM stream read (2 GiB): %.0f GB/s\n", bytes / (ms * 1e-3) / 1e9);
    }
    const size_t small = (size_t)160 << 20;   // 160 MiB (c3 Y fits the Infinity Cache)
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(stream_read, dim3(256 * 16), dim3(256), 0, 0, buf, small / sizeof(d2), out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("stream read 160 MiB (MALL-resident after rep 0): %.0f GB/s\n", small / (ms * 1e-3) / 1e9);
    }
    return 0;
}
