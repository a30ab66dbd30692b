// Microbenchmark (dev aid): fp64 v_mfma_f64_16x16x4 throughput vs independent accumulator
// chains per wave and waves per SIMD.  Build: hipcc -O3 --offload-arch=gfx950 mfma_chains.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int NC>
__global__ __launch_bounds__(256) void chains(double *out, int iters, double a0) {
    double a = a0 + threadIdx.x * 1e-3, b = a0 - threadIdx.x * 1e-3;
    d4 c[NC];
#pragma unroll
    for (int u = 0; u < NC; ++u) c[u] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < NC; ++u) c[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[u], 0, 0, 0);
        a += 1e-9;   // keep the operands live
    }
    double s = 0;
#pragma unroll
    for (int u = 0; u < NC; ++u) s += c[u][0] + c[u][1] + c[u][2] + c[u][3];
    if (s == 12345.0) out[0] = s;
}

template <int NC>
int run(double *out, hipEvent_t e0, hipEvent_t e1) {
    for (int wps : {1, 2, 4, 8}) {
        const int grid = 256 * wps;            // 4 waves per block: wps waves per SIMD
        const int iters = 2048 / NC * 8;
        hipLaunchKernelGGL(chains<NC>, dim3(grid), dim3(256), 0, 0, out, 4, 1.0);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(chains<NC>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double flops = (double)grid * 4 * iters * NC * 2048.0;
        printf("chains/wave %2d  waves/SIMD %d  chains/SIMD %3d  %6.1f TFLOP/s\n", NC, wps, NC * wps,
               flops / (ms * 1e-3) / 1e12);
    }
    return 0;
}

int main() {
    double *out;
    CHECK(hipMalloc(&out, 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    run<1>(out, e0, e1);
    run<2>(out, e0, e1);
    run<4>(out, e0, e1);
    run<8>(out, e0, e1);
    run<16>(out, e0, e1);
    return 0;
}
