// FETCH_SIZE / WRITE_SIZE calibration per access width on gfx950 (dev aid):
// streams a 2 GiB buffer (8x the Infinity Cache) with 8 B/lane and 16 B/lane loads
// and stores; compare the counters with the known byte count per dispatch.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d2v __attribute__((ext_vector_type(2)));
__global__ void rd8(const double *__restrict__ a, size_t n, double *out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    if (s == 12345.678) out[0] = s;
}
__global__ void rd16(const d2v *__restrict__ a, size_t n2, double *out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) { d2v v = a[i]; s += v.x + v.y; }
    if (s == 12345.678) out[0] = s;
}
__global__ void wr8(double *a, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = 1.0;
}
__global__ void wr16(d2v *a, size_t n2) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) a[i] = d2v{1.0, 2.0};
}
int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 8;
    double *a, *o;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipMemset(a, 0, bytes);
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(rd8, dim3(8192), dim3(256), 0, 0, a, n, o);
        hipLaunchKernelGGL(rd16, dim3(8192), dim3(256), 0, 0, (const d2v *)a, n / 2, o);
        hipLaunchKernelGGL(wr8, dim3(8192), dim3(256), 0, 0, a, n);
        hipLaunchKernelGGL(wr16, dim3(8192), dim3(256), 0, 0, (d2v *)a, n / 2);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("bytes per dispatch %zu\n", bytes);
    return 0;
}
