// Dev aid: accuracy of fp64 reciprocal square root variants on gfx950 against a long-double-free
// reference (x^{-1/2} from the 2-Newton form refined once more in double-double).  Prints the max
// relative error (in units of 2^-52) of: the hardware v_rsq_f64 estimate, one Newton step, one Halley
// step (y (1 + e/2 + 3e^2/8)), two Newton steps (rsqrt_f64 of linalg.h).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

__device__ double newton1(double x, double y) { const double e = fma(-x * y, y, 1.0); return fma(0.5 * y, e, y); }
__global__ void k(const double *x, double *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    const double y0 = __builtin_amdgcn_rsq(v);
    const double y1 = newton1(v, y0);
    const double e = fma(-v * y0, y0, 1.0);
    const double yh = fma(y0 * e, fma(e, 0.375, 0.5), y0);
    const double y2 = newton1(v, y1);
    out[4 * i + 0] = y0; out[4 * i + 1] = y1; out[4 * i + 2] = yh; out[4 * i + 3] = y2;
}
int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), o(4 * (size_t)n);
    unsigned long long s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        const double u = (double)(s >> 11) / 9007199254740992.0;
        x[i] = std::ldexp(1.0 + u, (int)((s >> 3) % 200) - 100);
    }
    double *dx, *dout;
    hipMalloc(&dx, n * 8); hipMalloc(&dout, 4 * (size_t)n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
    hipMemcpy(o.data(), dout, 4 * (size_t)n * 8, hipMemcpyDeviceToHost);
    double worst[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const long double ref = 1.0L / std::sqrt((long double)x[i]);
        for (int v = 0; v < 4; ++v) {
            const double r = (double)std::fabs(((long double)o[4 * (size_t)i + v] - ref) / ref) / 2.220446049250313e-16;
            if (r > worst[v]) worst[v] = r;
        }
    }
    printf("max rel err / 2^-52: hw %.3g  newton1 %.3g  halley %.3g  newton2 %.3g\n", worst[0], worst[1], worst[2], worst[3]);
    return 0;
}
