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


// variant B of chol16_step: the quad writes column k (every lane of row r the same value,
// no exec-mask branch), dr by select
template <int J>
__device__ __forceinline__ void stepB(double &a0, double &a1, double &a2, double &a3, double &R0, double &R1,
                                      double &R2, double &R3, double &dr, int kk, int r, int cg,
                                      double *lds_l, double *lds_u) {
    const int k = 4 * kk + J;
    const double v = quad_bcast<J>(a0);                         // a[r][k]
    lds_l[r] = (r > k) ? v : 0.0;
    if (r == k) {
        lds_u[cg] = R0; lds_u[4 + cg] = R1; lds_u[8 + cg] = R2; lds_u[12 + cg] = R3;
    }
    __builtin_amdgcn_wave_barrier();
    const double *pl = lds_l + 4 * kk + cg;
    const double l0 = pl[0], l1 = pl[4], l2 = pl[8], l3 = pl[12];
    const double u0 = lds_u[cg], u1 = lds_u[4 + cg], u2 = lds_u[8 + cg], u3 = lds_u[12 + cg];
    __builtin_amdgcn_sched_barrier(0);
    const double piv = readlane_d(a0, 4 * k + J);
    const double f = (r > k) ? v * rcp_f64(piv) : 0.0;
    a0 = fma(-f, l0, a0); a1 = fma(-f, l1, a1); a2 = fma(-f, l2, a2); a3 = fma(-f, l3, a3);
    R0 = fma(-f, u0, R0); R1 = fma(-f, u1, R1); R2 = fma(-f, u2, R2); R3 = fma(-f, u3, R3);
    dr = (r == k) ? piv : dr;
    __builtin_amdgcn_wave_barrier();
}
// variant C: no LDS for the column (pivot column values from readlanes of a0 is impossible
// in general; here: timing only, the column taken from the own registers) -- latency probe
template <int J>
__device__ __forceinline__ void stepC(double &a0, double &a1, double &a2, double &a3, double &R0, double &R1,
                                      double &R2, double &R3, double &dr, int kk, int r, int cg,
                                      double *lds_l, double *lds_u) {
    const int k = 4 * kk + J;
    const double v = quad_bcast<J>(a0);
    const double piv = readlane_d(a0, 4 * k + J);
    const double f = (r > k) ? v * rcp_f64(piv) : 0.0;
    a0 = fma(-f, a1, a0); a1 = fma(-f, a2, a1); a2 = fma(-f, a3, a2); a3 = fma(-f, v, a3);
    R0 = fma(-f, a1, R0); R1 = fma(-f, a2, R1); R2 = fma(-f, a3, R2); R3 = fma(-f, v, R3);
    dr = (r == k) ? piv : dr;
}

__device__ __forceinline__ double bperm_d(double x, int src_lane) {
    const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2loint(x));
    const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2hiint(x));
    return __hiloint2double(hi, lo);
}
// variant D: column k and row k of W fetched with ds_bpermute (no LDS memory round trip)
template <int J>
__device__ __forceinline__ void stepD(double &a0, double &a1, double &a2, double &a3, double &R0, double &R1,
                                      double &R2, double &R3, double &dr, int kk, int r, int cg,
                                      double *, double *) {
    const int k = 4 * kk + J;
    // column k: a[c][k] for c = 4 (kk + i) + cg is a0 of lane 4 c + J
    const int c0 = 4 * kk + cg;
    double l0 = bperm_d(a0, (4 * c0 + J) & 63), l1 = bperm_d(a0, (4 * (c0 + 4) + J) & 63);
    double l2 = bperm_d(a0, (4 * (c0 + 8) + J) & 63), l3 = bperm_d(a0, (4 * (c0 + 12) + J) & 63);
    // row k of W: R_i of lane 4 k + cg
    const int src = 4 * k + cg;
    const double u0 = bperm_d(R0, src), u1 = bperm_d(R1, src), u2 = bperm_d(R2, src), u3 = bperm_d(R3, src);
    const double v = quad_bcast<J>(a0);
    const double piv = readlane_d(a0, 4 * k + J);
    l0 = (c0 > k && c0 < 16) ? l0 : 0.0; l1 = (c0 + 4 > k && c0 + 4 < 16) ? l1 : 0.0;
    l2 = (c0 + 8 > k && c0 + 8 < 16) ? l2 : 0.0; l3 = (c0 + 12 > k && c0 + 12 < 16) ? l3 : 0.0;
    const double f = (r > k) ? v * rcp_f64(piv) : 0.0;
    a0 = fma(-f, l0, a0); a1 = fma(-f, l1, a1); a2 = fma(-f, l2, a2); a3 = fma(-f, l3, a3);
    R0 = fma(-f, u0, R0); R1 = fma(-f, u1, R1); R2 = fma(-f, u2, R2); R3 = fma(-f, u3, R3);
    dr = (r == k) ? piv : dr;
}


// variant E: every lane stores its row of W each step into a 16 x 16 image (no branch)
template <int J>
__device__ __forceinline__ void stepE(double &a0, double &a1, double &a2, double &a3, double &R0, double &R1,
                                      double &R2, double &R3, double &dr, int kk, int r, int cg,
                                      double *lds_l, double *lds_w) {
    const int k = 4 * kk + J;
    const double v = quad_bcast<J>(a0);
    lds_l[r] = (r > k) ? v : 0.0;
    double *wr = lds_w + r * 16 + cg;
    wr[0] = R0; wr[4] = R1; wr[8] = R2; wr[12] = R3;
    __builtin_amdgcn_wave_barrier();
    const double *pl = lds_l + 4 * kk + cg;
    const double l0 = pl[0], l1 = pl[4], l2 = pl[8], l3 = pl[12];
    const double *wk = lds_w + k * 16 + cg;
    const double u0 = wk[0], u1 = wk[4], u2 = wk[8], u3 = wk[12];
    __builtin_amdgcn_sched_barrier(0);
    const double piv = readlane_d(a0, 4 * k + J);
    const double f = (r > k) ? v * rcp_f64(piv) : 0.0;
    a0 = fma(-f, l0, a0); a1 = fma(-f, l1, a1); a2 = fma(-f, l2, a2); a3 = fma(-f, l3, a3);
    R0 = fma(-f, u0, R0); R1 = fma(-f, u1, R1); R2 = fma(-f, u2, R2); R3 = fma(-f, u3, R3);
    dr = (r == k) ? piv : dr;
    __builtin_amdgcn_wave_barrier();
}

template <int V>
__device__ __forceinline__ void cholX(const double *Sm, double *Ub, double *lds_l, double *lds_u, int lane) {
    constexpr int LDP = 17;
    const int r = lane >> 2, cg = lane & 3;
    const double *srow = Sm + r * LDP + cg;
    double a0 = srow[0], a1 = srow[4], a2 = srow[8], a3 = srow[12];
    double R0 = (cg == r) ? 1.0 : 0.0, R1 = (4 + cg == r) ? 1.0 : 0.0;
    double R2 = (8 + cg == r) ? 1.0 : 0.0, R3 = (12 + cg == r) ? 1.0 : 0.0;
    double dr = 1.0;
    if (lane < 16) lds_l[16 + lane] = 0.0;
#pragma unroll 1
    for (int kk = 0; kk < 4; ++kk) {
        if (V == 4) {
            stepE<0>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepE<1>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepE<2>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepE<3>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        } else if (V == 3) {
            stepD<0>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepD<1>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepD<2>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepD<3>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        } else if (V == 1) {
            stepB<0>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepB<1>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepB<2>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepB<3>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        } else {
            stepC<0>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepC<1>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepC<2>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
            stepC<3>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        }
        a0 = a1; a1 = a2; a2 = a3; a3 = 0.0;
    }
    const double ik = rsqrt_f64(dr);
    double *urow = Ub + r * LDP + cg;
    urow[0] = R0 * ik; urow[4] = R1 * ik; urow[8] = R2 * ik; urow[12] = R3 * ik;
}

__global__ __launch_bounds__(64) void bench(double *sink, unsigned long long *cyc, int reps) {
    constexpr int LD = 17;
    __shared__ double Sd[16 * LD], Ud[16 * LD], lds_l[32], lds_u[256], X[64];
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
    {   // agreement of the variants with chol_inv16_p (max abs diff over the tile, into cyc[.. + 5] bits)
        __shared__ double U1[16 * 17], U3[16 * 17];
        chol_inv16_p<17>(Sd, 0, Ud, lds_l, lds_u, lane);
        __builtin_amdgcn_wave_barrier();
        cholX<1>(Sd, U1, lds_l, lds_u, lane);
        __builtin_amdgcn_wave_barrier();
        cholX<4>(Sd, U3, lds_l, lds_u, lane);
        __syncthreads();
        double md = 0.0;
        for (int e = lane; e < 256; e += 64) {
            const int i = e >> 4, c = e & 15;
            md = fmax(md, fabs(U1[i * 17 + c] - Ud[i * 17 + c]));
            md = fmax(md, fabs(U3[i * 17 + c] - Ud[i * 17 + c]));
        }
        for (int o = 32; o >= 1; o >>= 1) md = fmax(md, __shfl_xor(md, o, 64));
        if (blockIdx.x == 0 && lane == 0) sink[1023 * 64] = md;
    }
    // (6) variant B, (7) variant D
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
        cholX<1>(Sd, Ud, lds_l, lds_u, lane);
        __builtin_amdgcn_wave_barrier();
        acc += Ud[lane];
    }
    t1 = stamp();
    if (lane == 0) cyc[blockIdx.x * 8 + 6] = (t1 - t0) / reps;
    t0 = stamp();
    for (int it = 0; it < reps; ++it) {
        cholX<4>(Sd, Ud, lds_l, lds_u, lane);
        __builtin_amdgcn_wave_barrier();
        acc += Ud[lane];
    }
    t1 = stamp();
    if (lane == 0) cyc[blockIdx.x * 8 + 7] = (t1 - t0) / reps;
    sink[blockIdx.x * 64 + lane] = acc;
}

int main() {
    const int nb = 1024, reps = 50;
    double *sink; unsigned long long *cyc;
    hipMalloc(&sink, nb * 64 * sizeof(double));
    hipMalloc(&cyc, nb * 8 * sizeof(unsigned long long));
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) { double md; hipMemcpy(&md, sink + 1023 * 64, 8, hipMemcpyDeviceToHost); printf("variants vs chol_inv16_p: max |diff| %.3e\n", md); }
        hipLaunchKernelGGL(bench, dim3(pass ? nb : 1), dim3(64), 0, 0, sink, cyc, reps);
        hipDeviceSynchronize();
        unsigned long long h[8 * 1024];
        const int n = pass ? nb : 1;
        hipMemcpy(h, cyc, n * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double s[8] = {0};
        for (int b = 0; b < n; ++b) for (int i = 0; i < 8; ++i) s[i] += h[b * 8 + i];
        printf("%s: chol_inv16 %.0f cyc | fma %.1f | lds rt %.1f | rcp_f64 %.1f | rsqrt_f64 %.1f | readlane+add %.1f (cycles per op)\n",
               pass ? "1024 waves" : "1 wave", s[0] / n, s[1] / n / 100, s[2] / n / 100, s[3] / n / 100, s[4] / n / 100, s[5] / n / 100);
        printf("   variant B (branch-light) %.0f cyc | variant E (W image) %.0f cyc\n", s[6] / n, s[7] / n);
    }
    return 0;
}
