// On-device data ingest: the driver's preprocessing of dc:30-59
// moved next to the sweep, so a raw n x p matrix goes to HBM once and Yd is formed there.
//
//   k_nnz_cols  dc:31-34   nnzcol(j) = nnz(Y(:,j))  (NaN counts as non-zero, as nnz does)
//   k_colstats  dc:57      Md = mean, VYd = var (n-1) of Yd(:,j,m) = Y(:,varind(...)), and
//                          yy = sum_i Yd_ij^2 (the residual-SS identity's input)
//   k_stdize    dc:50-59   Yd = (Yd - Md) .* (1./sqrt(VYd)) -> the sweep's [G][NP][PP]
//                          layout, padding zero-filled
//
// Both are one-time HBM passes.  Input columns are contiguous n-vectors (MATLAB column
// major), so every read is a 64-lane run of 512 B; k_stdize's output is [i][j] (j fastest),
// so a 64-row x 16-column tile is transposed through LDS and written as 128 B row runs.
// Algorithmic bytes: k_nnz_cols 8 n p;  k_colstats 8 n P G (its 2nd / 3rd passes re-read
// the wave's column from L2);  k_stdize 8 n P G read + 8 NP PP G write.
#include "dcfm_internal.h"

namespace dcfm {

static __device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// one wave per input column, 4 columns per 256-thread block
__global__ __launch_bounds__(256) void k_nnz_cols(const double *__restrict__ Y, int n, long long p,
                                                  int *__restrict__ nnz) {
    const int lane = threadIdx.x & 63;
    const long long c = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= p) return;
    const double *x = Y + c * (long long)n;
    int cnt = 0;
    int i = lane;
    for (; i + 192 < n; i += 256) {   // four independent loads in flight per lane
        const double a = x[i], b = x[i + 64], e = x[i + 128], f = x[i + 192];
        cnt += (a != 0.0) + (b != 0.0) + (e != 0.0) + (f != 0.0);
    }
    for (; i < n; i += 64) cnt += (x[i] != 0.0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) nnz[c] = cnt;
}

constexpr int CS_R = 32;   // doubles per lane of a register-resident column (n <= 2,048)

// k_colstats: one wave per output column (m, j): dc:57 two-pass mean and var (n - 1) of
// the gathered input column, then sum_i Yd_ij^2 of the standardised column -> mean /
// 1/sqrt(var) / yy / sd; up to n = 2,048 (every BASELINE config) the column is loaded once
// into registers (32 loads in flight per lane) and the three passes run there.  Columns are independent waves, so the grid
// has P*G waves however few shards there are (c4: 10,000; the old fused kernel had 16
// columns per block and a serial chain per wave: 223 us at c4).
__global__ __launch_bounds__(256) void k_colstats(const double *__restrict__ Yraw, int n,
                                                  const long long *__restrict__ cols, int P, int G, int PP,
                                                  double *__restrict__ mean_inv, double *__restrict__ yy,
                                                  double *__restrict__ sd, int *__restrict__ bad) {
    const int lane = threadIdx.x & 63;
    const long long q = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);   // m * P + j
    if (q >= (long long)P * G) return;
    const int m = (int)(q / P), j = (int)(q % P);
    const double *x = Yraw + cols[q] * (long long)n;
    double mu, var, inv, ys;
    if (n <= 64 * CS_R) {   // the column held in registers: one memory read, all loads in flight
        double v[CS_R];
#pragma unroll
        for (int r = 0; r < CS_R; ++r) v[r] = lane + 64 * r < n ? x[lane + 64 * r] : 0.0;
        double s0 = 0.0;
#pragma unroll
        for (int r = 0; r < CS_R; ++r) s0 += v[r];
        mu = wave_sum64(s0) / n;
        double q0 = 0.0;
#pragma unroll
        for (int r = 0; r < CS_R; ++r) {
            const double a = lane + 64 * r < n ? v[r] - mu : 0.0;
            q0 += a * a;
        }
        var = wave_sum64(q0) / (n - 1);
        inv = 1.0 / sqrt(var);                              // dc:59 1./sqrt(VYd)
        double y0 = 0.0;                                    // yy of the standardised column
#pragma unroll
        for (int r = 0; r < CS_R; ++r) {
            const double a = lane + 64 * r < n ? (v[r] - mu) * inv : 0.0;
            y0 += a * a;
        }
        ys = wave_sum64(y0);
    } else {                // long columns: three passes, the 2nd and 3rd from L2
        double s0 = 0.0, s1 = 0.0;
        int i = lane;
        for (; i + 64 < n; i += 128) { s0 += x[i]; s1 += x[i + 64]; }
        if (i < n) s0 += x[i];
        mu = wave_sum64(s0 + s1) / n;
        double q0 = 0.0, q1 = 0.0;
        for (i = lane; i + 64 < n; i += 128) {
            const double a = x[i] - mu, b = x[i + 64] - mu;
            q0 += a * a;
            q1 += b * b;
        }
        if (i < n) { const double a = x[i] - mu; q0 += a * a; }
        var = wave_sum64(q0 + q1) / (n - 1);
        inv = 1.0 / sqrt(var);
        double y0 = 0.0, y1 = 0.0;
        for (i = lane; i + 64 < n; i += 128) {
            const double a = (x[i] - mu) * inv, b = (x[i + 64] - mu) * inv;
            y0 += a * a;
            y1 += b * b;
        }
        if (i < n) { const double a = (x[i] - mu) * inv; y0 += a * a; }
        ys = wave_sum64(y0 + y1);
    }
    if (lane == 0) {
        if (var == 0.0) atomicOr(bad, 1);                   // Q13: dc:59 divides by zero
        mean_inv[2 * q] = mu;
        mean_inv[2 * q + 1] = inv;
        yy[(size_t)m * PP + j] = ys;
        if (sd) sd[q] = sqrt(var);
    }
}

// k_stdize: dc:58-59 (Yd - Md) .* (1./sqrt(VYd)) into [G][NP][PP], a 64-row x 16-column
// tile per block (grid (PP/16, NP/64, G)) transposed through LDS; padding rows / columns
// written as zeros.  A pure stream: 8nP read (MALL / HBM) + 8 NP PP write per shard.
constexpr int ST_COLS = 16;
__global__ __launch_bounds__(256) void k_stdize(const double *__restrict__ Yraw, int n,
                                                const long long *__restrict__ cols, int P, int NP, int PP,
                                                const double *__restrict__ mean_inv, double *__restrict__ Y) {
    __shared__ double tile[ST_COLS][65];
    const int m = blockIdx.z, j0 = blockIdx.x * ST_COLS, i0 = blockIdx.y * 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = i0 + lane;
#pragma unroll
    for (int c = 0; c < ST_COLS / 4; ++c) {                 // wave w reads columns w*4 .. w*4+3
        const int jl = w * (ST_COLS / 4) + c, j = j0 + jl;
        double v = 0.0;
        if (j < P && i < n) {
            const long long q = (long long)m * P + j;
            v = (Yraw[cols[q] * (long long)n + i] - mean_inv[2 * q]) * mean_inv[2 * q + 1];
        }
        tile[jl][lane] = v;
    }
    __syncthreads();
    const int tc = threadIdx.x % ST_COLS, tr = threadIdx.x / ST_COLS, jw = j0 + tc;
    if (jw >= PP) return;
    double *Ym = Y + (size_t)m * NP * PP;
#pragma unroll
    for (int r = 0; r < 64 / (256 / ST_COLS); ++r) {
        const int il = tr + (256 / ST_COLS) * r, ii = i0 + il;
        if (ii < NP) Ym[(size_t)ii * PP + jw] = tile[tc][il];
    }
}

void launch_nnz_cols(const double *Y, int n, long long p, int *nnz, hipStream_t s) {
    if (p <= 0) return;
    hipLaunchKernelGGL(k_nnz_cols, dim3((unsigned)((p + 3) / 4)), dim3(256), 0, s, Y, n, p, nnz);
}

void launch_stdize(const Dims &d, const double *Yraw, const long long *cols, double *Y, double *yy, double *sd,
                   int *bad, double *mean_inv, hipStream_t s) {
    const long long ncol = (long long)d.P * d.G;
    hipLaunchKernelGGL(k_colstats, dim3((unsigned)((ncol + 3) / 4)), dim3(256), 0, s, Yraw, d.n, cols, d.P, d.G, d.PP,
                       mean_inv, yy, sd, bad);
    hipLaunchKernelGGL(k_stdize, dim3((d.PP + ST_COLS - 1) / ST_COLS, (d.NP + 63) / 64, d.G), dim3(256), 0, s, Yraw,
                       d.n, cols, d.P, d.NP, d.PP, mean_inv, Y);
}

}  // namespace dcfm
