// On-device data ingest: the driver's preprocessing of dc:30-59
// moved next to the sweep, so a raw n x p matrix goes to HBM once and Yd is formed there.
//
//   k_nnz_cols  dc:31-34   nnzcol(j) = nnz(Y(:,j))  (NaN counts as non-zero, as nnz does)
//   k_stdize    dc:50-59   Yd(:,:,m) = Y(:,varind(block m)); Md = mean; VYd = var (n-1);
//                          Yd = (Yd - Md) .* (1./sqrt(VYd))  -> the sweep's [G][NP][PP] layout,
//                          padding zero-filled, plus yy = sum_i Yd_ij^2 (the residual-SS
//                          identity's input, formerly computed on the host in dcfm_set_data)
//
// Both are one-time HBM passes.  Input columns are contiguous n-vectors (MATLAB column
// major), so every read is a 64-lane run of 512 B; k_stdize's output is [i][j] (j fastest),
// so a 64-row x 16-column tile is transposed through LDS and written as 128 B row runs.
// Algorithmic bytes: k_nnz_cols 8 n p;  k_stdize 8 n P G (read) + 8 NP PP G (write) + the
// two statistics passes, which re-read a block's 16 columns from L2 (16 x n x 8 B = 128 KB
// at n = 1,000).
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

constexpr int ST_COLS = 16;            // output columns per block (1,280 blocks at c3)
constexpr int ST_CPW = ST_COLS / 4;    // columns per wave
constexpr int ST_RG = 256 / ST_COLS;   // row groups of the transposed write

// grid (cdiv(PP, ST_COLS), G); cols[m * P + j] = input column of local shard m, position j
__global__ __launch_bounds__(256) void k_stdize(const double *__restrict__ Yraw, int n, const long long *__restrict__ cols,
                                                int P, int NP, int PP, double *__restrict__ Y,
                                                double *__restrict__ yy, double *__restrict__ sd,
                                                int *__restrict__ bad) {
    __shared__ double tile[ST_COLS][65];
    __shared__ double s_mean[ST_COLS], s_inv[ST_COLS];
    __shared__ double s_yy[ST_RG][ST_COLS];
    const int m = blockIdx.y, j0 = blockIdx.x * ST_COLS;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;

    // column base pointers of this wave's ST_CPW columns (null past P: padding columns)
    const double *src[ST_CPW];
#pragma unroll
    for (int c = 0; c < ST_CPW; ++c) {
        const int j = j0 + w * ST_CPW + c;
        src[c] = j < P ? Yraw + cols[(long long)m * P + j] * (long long)n : nullptr;
    }
    // dc:57 Md = mean(Yd), VYd = var(Yd) (two-pass, n - 1); the wave's columns advance
    // together so ST_CPW independent loads per lane are in flight in each pass
    double mu[ST_CPW], q[ST_CPW];
#pragma unroll
    for (int c = 0; c < ST_CPW; ++c) mu[c] = 0.0;
    for (int i = lane; i < n; i += 64) {
#pragma unroll
        for (int c = 0; c < ST_CPW; ++c)
            if (src[c]) mu[c] += src[c][i];
    }
#pragma unroll
    for (int c = 0; c < ST_CPW; ++c) { mu[c] = wave_sum64(mu[c]) / n; q[c] = 0.0; }
    for (int i = lane; i < n; i += 64) {
#pragma unroll
        for (int c = 0; c < ST_CPW; ++c)
            if (src[c]) { const double a = src[c][i] - mu[c]; q[c] += a * a; }
    }
#pragma unroll
    for (int c = 0; c < ST_CPW; ++c) {
        const int jl = w * ST_CPW + c;
        double inv = 0.0;
        if (src[c]) {
            const double var = wave_sum64(q[c]) / (n - 1);
            if (var == 0.0 && lane == 0) atomicOr(bad, 1);      // Q13: dc:59 divides by zero
            inv = 1.0 / sqrt(var);                              // dc:59 1./sqrt(VYd)
            if (sd && lane == 0) sd[(long long)m * P + j0 + jl] = sqrt(var);
        }
        if (lane == 0) { s_mean[jl] = src[c] ? mu[c] : 0.0; s_inv[jl] = inv; }
    }
    __syncthreads();

    // dc:58-59 centre and scale, transposed through LDS into [i][j]
    const int tc = threadIdx.x % ST_COLS, tr = threadIdx.x / ST_COLS;
    const int jw = j0 + tc;
    double acc = 0.0;
    double *Ym = Y + (size_t)m * NP * PP;
    for (int i0 = 0; i0 < NP; i0 += 64) {
        const int i = i0 + lane;
#pragma unroll
        for (int c = 0; c < ST_CPW; ++c) {
            const int jl = w * ST_CPW + c;
            double v = 0.0;
            if (src[c] && i < n) v = (src[c][i] - s_mean[jl]) * s_inv[jl];
            tile[jl][lane] = v;
        }
        __syncthreads();
        if (jw < PP) {
#pragma unroll
            for (int r = 0; r < 64 / ST_RG; ++r) {
                const int il = tr + ST_RG * r, ii = i0 + il;
                if (ii < NP) {
                    const double v = tile[tc][il];
                    Ym[(size_t)ii * PP + jw] = v;
                    acc += v * v;
                }
            }
        }
        __syncthreads();
    }
    s_yy[tr][tc] = acc;
    __syncthreads();
    if (threadIdx.x < ST_COLS && j0 + (int)threadIdx.x < PP) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < ST_RG; ++r) s += s_yy[r][threadIdx.x];
        yy[(size_t)m * PP + j0 + threadIdx.x] = s;
    }
}

void launch_nnz_cols(const double *Y, int n, long long p, int *nnz, hipStream_t s) {
    if (p <= 0) return;
    hipLaunchKernelGGL(k_nnz_cols, dim3((unsigned)((p + 3) / 4)), dim3(256), 0, s, Y, n, p, nnz);
}

void launch_stdize(const Dims &d, const double *Yraw, const long long *cols, double *Y, double *yy, double *sd,
                   int *bad, hipStream_t s) {
    hipLaunchKernelGGL(k_stdize, dim3((d.PP + ST_COLS - 1) / ST_COLS, d.G), dim3(256), 0, s, Yraw, d.n, cols,
                       d.P, d.NP, d.PP, Y, yy, sd, bad);
}

}  // namespace dcfm
