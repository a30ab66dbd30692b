// Error of the posterior-mean covariance against a synthetic truth, on the device.
//
// SURVEY §8(f) row 2 / north_star check (2): the reference's output Sigmaout
// (dc:194-196, p x p in permuted, standardised coordinates, Q7) is compared with the
// truth Sigma0 = U U' + diag(s) given in the same coordinates (U p x r, r <= 32: the
// sparse loadings of the generator, permuted by varind and divided by the sample
// standard deviations, dc:50-59).  At c5 Sigmaout is 80 GB: it never leaves HBM.
//
// k_sigma_err: block = 32 rows [r0, r0 + 32) of M = Sigmaout - Sigma0, all p columns
// in 32 x 32 tiles.  The accumulator holds the lower triangle S[r][c], r >= c (row
// major, dc:194-195's symmetrisation is the mirror), so a tile left of the diagonal is
// read along c and a tile right of it is read as S[c][r] along r (coalesced both ways,
// transposed through LDS).  Sigma0's tile is U_rows U_cols' + diag(s) from LDS.  Per
// row: y_r = sum_c M_rc v_c (the Lanczos matvec), and on the first pass sum_c M_rc^2
// and sum_c Sigma0_rc^2 (Frobenius norms).  Every block writes its rows' sums; the
// host adds rows in a fixed order, so results are deterministic.
//
// Several ranks: the accumulator is block-sharded (dcfm_internal.h): rank r holds the
// tile rows [T0, T1) of the lower triangle, tile-packed.  A rank counts only the elements
// it owns — S minus truth, both — so the per-rank sums and matvecs add up exactly to those
// of the full matrix.
//
// Roofline: HBM-bound, 8 p^2 bytes per pass (the full matrix, both halves of the
// stored triangle); U / s / v are L2-resident.
#include <hip/hip_runtime.h>

#include "dcfm_internal.h"

#include <algorithm>

namespace dcfm {

constexpr int ERR_RMAX = 32;
#ifndef ERR_NT
#define ERR_NT 2   // 32 x 32 tiles per pipelined step
#endif
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// stored element (a, b), a >= b: does this rank own it (tile row a / 128 in [T0, T1))?
__device__ __forceinline__ bool owns(int a, int T0, int T1) {
    const int ta = a / ASM_TILE;
    return ta >= T0 && ta < T1;
}

template <int RM>
__global__ __launch_bounds__(256) void k_sigma_err(const double *__restrict__ S, int p,
                                                   const double *__restrict__ U, int R,
                                                   const double *__restrict__ sdiag,
                                                   const double *__restrict__ v, int T0, int T1,
                                                   int first, double *__restrict__ y,
                                                   double *__restrict__ fro, double *__restrict__ tru) {
    constexpr int NT = ERR_NT;
    __shared__ double tile[NT][32][33];
    __shared__ double Uc[NT][32][RM + 1];
    __shared__ double vc[NT][32];
    __shared__ bool okt[NT][32][33];
    const int t = threadIdx.x, tx = t & 31, ty = t >> 5;
    const int r0 = blockIdx.x * 32;
    // compute mapping: thread = (row i = t >> 3, columns j = (t & 7) + 8 q); the row's
    // truth factors stay in registers for the whole stripe
    const int ri = t >> 3, cj = t & 7;
    const int r = r0 + ri;
    double ur[RM];
#pragma unroll
    for (int k = 0; k < RM; ++k) ur[k] = (r < p && k < R) ? U[(size_t)k * p + r] : 0.0;
    const double sr = r < p ? sdiag[r] : 0.0;
    double ysum = 0.0, fsum = 0.0, tsum = 0.0;
    // this block's share of the column tiles (gridDim.y splits: enough blocks in flight
    // to cover HBM latency; the sum over splits runs in a fixed order)
    const int nct = (p + 31) / 32, per = (nct + gridDim.y - 1) / gridDim.y;
    const int ct0 = blockIdx.y * per, ct1 = min(nct, ct0 + per);
    // One load per thread and slot, coalesced along tx in every case:
    //   left of the diagonal (c0 < r0): S[r0 + yy][c0 + tx] -> tile (yy, tx)
    //   right of it (c0 > r0):          S[c0 + yy][r0 + tx] -> tile (tx, yy)
    //   the diagonal tile (c0 == r0):   S[r0 + yy][r0 + tx], tx <= yy -> (yy, tx) and (tx, yy)
    // NT tiles per step; the next step's loads are issued before this step is computed,
    // so a block keeps NT tiles of HBM reads in flight across the compute phase.
    double sv_[NT][4], ucv[NT][RM / 8], vv[NT];
    bool ok_[NT][4];
    auto fetch = [&](int cs) {
#pragma unroll
        for (int u = 0; u < NT; ++u) {
            const int ct = cs + u, c0 = ct * 32;
            const bool live = ct < ct1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int yy = ty + 8 * i;
                int a, b;
                bool ok;
                if (c0 < r0) { a = r0 + yy; b = c0 + tx; ok = true; }
                else if (c0 > r0) { a = c0 + yy; b = r0 + tx; ok = true; }
                else { a = r0 + yy; b = r0 + tx; ok = tx <= yy; }
                ok = ok && live && a < p && b < p && owns(a, T0, T1);
                ok_[u][i] = ok;
                sv_[u][i] = ok ? S[sig_off(a, b, T0)] : 0.0;
            }
#pragma unroll
            for (int i = 0; i < RM / 8; ++i) {
                const int e = t + 256 * i, ci = e / RM, k = e % RM;
                ucv[u][i] = (live && c0 + ci < p && k < R) ? U[(size_t)k * p + c0 + ci] : 0.0;
            }
            vv[u] = (t < 32 && v && live && c0 + t < p) ? v[c0 + t] : 0.0;
        }
    };
    auto commit = [&](int cs) {
#pragma unroll
        for (int u = 0; u < NT; ++u) {
            const int c0 = (cs + u) * 32;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int yy = ty + 8 * i;
                if (c0 < r0) {
                    tile[u][yy][tx] = sv_[u][i];
                    okt[u][yy][tx] = ok_[u][i];
                } else if (c0 > r0) {
                    tile[u][tx][yy] = sv_[u][i];
                    okt[u][tx][yy] = ok_[u][i];
                } else {
                    if (tx <= yy) {
                        tile[u][yy][tx] = sv_[u][i];
                        okt[u][yy][tx] = ok_[u][i];
                    }
                    if (tx < yy) {
                        tile[u][tx][yy] = sv_[u][i];
                        okt[u][tx][yy] = ok_[u][i];
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < RM / 8; ++i) {
                const int e = t + 256 * i;
                Uc[u][e / RM][e % RM] = ucv[u][i];
            }
            if (t < 32) vc[u][t] = vv[u];
        }
    };
    if (ct0 < ct1) fetch(ct0);
    for (int cs = ct0; cs < ct1; cs += NT) {
        __syncthreads();   // previous step consumed
        commit(cs);
        __syncthreads();
        if (cs + NT < ct1) fetch(cs + NT);
        if (r < p) {
#pragma unroll
            for (int u = 0; u < NT; ++u) {
                const int c0 = (cs + u) * 32;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int j = cj + 8 * q, c = c0 + j;
                    if (okt[u][ri][j]) {
                        double tv = (r == c) ? sr : 0.0;
#pragma unroll
                        for (int k = 0; k < RM; ++k)
                            if (k < R) tv = fma(ur[k], Uc[u][j][k], tv);
                        const double m = tile[u][ri][j] - tv;
                        ysum = fma(m, vc[u][j], ysum);
                        if (first) {
                            fsum = fma(m, m, fsum);
                            tsum = fma(tv, tv, tsum);
                        }
                    }
                }
            }
        }
    }
    // the 8 threads of a row are adjacent lanes: fixed-order butterfly
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        ysum += __shfl_xor(ysum, o, 8);
        fsum += __shfl_xor(fsum, o, 8);
        tsum += __shfl_xor(tsum, o, 8);
    }
    if (cj == 0 && r < p) {   // partials of split blockIdx.y
        const size_t o = (size_t)blockIdx.y * p + r;
        if (y) y[o] = ysum;
        if (first) {
            fro[o] = fsum;
            tru[o] = tsum;
        }
    }
}

// out[r] = sum over splits s of part[s][r], in split order (deterministic)
__global__ __launch_bounds__(256) void k_sigma_err_sum(const double *__restrict__ part, int ns, int p,
                                                       double *__restrict__ out) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= p) return;
    double acc = 0.0;
    for (int s2 = 0; s2 < ns; ++s2) acc += part[(size_t)s2 * p + r];
    out[r] = acc;
}

int sigma_err_splits(int p) {
    const int nrs = cdiv(p, 32), nct = nrs;
    return std::max(1, std::min(nct, 8192 / nrs));
}
// y / fro / tru: [splits][p] partials; work: 3 x p outputs (y, fro, tru summed over splits)
void launch_sigma_err(const double *S, int p, const double *U, int R, const double *sdiag, const double *v,
                      int T0, int T1, bool first, double *y, double *fro, double *tru, double *out,
                      hipStream_t s) {
    const int ns = sigma_err_splits(p);
    if (R <= 16)
        hipLaunchKernelGGL(k_sigma_err<16>, dim3(cdiv(p, 32), ns), dim3(256), 0, s, S, p, U, R, sdiag, v, T0,
                           T1, first ? 1 : 0, y, fro, tru);
    else
        hipLaunchKernelGGL(k_sigma_err<ERR_RMAX>, dim3(cdiv(p, 32), ns), dim3(256), 0, s, S, p, U, R, sdiag, v,
                           T0, T1, first ? 1 : 0, y, fro, tru);
    if (y) hipLaunchKernelGGL(k_sigma_err_sum, dim3(cdiv(p, 256)), dim3(256), 0, s, y, ns, p, out);
    if (first) {
        hipLaunchKernelGGL(k_sigma_err_sum, dim3(cdiv(p, 256)), dim3(256), 0, s, fro, ns, p, out + p);
        hipLaunchKernelGGL(k_sigma_err_sum, dim3(cdiv(p, 256)), dim3(256), 0, s, tru, ns, p, out + 2 * (size_t)p);
    }
}

}  // namespace dcfm
