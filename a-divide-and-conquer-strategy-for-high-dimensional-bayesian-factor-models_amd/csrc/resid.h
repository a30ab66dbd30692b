// The residual-precision update by the reference's own formula, one tile of 32 loading rows
// (divideconquer.m:168-172):   Ytil = Yd(:,:,m) - eta(:,:,m)*Lambda(:,:,m)';
//                              ps(:,:,m) = gamrnd(as + 0.5*n, 1./(bs + 0.5*sum(Ytil.^2)));
//                              Omega(:,:,m) = diag(1./ps(:,:,m));
// Used by k_resid (resid.hip: every tile with DCFM_FLAG_EXACT_RESIDUAL) and k_resid_flagged (the
// K > 32 tiles whose SS identity k_lambda_w's guard rejected).  k_lambda's guard (K <= 32) runs
// the same arithmetic per wave for its 8 rows (resid_rows8 in lambda.h), not this tile.
//
// 256 threads = 4 waves splitting the rows i in 16-row chunks.  Per chunk a wave forms Ytil for
// 16 rows x 32 columns as fp64 MFMA v_mfma_f64_16x16x4 with the Y tile as the C operand and -eta
// as A (D = Y - eta Lambda', the subtraction of dc:169 inside the accumulation), A[i = lane&15][k],
// B[k][j = lane&15] with k = 8t + 2q (+1) so both operands are 16-byte pair loads; lane (c, q) then
// holds Ytil for rows i0 + q + 4v of column j0 + c and squares them into its column sum.  The 4
// lanes of a column, then the 4 waves, are summed in a fixed order; ps_j, omega_j use the row's
// standard gamma variate (Gps, LamDraws layout [G][P]).
#pragma once
#include "dcfm_internal.h"
#include "linalg.h"

namespace dcfm {

// COH: Lambda was written by this launch (agent-scope stores): read it with agent-scope loads
template <int KW, bool COH = false>
__device__ __forceinline__ void resid_tile(const Dims &d, const double *__restrict__ Y, const double *__restrict__ X,
                                           const double *__restrict__ Z, const double *__restrict__ Lam,
                                           const double *__restrict__ Gps, double *__restrict__ ps,
                                           double *__restrict__ omega, int m, int j0, double (*red)[32]) {
    constexpr int NT = KW / 8;                  // k steps of 8 (two MFMAs each)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, q = lane >> 4;
    const double *Ym = Y + (size_t)m * d.NP * d.PP;
    const double *Zm = Z + (size_t)m * d.NP * KW;
    // B operands: Lambda rows j0 + 16h + c, columns 8t + 2q, +1 (register-resident for the tile)
    d2 lb[2][NT];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const double *pl = Lam + ((size_t)m * d.PP + j0 + 16 * h + c) * KW + 8 * t + 2 * q;
            if constexpr (COH) {
                lb[h][t].x = ld_agent(pl);
                lb[h][t].y = ld_agent(pl + 1);
            } else {
                lb[h][t] = *reinterpret_cast<const d2 *>(pl);
            }
        }
    double ss[2] = {0.0, 0.0};
    const int nch = d.NP / 16;
    for (int ch = w; ch < nch; ch += 4) {
        const int i0 = 16 * ch;
        d4 acc[2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[h][v] = Ym[(size_t)(i0 + q + 4 * v) * d.PP + j0 + 16 * h + c];
        const double *xr = X + (size_t)(i0 + c) * KW + 2 * q;
        const double *zr = Zm + (size_t)(i0 + c) * KW + 2 * q;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const d2 xa = *reinterpret_cast<const d2 *>(xr + 8 * t);
            const d2 za = *reinterpret_cast<const d2 *>(zr + 8 * t);
            const double e0 = -eta_of(d.sr, d.s1r, xa.x, za.x), e1 = -eta_of(d.sr, d.s1r, xa.y, za.y);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                acc[h] = mfma16x16x4(e0, lb[h][t].x, acc[h]);
                acc[h] = mfma16x16x4(e1, lb[h][t].y, acc[h]);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const double r = acc[h][v];
                ss[h] = (i0 + q + 4 * v < d.n) ? fma(r, r, ss[h]) : ss[h];   // padding rows: not data
            }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // the column's 4 lane rows: (q0 + q1) + (q2 + q3)
        ss[h] += xor16_d(ss[h]);
        ss[h] += xor32_d(ss[h]);
    }
    if (q == 0) {
        red[w][c] = ss[0];
        red[w][16 + c] = ss[1];
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        const int j = j0 + threadIdx.x;
        const double SS = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        if (j < d.P) {
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps[(size_t)m * d.P + j];   // dc:170
            st_agent(ps + (size_t)m * d.PP + j, psn);
            st_agent(omega + (size_t)m * d.PP + j, 1.0 / psn);                        // dc:171 (Q1)
        }
    }
}

}  // namespace dcfm
