// Residual-precision update by the reference's own formula (DCFM_FLAG_EXACT_RESIDUAL).
//
// divideconquer.m:168-172:   Ytil = Yd(:,:,m) - eta(:,:,m)*Lambda(:,:,m)';
//                            ps(:,:,m) = gamrnd(as + 0.5*n, 1./(bs + 0.5*sum(Ytil.^2)));
//                            Omega(:,:,m) = diag(1./ps(:,:,m));
//
// The default chain forms SS_j = sum_i Ytil_ij^2 inside k_lambda by the identity
// yy_j - 2 lambda_j.C_j + lambda_j E lambda_j' (no Y pass).  That sum cancels when SS_j is
// small against its terms: its rounding error grows like kappa_j eps with kappa_j = (yy_j +
// 2 sum_k |lambda_jk C_jk| + |lambda_j| |E| |lambda_j|') / SS_j (measured ~1e6 at the second
// iteration of config c2, where the X excursions make E large: 1.3e-10 relative in SS).  The
// direct residual's error grows like sqrt(kappa_j) eps.  With the flag, this kernel runs after
// k_lambda / k_lambda_w and overwrites ps and omega from the direct residual: a third pass over
// Y (the reference's own third product) for parity runs; the identity stays the throughput path.
//
// k_resid<KW>: block = (32-column tile of shard m's loading rows, shard m), 4 waves splitting the
// rows i in 16-row chunks.  Per chunk a wave forms Ytil for 16 rows x 32 columns as fp64 MFMA
// v_mfma_f64_16x16x4 with the Y tile as the C operand and -eta as A (D = Y - eta Lambda', the
// subtraction of dc:169 inside the accumulation), A[i = lane&15][k], B[k][j = lane&15] with k =
// 8t + 2q (+1) so both operands are 16-byte pair loads; lane (c, q) then holds Ytil for rows
// i0 + q + 4v of column j0 + c and squares them into its column sum.  The 16 lanes of a column,
// then the 4 waves, are summed in a fixed order; the column's ps_j, omega_j use the same standard
// gamma variate k_lambda read (Gps: LamDraws layout).
#include "dcfm_internal.h"
#include "linalg.h"

namespace dcfm {

constexpr int RS_WAVES = 4;

template <int KW>
__global__ __launch_bounds__(64 * RS_WAVES) void k_resid(Dims d, const double *__restrict__ Y,
                                                        const double *__restrict__ X, const double *__restrict__ Z,
                                                        const double *__restrict__ Lam, const double *__restrict__ Gps,
                                                        double *__restrict__ ps, double *__restrict__ omega) {
    constexpr int NT = KW / 8;                  // k steps of 8 (two MFMAs each)
    __shared__ double red[RS_WAVES][32];
    const int m = blockIdx.y, j0 = blockIdx.x * 32;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, q = lane >> 4;
    const double *Ym = Y + (size_t)m * d.NP * d.PP;
    const double *Zm = Z + (size_t)m * d.NP * KW;
    // B operands: Lambda rows j0 + 16h + c, columns 8t + 2q, +1 (register-resident for the block)
    d2 lb[2][NT];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < NT; ++t)
            lb[h][t] = *reinterpret_cast<const d2 *>(Lam + ((size_t)m * d.PP + j0 + 16 * h + c) * KW + 8 * t + 2 * q);
    double ss[2] = {0.0, 0.0};
    const int nch = d.NP / 16;
    for (int ch = w; ch < nch; ch += RS_WAVES) {
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
        ss[h] += __shfl_xor(ss[h], 16, 64);
        ss[h] += __shfl_xor(ss[h], 32, 64);
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
            ps[(size_t)m * d.PP + j] = psn;
            omega[(size_t)m * d.PP + j] = 1.0 / psn;                                  // dc:171 (Q1)
        }
    }
}

void launch_resid(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s, bool gen) {
    const double *Gps;
    if (gen) Gps = lam_gen_plan(d, b.ldraw[iter & 1]).Gps;   // the generated fused chain's slot
    else Gps = dr.Gps + ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
    const dim3 grid(d.PP / 32, d.G);
    switch (d.kp) {
    case 32: hipLaunchKernelGGL(k_resid<32>, grid, dim3(64 * RS_WAVES), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    case 64: hipLaunchKernelGGL(k_resid<64>, grid, dim3(64 * RS_WAVES), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    default: hipLaunchKernelGGL(k_resid<128>, grid, dim3(64 * RS_WAVES), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    }
}

}  // namespace dcfm
