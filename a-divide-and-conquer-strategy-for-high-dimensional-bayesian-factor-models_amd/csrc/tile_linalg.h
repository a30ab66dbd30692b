// Workgroup-level (any multiple of 64 threads) dense linear algebra on the K x K systems
// of the wide-factor path (K = 33..128): the Cholesky factor of Zprec / Xprec
// (dc:100,118 cholcov), L^{-1} and U U' — the Z / X draw operators (k_prep, k_xchol).
//
// Storage: the lower triangle as 16x16 tiles in LDS, tile (I, J), I >= J, at
// index I(I+1)/2 + J, each tile column-major with a 17-double pitch
// (element (r, c) at c*TLD + r).  nb = ceil(K/16) tile rows; rows >= K are an
// identity pad.
//   * diagonal tile: one wave, chol_inv16 (its inverse U_JJ as well), one column ahead of
//     the trailing update (potrf_inv's look-ahead);
//   * panel below it: L_IJ = A_IJ U_JJ' as v_mfma_f64_16x16x4;
//   * trailing update A_IK -= L_IJ L_KJ' as v_mfma_f64_16x16x4 (4 k-steps per
//     tile, tiles dealt over the other waves).
// Two barriers per tile column: a K = 100 factorisation is 7 tile columns.
#pragma once
#include "linalg.h"

namespace dcfm {
namespace tile {

constexpr int TS = 16, TLD = 17, TSZ = TS * TLD;

__host__ __device__ constexpr int tix(int I, int J) { return I * (I + 1) / 2 + J; }
__host__ __device__ constexpr int ntiles(int nb) { return nb * (nb + 1) / 2; }

// (a, b), a >= b, of the t-th lower-triangular pair in row-major order
__device__ __forceinline__ void tri_pair(int t, int &a, int &b) {
    a = 0;
    while ((a + 1) * (a + 2) / 2 <= t) ++a;
    b = t - a * (a + 1) / 2;
}

// C(I,K) += sgn * A(I,J) B(K,J)'  for one 16x16 tile pair, fp64 MFMA (whole wave)
__device__ __forceinline__ void tile_nt_acc(double *C, const double *A, const double *B, double sgn, int lane) {
    const int i = lane & 15, kq = lane >> 4;
    d4 acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = C[i * TLD + kq + 4 * g];
#pragma unroll
    for (int s = 0; s < 4; ++s)
        acc = mfma16x16x4(sgn * A[(4 * s + kq) * TLD + i], B[(4 * s + kq) * TLD + i], acc);
#pragma unroll
    for (int g = 0; g < 4; ++g) C[i * TLD + kq + 4 * g] = acc[g];
}

// Blocked right-looking Cholesky of the tiled lower triangle together with the diagonal
// blocks of its inverse (any multiple of 64 threads, at least two waves).  Per tile column J: the
// panel tiles become L_IJ = A_IJ U_JJ' (one MFMA product each, tiles dealt over the waves); then
// wave 0 takes the next diagonal tile's update A_{J+1,J+1} -= L_{J+1,J} L_{J+1,J}' and factors it
// (chol_inv16, LDL' form: U_{J+1,J+1} = L^{-1} into U) while the other waves run the rest of the
// trailing update A_IK -= L_IJ L_KJ' (look-ahead: the one-wave factorisation, the serial part,
// overlaps the trailing update instead of following it).  Every tile sees the same operations in
// the same order as without the look-ahead.  The diagonal tiles stay symmetric (the trailing
// product updates the whole tile), so chol_inv16's row-major read of the column-major tile sees the
// same values.
__device__ __forceinline__ void potrf_inv(double *T, double *U, int nb, double *lds_l, double *lds_u) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, nw = blockDim.x >> 6;
    const int i = lane & 15, kq = lane >> 4;
    // the look-ahead gives the trailing update to waves 1 .. nw - 1: every caller launches at least
    // two waves (kernels_wide.hip static_asserts TILE_THREADS >= 128)
    if (wave == 0) chol_inv16_p<TLD, true>(T, 0, U, lds_l, lds_u, lane);
    __syncthreads();
#pragma unroll 1
    for (int J = 0; J < nb; ++J) {
        const double *Uj = U + tix(J, J) * TSZ;
        for (int I = J + 1 + wave; I < nb; I += nw) {
            double *A = T + tix(I, J) * TSZ;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s) acc = mfma16x16x4(A[(4 * s + kq) * TLD + i], Uj[(4 * s + kq) * TLD + i], acc);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int g = 0; g < 4; ++g) A[i * TLD + kq + 4 * g] = acc[g];
        }
        __syncthreads();
        if (J + 1 == nb) break;
        if (wave == 0) {
            double *D = T + tix(J + 1, J + 1) * TSZ;
            const double *L = T + tix(J + 1, J) * TSZ;
            tile_nt_acc(D, L, L, -1.0, lane);
            __builtin_amdgcn_wave_barrier();              // D's LDS stores before chol_inv16_p's reads
            asm volatile("" ::: "memory");
            chol_inv16_p<TLD, true>(D, 0, U + tix(J + 1, J + 1) * TSZ, lds_l, lds_u, lane);
        } else {   // trailing tiles of column J but the next diagonal one (tri_pair(0))
            const int m = nb - 1 - J, ntr = m * (m + 1) / 2;
            for (int tt = wave; tt < ntr; tt += nw - 1) {
                int a, b;
                tri_pair(tt, a, b);
                const int I = J + 1 + a, K = J + 1 + b;
                tile_nt_acc(T + tix(I, K) * TSZ, T + tix(I, J) * TSZ, T + tix(K, J) * TSZ, -1.0, lane);
            }
        }
        __syncthreads();
    }
}

// U = L^{-1} below the diagonal blocks (potrf_inv wrote U_JJ), per tile column J (waves take
// J = w mod 4):  U_IJ = -U_II sum_{K=J}^{I-1} L_IK U_KJ   (two MFMA products per tile)
__device__ __forceinline__ void trtri(const double *T, double *U, int nb) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int i = lane & 15, kq = lane >> 4;
    for (int J = wave; J < nb; J += (int)(blockDim.x >> 6)) {
        for (int I = J + 1; I < nb; ++I) {
            d4 S = {0.0, 0.0, 0.0, 0.0};
            for (int K = J; K < I; ++K) {
                const double *A = T + tix(I, K) * TSZ, *B = U + tix(K, J) * TSZ;
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    S = mfma16x16x4(A[(4 * s + kq) * TLD + i], B[i * TLD + 4 * s + kq], S);
            }
            const double *Uii = U + tix(I, I) * TSZ;
            d4 R = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s) R = mfma16x16x4_na(Uii[(4 * s + kq) * TLD + i], S[s], R);
            double *Uij = U + tix(I, J) * TSZ;
#pragma unroll
            for (int g = 0; g < 4; ++g) Uij[i * TLD + kq + 4 * g] = R[g];
        }
    }
    __syncthreads();
}

// out (row-major, ld, global) = scale * U U' (symmetric, both triangles), entries
// with row or column >= N are written 0.  Also writes U itself (lower, 0 above) to
// uout when uout != nullptr.
__device__ __forceinline__ void uut_store(const double *U, int nb, int N, double scale, double *out, int ld, double *uout) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int i = lane & 15, kq = lane >> 4;
    const int npair = ntiles(nb);
    for (int tt = wave; tt < npair; tt += (int)(blockDim.x >> 6)) {
        int I, K;
        tri_pair(tt, I, K);
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int J = 0; J <= K; ++J) {
            const double *A = U + tix(I, J) * TSZ, *B = U + tix(K, J) * TSZ;
#pragma unroll
            for (int s = 0; s < 4; ++s)
                acc = mfma16x16x4(A[(4 * s + kq) * TLD + i], B[(4 * s + kq) * TLD + i], acc);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int row = TS * I + kq + 4 * g, col = TS * K + i;   // D[q+4g][j]
            const double v = (row < N && col < N) ? scale * acc[g] : 0.0;
            if (I != K || row >= col) {                                // lower element, then its mirror
                out[(size_t)row * ld + col] = v;
                out[(size_t)col * ld + row] = v;
            }
        }
    }
    if (uout) {
        const int nr = nb * TS;
        for (int row = wave; row < nr; row += (int)(blockDim.x >> 6))
            for (int col = lane; col < nr; col += 64) {
                double v = 0.0;
                if (row < N && col < N && row >= col) v = U[tix(row >> 4, col >> 4) * TSZ + (col & 15) * TLD + (row & 15)];
                uout[(size_t)row * ld + col] = v;
            }
    }
}

}  // namespace tile
}  // namespace dcfm
