// Workgroup-level (any multiple of 64 threads) dense linear algebra on the K x K systems
// of the wide-factor path (K = 33..128): the Cholesky factor of Zprec / Xprec
// (dc:100,118 cholcov), L^{-1} and U U' — the Z / X draw operators (k_prep, k_xchol).
//
// Storage: the lower triangle as 16x16 tiles in LDS, tile (I, J), I >= J, at
// index I(I+1)/2 + J, each tile column-major with a 17-double pitch
// (element (r, c) at c*TLD + r).  nb = ceil(K/16) tile rows; rows >= K are an
// identity pad.
//   * diagonal tile: one quarter wave, lane = row, 16 right-looking steps with
//     v_mov_dpp row_newbcast broadcasts (compile-time lanes);
//   * panel below it: one lane per panel row, forward substitution against the
//     diagonal tile (LDS broadcast reads);
//   * trailing update A_IK -= L_IJ L_KJ' as v_mfma_f64_16x16x4 (4 k-steps per
//     tile, tiles dealt over the 4 waves).
// Three barriers per tile column: a K = 100 factorisation is 7 tile columns.
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

// Cholesky of the diagonal tile D in place (lower); dinv16[k] = 1/L_kk.
// Called by a whole wave; lanes 0..15 own the rows (lane = row r), the rest idle.
// The tile stays in LDS (register-light): step k reads the pivot, lane r > k
// scales its column-k entry, then updates its row from column k.  One wave, so
// LDS order is program order; wave_barrier keeps the compiler from reordering.
__device__ __forceinline__ void potrf16(double *D, double *dinv16, int lane) {
    if (lane >= TS) return;
    const int r = lane;
#pragma unroll 1
    for (int k = 0; k < TS; ++k) {
        const double piv = D[k * TLD + k];
        const double ikk = rsqrt_f64(piv);
        __builtin_amdgcn_wave_barrier();
        double lr = 0.0;
        if (r > k) {
            lr = D[k * TLD + r] * ikk;
            D[k * TLD + r] = lr;
        } else if (r == k) {
            D[k * TLD + k] = piv * ikk;
            dinv16[k] = ikk;
        }
        __builtin_amdgcn_wave_barrier();
        for (int c = k + 1; c <= r; ++c) D[c * TLD + r] = fma(-lr, D[k * TLD + c], D[c * TLD + r]);   // a_rc -= l_rk l_ck
        __builtin_amdgcn_wave_barrier();
    }
}

// L_IJ = A_IJ L_JJ^{-T} for every panel tile I > J; pair t: tile J+1+t/16, row t%16
__device__ __forceinline__ void trsm_panel_one(double *T, const double *dinv, int J, int nb, int t) {
    const int I = J + 1 + (t >> 4), r = t & 15;
    if (I >= nb) return;
    const double *L = T + tix(J, J) * TSZ;
    double *A = T + tix(I, J) * TSZ;
    double y[TS];
#pragma unroll
    for (int c = 0; c < TS; ++c) y[c] = A[c * TLD + r];
#pragma unroll
    for (int c = 0; c < TS; ++c) {
        double s = y[c];
#pragma unroll
        for (int c2 = 0; c2 < c; ++c2) s = fma(-L[c2 * TLD + c], y[c2], s);   // L_JJ[c][c2]
        y[c] = s * dinv[TS * J + c];
        asm volatile("" ::: "memory");   // keep each step's L_JJ loads in the step (else all 120 are hoisted)
    }
#pragma unroll
    for (int c = 0; c < TS; ++c) A[c * TLD + r] = y[c];
}
__device__ __forceinline__ void trsm_panel(double *T, const double *dinv, int J, int nb) {
    for (int t = threadIdx.x; t < (nb - 1 - J) * TS; t += blockDim.x) trsm_panel_one(T, dinv, J, nb, t);
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

// trailing update after tile column J: A_IK -= L_IJ L_KJ' for J < K <= I < nb
__device__ __forceinline__ void trailing(double *T, int J, int nb, int wave, int lane) {
    const int m = nb - 1 - J, ntr = m * (m + 1) / 2, nw = blockDim.x >> 6;
    for (int tt = wave; tt < ntr; tt += nw) {
        int a, b;
        tri_pair(tt, a, b);
        const int I = J + 1 + a, K = J + 1 + b;
        tile_nt_acc(T + tix(I, K) * TSZ, T + tix(I, J) * TSZ, T + tix(K, J) * TSZ, -1.0, lane);
    }
}

// blocked right-looking Cholesky of the tiled lower triangle (any multiple of 64 threads)
__device__ __forceinline__ void potrf(double *T, double *dinv, int nb) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
#pragma unroll 1
    for (int J = 0; J < nb; ++J) {
        if (wave == 0) potrf16(T + tix(J, J) * TSZ, dinv + TS * J, lane);
        __syncthreads();
        trsm_panel(T, dinv, J, nb);
        __syncthreads();
        trailing(T, J, nb, wave, lane);
        __syncthreads();
    }
}

// U = L^{-1} into the tiled array U (same layout).  Diagonal tiles by forward
// substitution (thread per column), then per tile column J (waves take J = w mod 4):
//   U_IJ = -U_II sum_{K=J}^{I-1} L_IK U_KJ   (two MFMA products per tile)
__device__ __forceinline__ void trtri(const double *T, const double *dinv, double *U, int nb) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    for (int e = t; e < nb * TS; e += blockDim.x) {
        const int J = e >> 4, c = e & 15;
        const double *L = T + tix(J, J) * TSZ;
        double *Ud = U + tix(J, J) * TSZ;
        double u[TS];
#pragma unroll
        for (int r = 0; r < TS; ++r) {
            double s = (r == c) ? 1.0 : 0.0;
#pragma unroll
            for (int r2 = 0; r2 < r; ++r2) s = fma(-L[r2 * TLD + r], u[r2], s);
            u[r] = (r >= c) ? s * dinv[TS * J + r] : 0.0;
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int r = 0; r < TS; ++r) Ud[c * TLD + r] = u[r];
    }
    __syncthreads();
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
            for (int s = 0; s < 4; ++s) R = mfma16x16x4(-Uii[(4 * s + kq) * TLD + i], S[s], R);
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
        for (int e = t; e < nb * TS * nb * TS; e += blockDim.x) {
            const int row = e / (nb * TS), col = e % (nb * TS);
            double v = 0.0;
            if (row < N && col < N && row >= col) v = U[tix(row >> 4, col >> 4) * TSZ + (col & 15) * TLD + (row & 15)];
            uout[(size_t)row * ld + col] = v;
        }
    }
}

}  // namespace tile
}  // namespace dcfm
