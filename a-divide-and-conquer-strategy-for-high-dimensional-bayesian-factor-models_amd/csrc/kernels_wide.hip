// Wide-factor kernels (K = 33 .. 128, padded width KW = 64 or 128) for the Gibbs
// sweep of divideconquer.m:90-178.  Config c4 of BASELINE.json (p = 10,000,
// n = 2,000, K = 100) runs here; K <= 32 uses the register-blocked narrow
// kernels of kernels.hip.  The layout-generic kernels (k_wpass, k_cpass, k_xred,
// k_asum, k_save, k_assemble) are shared and templated on KW in kernels.hip.
//
// Kernel map (same dataflow as the narrow path)                reference lines
//   k_gram     A_m = Lambda' diag(w) Lambda, 32x32 tiles, fp64 MFMA    dc:98-99,114-115
//   k_prep     Zprec chol (LDS, packed), U = L^-1, T = U U',           dc:100-107
//              Z-draw operators {M1 = s1r T, U} of shard m
//   k_xchol    Xprec = g I + rho sum A, chol, {Tx, Ux}                  dc:117-118
//   k_zdraw    V' = W' - sr A X'; Z' = M1 V' + U eps';                  dc:101-107,121-123
//              S' = W' - s1r A Z'                             fp64 MFMA
//   k_xdraw    X' = Tx S' + Ux eps'                           fp64 MFMA  dc:119-128
//   k_lambda   one workgroup per loading row j: register-blocked        dc:140-145,150,
//              Cholesky of Q_j (8x8 blocks per thread), fused forward   dc:156,169-171
//              solve, blocked back solve; psi, SS identity, ps, omega
//   k_delta    MGP chain over up to 128 factors (2 per lane)            dc:155-165
#include <cmath>
#include <cstdlib>

#include "dcfm_internal.h"
#include "philox.h"
#include "linalg.h"
#include "tile_linalg.h"

namespace dcfm {
namespace wide {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// ============================================================================
// k_gram: A_m = (w o Lambda_m)' Lambda_m, 32x32 tile (ta, tb) per block; the GRAM_WAVES
// waves take the k-steps (4 rows j each) round-robin, one register prefetch ahead, and the
// partial tiles are summed in LDS in a fixed order (pairwise tree).  16 waves: the c4 launch
// is 128 blocks, each wave's chain a latency-bound run of dependent loads and MFMAs (4 waves:
// 40 us, on the critical path between k_lambda and the W pass).                     dc:98-99
// Lane (r, q), k-step s: rows j = 4s + q; A operand w_j L[j][32ta+2r+ea],
// B operand L[j][32tb+2r+eb]  ->  acc[ea][eb][g] = A[32ta+2(q+4g)+ea][32tb+2r+eb].
// ============================================================================
#ifndef DCFM_GRAM_WAVES
#define DCFM_GRAM_WAVES 16
#endif
constexpr int GRAM_WAVES = DCFM_GRAM_WAVES;
template <int KW>
__global__ __launch_bounds__(64 * GRAM_WAVES) void k_gram(Dims d, const double *__restrict__ Lam,
                                                          const double *__restrict__ omega, double *__restrict__ A) {
    constexpr int KT = KW / 32;
    __shared__ double red[GRAM_WAVES][32][33];
    const int m = blockIdx.y, ta = blockIdx.x / KT, tb = blockIdx.x % KT;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, q = lane >> 4;
    const double *L = Lam + (size_t)m * d.PP * KW;
    const double *w = omega + (size_t)m * d.PP;
    const int nks = d.PP >> 2;                 // k-steps of 4 rows
    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    auto ld = [&](int s, double &wj, d2 &la, d2 &lb) {
        const int j = 4 * (s < nks ? s : nks - 1) + q;   // clamped: the prefetch past the end is unused
        wj = w[j];
        la = *reinterpret_cast<const d2 *>(L + (size_t)j * KW + 32 * ta + 2 * r);
        lb = *reinterpret_cast<const d2 *>(L + (size_t)j * KW + 32 * tb + 2 * r);
    };
    double wj;
    d2 la, lb;
    ld(wave, wj, la, lb);
    for (int s = wave; s < nks; s += GRAM_WAVES) {
        double wn;
        d2 lan, lbn;
        ld(s + GRAM_WAVES, wn, lan, lbn);
        const double a0 = la.x * wj, a1 = la.y * wj;
        acc[0][0] = mfma16x16x4(a0, lb.x, acc[0][0]);
        acc[0][1] = mfma16x16x4(a0, lb.y, acc[0][1]);
        acc[1][0] = mfma16x16x4(a1, lb.x, acc[1][0]);
        acc[1][1] = mfma16x16x4(a1, lb.y, acc[1][1]);
        wj = wn; la = lan; lb = lbn;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int ea = 0; ea < 2; ++ea)
#pragma unroll
            for (int eb = 0; eb < 2; ++eb) red[wave][2 * (q + 4 * g) + ea][2 * r + eb] = acc[ea][eb][g];
    __syncthreads();
    double *out = A + (size_t)m * KW * KW + (size_t)(32 * ta) * KW + 32 * tb;
    for (int e = threadIdx.x; e < 32 * 32; e += 64 * GRAM_WAVES) {
        const int a = e >> 5, b = e & 31;
        double v[GRAM_WAVES];
#pragma unroll
        for (int u = 0; u < GRAM_WAVES; ++u) v[u] = red[u][a][b];
#pragma unroll
        for (int h = 1; h < GRAM_WAVES; h <<= 1)   // pairwise: ((v0 + v1) + (v2 + v3)) + ...
#pragma unroll
            for (int u = 0; u < GRAM_WAVES; u += 2 * h) v[u] += v[u + h];
        out[(size_t)a * KW + b] = v[0];
    }
}

// ============================================================================
// k_prep: Z-draw operators of shard m (one block per local shard).        dc:100-107
//   R = cholcov(Zprec), Zprec = I + (1-rho) A_m; cholcov reads the upper triangle,
//   so the lower factor L = R' is the Cholesky of S[r][c] = Zprec[c][r] (c <= r).
//   U = L^{-1}, T = U U';  ZM[m] = {M1 = s1r T, -, U, -}: the reference's
//   R'\(R\bz) + R'\z is T bz + U z (quirk Q2), with bz = s1r (W - sr A X) formed in
//   k_zdraw from A directly.  Tiled LDS Cholesky / inverse / U U' (tile_linalg.h).
// ============================================================================
#ifndef DCFM_TILE_THREADS
#define DCFM_TILE_THREADS 1024
#endif
constexpr int TILE_THREADS = DCFM_TILE_THREADS;   // k_prep / k_xchol: 16 waves share the tile steps (c4: 4 waves
                                                  // 99 / 77 us, 16 with the look-ahead 40 / 48 us)
static_assert(TILE_THREADS >= 128 && TILE_THREADS % 64 == 0, "potrf_inv's look-ahead needs at least two whole waves");
template <int KW>
__global__ __launch_bounds__(TILE_THREADS) void k_prep(Dims d, const double *__restrict__ A, double *__restrict__ ZM) {
    constexpr int NB = KW / tile::TS, NT = tile::ntiles(NB);
    __shared__ double Ts[NT * tile::TSZ], Us[NT * tile::TSZ], lds_l[32], lds_u[16];
    const int m = blockIdx.x, N = d.K, nb = (N + tile::TS - 1) / tile::TS, t = threadIdx.x;
    const double *Am = A + (size_t)m * KW * KW;
    for (int e = t; e < tile::ntiles(nb) * tile::TS * tile::TS; e += TILE_THREADS) {
        int I, J;
        tile::tri_pair(e >> 8, I, J);
        const int r = (e >> 4) & 15, c = e & 15, R = 16 * I + r, Cc = 16 * J + c;
        const double v = (R < N && Cc < N) ? (R == Cc ? 1.0 : 0.0) + (1.0 - d.rho) * Am[(size_t)Cc * KW + R]
                                           : (R == Cc ? 1.0 : 0.0);
        Ts[tile::tix(I, J) * tile::TSZ + c * tile::TLD + r] = v;
    }
    __syncthreads();
    tile::potrf_inv(Ts, Us, nb, lds_l, lds_u);
    tile::trtri(Ts, Us, nb);
    double *Zm = ZM + (size_t)m * 4 * KW * KW;
    tile::uut_store(Us, nb, N, d.s1r, Zm, KW, Zm + (size_t)2 * KW * KW);
}

// ============================================================================
// k_xchol: Xprec = g I + rho sum_m A_m (dc:117, summed over ranks in the canonical tree),
// Rx = cholcov(Xprec) (dc:118); XM = {Tx = sqrt(rho) Ux Ux', Ux = Rx^{-T}}.
// ============================================================================
template <int KW>
__global__ __launch_bounds__(TILE_THREADS) void k_xchol(Dims d, const double *__restrict__ xa_all, double *__restrict__ XM) {
    constexpr int NB = KW / tile::TS, NT = tile::ntiles(NB);
    __shared__ double Ts[NT * tile::TSZ], Us[NT * tile::TSZ], lds_l[32], lds_u[16];
    const int N = d.K, nb = (N + tile::TS - 1) / tile::TS, t = threadIdx.x;
    for (int e = t; e < tile::ntiles(nb) * tile::TS * tile::TS; e += TILE_THREADS) {
        int I, J;
        tile::tri_pair(e >> 8, I, J);
        const int r = (e >> 4) & 15, c = e & 15, R = 16 * I + r, Cc = 16 * J + c;
        double v = (R == Cc) ? 1.0 : 0.0;
        if (R < N && Cc < N) {
            const size_t o = (size_t)Cc * KW + R;   // upper triangle: Xprec[c][r]
            const double sa = tree_sum(xa_all + o, d.nranks, (size_t)KW * KW);   // ranks' sums, canonical tree
            v = (R == Cc ? (double)d.g : 0.0) + d.rho * sa;
        }
        Ts[tile::tix(I, J) * tile::TSZ + c * tile::TLD + r] = v;
    }
    __syncthreads();
    tile::potrf_inv(Ts, Us, nb, lds_l, lds_u);
    tile::trtri(Ts, Us, nb);
    tile::uut_store(Us, nb, N, d.sr, XM, KW, XM + (size_t)KW * KW);
}

// standard normals eps[i][kk], eps[i][kk+1] of a Z / X row (kk even)       dc:104,126
__device__ __forceinline__ d2 row_normals(const Dims &d, const double *inj, bool live, int site, int mg, int i,
                                          int kk, int64_t iter) {
    d2 ev = {0.0, 0.0};
    if (!live || kk >= d.K) return ev;
    ev.x = inj[kk];
    ev.y = (kk + 1 < d.K) ? inj[kk + 1] : 0.0;
    return ev;
}

// ============================================================================
// k_zdraw: per (shard m, 16 ZD_RT rows i), the KW/16 output tiles of each product dealt
// over the block's 4 waves (KW/64 tiles each, for ZD_RT 16-row tiles).     dc:101-107,121-123
//   V' = W' - sr A X'        (= bz / s1r: Zmsg'(Y_i - sr L X_i) by the identity W = Y (w o L))
//   Z' = M1 V' + U eps'      (M1 = s1r T, U from k_prep)
//   S' = W' - s1r A Z'       (the shard's X message, dc:121-123)
// The f64 C/D layout of a product (row = q + 4g of tile mt) is the B operand of the next
// one (k-step 4 mt + g); V' and Z' pass between the waves through LDS (16 rows x KW),
// the A operands (A_m, M1, U) stream from L2, each load serving the block's ZD_RT row tiles
// (one wave per 16 rows with every tile left the MFMA pipe idle 80 % of the time at c4).
// ============================================================================
#ifndef DCFM_ZD_RT
#define DCFM_ZD_RT 4
#endif
constexpr int ZD_RT = DCFM_ZD_RT;   // 16-row tiles per block: the A operands (A_m, M1, U) serve 4 (c4: 138 -> 81 us vs 1)
// TK = ceil(K / 8) (a template argument, so the k loops keep their unrolling): the k-steps past K add exact
// zeros (A_m, M1, U zero across the live / padding boundary; X, V, eps, Z zero in the padding) and are not
// issued -- c4: 13 of 16 eight-wide and 26 of 32 four-wide steps; the same values
template <int KW, int TK = KW / 8>
__global__ __launch_bounds__(256) void k_zdraw(Dims d, const double *__restrict__ W, const double *__restrict__ A,
                                               const double *__restrict__ ZM, const double *__restrict__ X,
                                               double *__restrict__ Z, double *__restrict__ Sp, DrawsDev dr,
                                               int64_t iter) {
    constexpr int MW = KW / 64, RT = ZD_RT;         // output tiles per wave, row tiles per block
    __shared__ double Vs[RT][KW][16], Zs[RT][KW][16];
    const int nrb = d.NP / (16 * RT);
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int m = w / nrb, rb = w % nrb;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = lane & 15, q = lane >> 4;
    const int mg = d.shard0 + m;
    const int mt0 = wave * MW;
    const double *Am = A + (size_t)m * KW * KW;
    const double *M1 = ZM + (size_t)m * 4 * KW * KW, *U = M1 + 2 * KW * KW;
    int iv[RT];
    bool live[RT];
    const double *Wi[RT], *Xi[RT];
#pragma unroll
    for (int h = 0; h < RT; ++h) {
        iv[h] = (rb * RT + h) * 16 + c;
        live[h] = iv[h] < d.n;
        Wi[h] = W + ((size_t)m * d.NP + iv[h]) * KW;
        Xi[h] = X + (size_t)iv[h] * KW;
    }
    // --- A X' for this wave's tiles
    d4 av[RT][MW];
#pragma unroll
    for (int h = 0; h < RT; ++h)
#pragma unroll
        for (int u = 0; u < MW; ++u) av[h][u] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 2
    for (int t = 0; t < TK; ++t) {
        const int kk = 8 * t + 2 * q;
        d2 xv[RT];
#pragma unroll
        for (int h = 0; h < RT; ++h) xv[h] = *reinterpret_cast<const d2 *>(Xi[h] + kk);
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const d2 a2 = *reinterpret_cast<const d2 *>(Am + (size_t)(16 * (mt0 + u) + c) * KW + kk);
#pragma unroll
            for (int h = 0; h < RT; ++h) {
                av[h][u] = mfma16x16x4(a2.x, xv[h].x, av[h][u]);
                av[h][u] = mfma16x16x4(a2.y, xv[h].y, av[h][u]);
            }
        }
    }
    // --- V' = W' - sr (A X') -> LDS
#pragma unroll
    for (int h = 0; h < RT; ++h)
#pragma unroll
        for (int u = 0; u < MW; ++u)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int k = 16 * (mt0 + u) + q + 4 * g;
                Vs[h][k][c] = Wi[h][k] - d.sr * av[h][u][g];
            }
    __syncthreads();
    // --- Z' = M1 V' + U eps'      eps[i][kk] of dc:104, kk = 4 t + q
    d4 az[RT][MW];
#pragma unroll
    for (int h = 0; h < RT; ++h)
#pragma unroll
        for (int u = 0; u < MW; ++u) az[h][u] = d4{0.0, 0.0, 0.0, 0.0};
    const size_t nzb = ((size_t)(iter - dr.first_iter) * d.g + mg) * d.n;
#pragma unroll 2
    for (int t = 0; t < 2 * TK; ++t) {
        const int kk = 4 * t + q;
        double vb[RT], e[RT];
#pragma unroll
        for (int h = 0; h < RT; ++h) {
            vb[h] = Vs[h][kk][c];
            e[h] = (live[h] && kk < d.K) ? dr.NZ[(nzb + iv[h]) * d.K + kk] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const size_t o = (size_t)(16 * (mt0 + u) + c) * KW + kk;
            const double m1 = M1[o], uu = U[o];
#pragma unroll
            for (int h = 0; h < RT; ++h) {
                az[h][u] = mfma16x16x4(m1, vb[h], az[h][u]);
                az[h][u] = mfma16x16x4(uu, e[h], az[h][u]);
            }
        }
    }
#pragma unroll
    for (int h = 0; h < RT; ++h)
#pragma unroll
        for (int u = 0; u < MW; ++u)
#pragma unroll
            for (int g = 0; g < 4; ++g) Zs[h][16 * (mt0 + u) + q + 4 * g][c] = az[h][u][g];
    __syncthreads();
    // --- S' = W' - s1r (A Z')
    d4 as[RT][MW];
#pragma unroll
    for (int h = 0; h < RT; ++h)
#pragma unroll
        for (int u = 0; u < MW; ++u) as[h][u] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 2
    for (int t = 0; t < 2 * TK; ++t) {
        const int kk = 4 * t + q;
        double zb[RT];
#pragma unroll
        for (int h = 0; h < RT; ++h) zb[h] = Zs[h][kk][c];
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const double a1 = Am[(size_t)(16 * (mt0 + u) + c) * KW + kk];
#pragma unroll
            for (int h = 0; h < RT; ++h) as[h][u] = mfma16x16x4(a1, zb[h], as[h][u]);
        }
    }
#pragma unroll
    for (int h = 0; h < RT; ++h) {
        double *Zr = Z + ((size_t)m * d.NP + iv[h]) * KW;
        double *Sr = Sp + ((size_t)m * d.NP + iv[h]) * KW;
#pragma unroll
        for (int u = 0; u < MW; ++u)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int k = 16 * (mt0 + u) + q + 4 * g;
                if (live[h]) Zr[k] = (k < d.K) ? az[h][u][g] : 0.0;
                Sr[k] = live[h] ? Wi[h][k] - d.s1r * as[h][u][g] : 0.0;
            }
    }
}

// ============================================================================
// k_xdraw: X' = Tx S' + Ux eps' (S summed over ranks, canonical tree), one block of XD_WAVES waves per
// 16 rows, the KW/16 output tiles dealt over the waves.  One wave per 16 rows issued all 8 tiles' 512
// MFMAs on one SIMD behind 16 rounds of dependent L2 loads (c4: 125 waves on 1,024 SIMDs, 39 us);
// every tile keeps its products and their order, so X keeps its bits.               dc:119-128
// ============================================================================
#ifndef DCFM_XD_WAVES
#define DCFM_XD_WAVES 4
#endif
template <int KW> constexpr int xd_waves() { return KW / 16 < DCFM_XD_WAVES ? KW / 16 : DCFM_XD_WAVES; }
template <int KW, int TK = KW / 8>   // TK = ceil(K / 8): as k_zdraw
__global__ __launch_bounds__(64 * xd_waves<KW>()) void k_xdraw(Dims d, const double *__restrict__ xall, const double *__restrict__ XM,
                                                         double *__restrict__ X, DrawsDev dr, int64_t iter) {
    constexpr int MT = KW / 16, MPW = MT / xd_waves<KW>();   // output tiles per wave
    static_assert(MT % xd_waves<KW>() == 0, "whole tiles per wave");
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = lane & 15, q = lane >> 4;
    const int i = blockIdx.x * 16 + c;
    const bool live = i < d.n;
    const size_t stride = (size_t)d.NP * KW;
    const double *Tx = XM, *Ux = XM + KW * KW;
    const double *nx = dr.NX + ((size_t)(iter - dr.first_iter) * d.n + (live ? i : 0)) * d.K;
    d4 ax[MPW];
#pragma unroll
    for (int u = 0; u < MPW; ++u) ax[u] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int t = 0; t < TK; ++t) {
        const int kk = 8 * t + 2 * q;
        TreeSum<d2> ts;                                  // the ranks' message sums, canonical tree
        for (int rk = 0; rk < d.nranks; ++rk) ts.push(*reinterpret_cast<const d2 *>(xall + rk * stride + (size_t)i * KW + kk));
        const d2 sv = ts.total();
        const d2 ev = row_normals(d, nx, live, SITE_X, 0, i, kk, iter);
#pragma unroll
        for (int u = 0; u < MPW; ++u) {
            const int mt = wave * MPW + u;
            const size_t o = (size_t)(16 * mt + c) * KW + kk;
            const d2 a1 = *reinterpret_cast<const d2 *>(Tx + o);
            const d2 a2 = *reinterpret_cast<const d2 *>(Ux + o);
            ax[u] = mfma16x16x4(a1.x, sv.x, ax[u]);
            ax[u] = mfma16x16x4(a2.x, ev.x, ax[u]);
            ax[u] = mfma16x16x4(a1.y, sv.y, ax[u]);
            ax[u] = mfma16x16x4(a2.y, ev.y, ax[u]);
        }
    }
    if (!live) return;
    double *Xr = X + (size_t)i * KW;
#pragma unroll
    for (int u = 0; u < MPW; ++u)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int k = 16 * (wave * MPW + u) + q + 4 * g;
            Xr[k] = (k < d.K) ? ax[u][g] : 0.0;
        }
}

// ============================================================================
// k_lambda_w: one wave per loading row j (K = 33..128).        dc:140-145 (+150,156,169-171)
// Q_j = R'R (R = Llam', dc:142) on the NB x NB upper tiles T_{Kc,I} (Kc <= I) of Q_j, all held
// in this wave's registers in the fp64 MFMA C/D layout (lane (c16, q) holds T[q + 4g][c16],
// g = 0..3).  That layout is the B operand of a product with k = q + 4g and the A operand of
// its transpose, so per block column J, with U_JJ = L_JJ^{-1} from chol_inv16_blk (staged in LDS):
//   panel     R_{J,I}  = U_JJ T_{J,I}                (A = U_JJ from LDS, B = registers)
//   trailing  T_{Kc,I} -= R_{J,Kc}' R_{J,I}           (both operands in registers)
//   forward   b_I -= R_{J,I}' v_J,  v_J = U_JJ b_J    (dc:143, sums over q by lane shuffles)
// and the back solve R x = v + z (dc:142-144) sums each block row's products in registers
// before one reduction over the 16 lanes of a tile row.  No workgroup barriers: the row's
// whole chain is one wave, and the CU's other waves (other rows) fill its latency.  The
// epilogue forms psi (dc:150), cpart (dc:156) and SS_j = yy_j - 2 x.C_j + x'E x (dc:169 by
// identity: x'E x = (|w|^2 - sum_r Plam_jr x_r^2) / ps_j since x'Q_j x = |w|^2), ps, omega.
// ============================================================================
template <int NB>
__host__ __device__ constexpr int utix(int Kc, int I) { return Kc * NB - Kc * (Kc - 1) / 2 + (I - Kc); }

// T_{Kc,I} -= R_{J,Kc}' R_{J,I}  (block column J's trailing update of one upper tile)
template <int NB, int J, int Kc, int I>
__device__ __forceinline__ void trail_tile(d4 *T) {
    constexpr int a = utix<NB>(J, Kc), b = utix<NB>(J, I), t = utix<NB>(Kc, I);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) T[t] = mfma16x16x4_na(T[a][s4], T[b][s4], T[t]);
}

// The trailing tiles of block column J but the next diagonal one, (Kc, I) with J < Kc <= I < NB in
// row-major order, numbered from 0: pivot step S of the next diagonal block issues tiles
// [S n / 16, (S + 1) n / 16) of the n = NT_J of them.
template <int NB, int J>
__host__ __device__ constexpr int la_count() { return (NB - J - 1) * (NB - J) / 2 - 1; }
template <int NB, int J>
__host__ __device__ constexpr int la_index(int Kc, int I) {
    int e = 0;
    for (int a = J + 1; a < NB; ++a)
        for (int b = a; b < NB; ++b) {
            if (a == J + 1 && b == J + 1) continue;
            if (a == Kc && b == I) return e;
            ++e;
        }
    return -1;
}
template <int NB, int J, int S, int NS = 16>
__device__ __forceinline__ void la_step(d4 *T) {
    constexpr int n = la_count<NB, J>(), lo = S * n / NS, hi = (S + 1) * n / NS;
    static_for<NB>([&](auto KC) {
        constexpr int Kc = decltype(KC)::value;
        static_for<NB>([&](auto IC) {
            constexpr int I = decltype(IC)::value;
            if constexpr (Kc > J && I >= Kc && !(Kc == J + 1 && I == J + 1)) {
                constexpr int e = la_index<NB, J>(Kc, I);
                if constexpr (e >= lo && e < hi) trail_tile<NB, J, Kc, I>(T);
            }
        });
    });
}

template <int KW, int NB>
__global__ __launch_bounds__(64) void k_lambda_w(
    Dims d, const double *__restrict__ C, const double *__restrict__ E, const double *__restrict__ yy,
    const double *__restrict__ tau_cur, const double *__restrict__ plam_src, double *__restrict__ Lam,
    double *__restrict__ psi, double *__restrict__ ps, double *__restrict__ omega, double *__restrict__ cpart,
    DrawsDev dr, int64_t iter, double kappa_max, int *__restrict__ rflag) {
    constexpr int NT = NB * (NB + 1) / 2, LD = 17, TZ = 16 * LD, NH = KW / 64;
    __shared__ double Ud[TZ];
    __shared__ double vb[KW], vx[KW], ein[5][KW];   // per row index r: NL, Gpsi, tau, C, Plam
    __shared__ double edg[KW], udg[KW];             // the guard: E_m[r][r], 1 / L_rr (L = chol(Q_j))
    const int j = blockIdx.x, m = blockIdx.y, mg = d.shard0 + m;
    const int lane = threadIdx.x, c16 = lane & 15, q = lane >> 4;
    const int K = d.K;
    const double *Em = E + (size_t)m * KW * KW;
    const size_t rowoff = ((size_t)m * d.PP + j) * KW;
    const double psj = ps[(size_t)m * d.PP + j];
    // ---- every load issued before the first wait (indices clamped, values selected after)
    const size_t drow = ((size_t)(iter - dr.first_iter) * d.g + mg) * d.P + j;
    double zr[NH], Gr[NH], trr[NH], cr[NH], pr[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int r = lane + 64 * h, re = r < K ? r : 0;
        zr[h] = dr.NL[drow * K + re];                                       // dc:142
        Gr[h] = dr.Gpsi[drow * K + re];                                     // dc:150
        trr[h] = tau_cur[(size_t)mg * KW + re];
        cr[h] = C[rowoff + re];
        pr[h] = (plam_src ? plam_src : psi)[rowoff + re];
    }
    const double yyj = yy[(size_t)m * d.PP + j], Gps = dr.Gps[drow];   // dc:169-170
    d4 T[NT];   // E_m's upper tiles, stored by k_cpass in this layout (etile_index): 16-byte reads
    static_for<NB>([&](auto KC) {
        constexpr int Kc = decltype(KC)::value;
        static_for<NB>([&](auto IC) {
            constexpr int I = decltype(IC)::value;
            if constexpr (I >= Kc) {
                constexpr int tw = etile(KW / 16, Kc, I);
                const d2 e0 = *reinterpret_cast<const d2 *>(Em + (2 * tw) * 128 + 2 * lane);
                const d2 e1 = *reinterpret_cast<const d2 *>(Em + (2 * tw + 1) * 128 + 2 * lane);
                T[utix<NB>(Kc, I)] = d4{e0.x, e0.y, e1.x, e1.y};
            }
        });
    });
    static_for<NB>([&](auto JC) {                       // diag(E_m): lane (c16, q) holds T[q + 4g][c16]
        constexpr int J = decltype(JC)::value;
#pragma unroll
        for (int g = 0; g < 4; ++g)
            if (q + 4 * g == c16) edg[16 * J + c16] = T[utix<NB>(J, J)][g];
    });
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int r = lane + 64 * h;
        const bool tl = r < K;
        ein[0][r] = tl ? zr[h] : 0.0;
        ein[1][r] = tl ? Gr[h] : 0.0;
        ein[2][r] = tl ? trr[h] : 0.0;
        ein[3][r] = tl ? cr[h] : 0.0;
        // Plam_j (dc:176); 1 in the padding: E_m is exactly zero there (X, Z padding zero), so
        // ps_j E_m + diag(Plam_j) is the identity padding with no selects on K
        ein[4][r] = tl ? (plam_src ? pr[h] : pr[h] * trr[h]) : 1.0;
        vb[r] = tl ? psj * cr[h] : 0.0;                                  // blam (dc:141)
    }
    __syncthreads();
    // ---- Q_j tiles: ps_j eta2 + diag(Plam_j) (dc:141); the padding is the identity by construction
    //      (ein[4] above).  Plam_j only meets the diagonal tiles (a compile-time fact: an LDS read per
    //      element of every tile made this a chain of 112 dependent LDS round trips)
    double pl[NB][4];
    static_for<NB>([&](auto JC) {
        constexpr int J = decltype(JC)::value;
#pragma unroll
        for (int g = 0; g < 4; ++g) pl[J][g] = ein[4][16 * J + q + 4 * g];
    });
    static_for<NB>([&](auto KC) {
        constexpr int Kc = decltype(KC)::value;
        static_for<NB>([&](auto IC) {
            constexpr int I = decltype(IC)::value;
            if constexpr (I >= Kc) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    double val = psj * T[utix<NB>(Kc, I)][g];
                    if constexpr (I == Kc) val = (q + 4 * g == c16) ? val + pl[Kc][g] : val;
                    T[utix<NB>(Kc, I)][g] = val;
                }
            }
        });
    });
    // ---- blocked factorisation with the forward solve.  Look-ahead: block column J's trailing update
    //      of the next diagonal tile goes first, then that block's factor U = L^{-1} from its registers
    //      (chol_inv16_blk: 4 x 4 block steps, no LDS) with the rest of J's trailing MFMAs issued into
    //      its four steps (la_step).  Round 6 replaced the pivot-by-pivot LDS factor (chol_inv16_hook,
    //      16 round trips per block): k_lambda_w 369 -> 337 us at c4
    {
        const d4 U0 = chol_inv16_blk(T[utix<NB>(0, 0)], lane, [](auto) {});
#pragma unroll
        for (int g = 0; g < 4; ++g) Ud[(q + 4 * g) * LD + c16] = U0[g];
    }
    __syncthreads();
    static_for<NB>([&](auto JC) {
        constexpr int J = decltype(JC)::value, tJ = utix<NB>(J, J);
        if (q == 0) udg[16 * J + c16] = Ud[c16 * LD + c16];                    // 1 / L_kk (the guard)
        double u[4], bq[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            u[s4] = Ud[c16 * LD + 4 * s4 + q];                                 // A operand of U_JJ
            bq[s4] = vb[16 * J + 4 * s4 + q];                                  // b_J, same in every column
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) T[tJ][g] = Ud[(q + 4 * g) * LD + c16];      // U_JJ kept (back solve)
        // v_J = U_JJ b_J (dc:143) as a product whose 16 columns all hold it: lane (c16, q) gets
        // v[q + 4g] in element g, the layout the panel's forward-solve update reads (two chains)
        d4 va = {0.0, 0.0, 0.0, 0.0}, vc = {0.0, 0.0, 0.0, 0.0};
        va = mfma16x16x4(u[0], bq[0], va);
        vc = mfma16x16x4(u[1], bq[1], vc);
        va = mfma16x16x4(u[2], bq[2], va);
        vc = mfma16x16x4(u[3], bq[3], vc);
        double vj[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) vj[g] = va[g] + vc[g];
        __syncthreads();                                                       // b_J read by every lane
        if (c16 == 0) {
#pragma unroll
            for (int g = 0; g < 4; ++g) vb[16 * J + q + 4 * g] = vj[g];        // v_J for the back solve
        }
        static_for<NB>([&](auto IC) {                     // panel R_{J,I} = U_JJ T_{J,I}
            constexpr int I = decltype(IC)::value;
            if constexpr (I > J) {
                constexpr int t = utix<NB>(J, I);
                d4 R = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) R = mfma16x16x4(u[s4], T[t][s4], R);
                T[t] = R;
                double pv = 0.0;                          // (R_{J,I}' v_J)[c16]: sum over rows q + 4g
#pragma unroll
                for (int g = 0; g < 4; ++g) pv = fma(R[g], vj[g], pv);
                pv += xor16_d(pv);
                pv += xor32_d(pv);
                if (q == 0) vb[16 * I + c16] -= pv;
            }
        });
        if constexpr (J + 1 < NB) {   // trailing T_{Kc,I} -= R_{J,Kc}' R_{J,I}: the next diagonal tile first
            trail_tile<NB, J, J + 1, J + 1>(T);
            // the next diagonal block's factor from its registers (chol_inv16_blk), the rest of J's
            // trailing MFMAs issued into its four block steps
            const d4 Un = chol_inv16_blk(T[utix<NB>(J + 1, J + 1)], lane, [&](auto S) {
                la_step<NB, J, decltype(S)::value, 4>(T);
            });
            __syncthreads();                                                   // U_JJ's reads are done
#pragma unroll
            for (int g = 0; g < 4; ++g) Ud[(q + 4 * g) * LD + c16] = Un[g];
            __syncthreads();
        }
    });
    // ---- w = v + z (dc:142 normrnd), back solve R x = w (dc:144):
    //      x_J = U_JJ' (w_J - sum_{I>J} R_{J,I} x_I); lane (c16, .) holds x_I[c16] in xr[I]
    __syncthreads();
#pragma unroll
    for (int h = 0; h < NH; ++h) vb[lane + 64 * h] += ein[0][lane + 64 * h];
    __syncthreads();
    double xr[NB];
    static_for<NB>([&](auto JJ) {
        constexpr int J = NB - 1 - decltype(JJ)::value;
        double pg[4] = {0.0, 0.0, 0.0, 0.0};
        static_for<NB>([&](auto IC) {
            constexpr int I = decltype(IC)::value;
            if constexpr (I > J) {
#pragma unroll
                for (int g = 0; g < 4; ++g) pg[g] = fma(T[utix<NB>(J, I)][g], xr[I], pg[g]);
            }
        });
        double sx = 0.0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            double y = vb[16 * J + q + 4 * g];
            if constexpr (J < NB - 1) y -= rowsum16(pg[g]);
            sx = fma(T[utix<NB>(J, J)][g], y, sx);        // (U_JJ' y)[c16]: sum over rows q + 4g
        }
        sx += xor16_d(sx);
        sx += xor32_d(sx);
        xr[J] = sx;
    });
#pragma unroll
    for (int I = 0; I < NB; ++I)
        if (q == 0) vx[16 * I + c16] = xr[I];
#pragma unroll
    for (int h = 0; h < NH; ++h)
        if (lane + 64 * h >= 16 * NB) vx[lane + 64 * h] = 0.0;
    __syncthreads();
    // ---- epilogue: Lambda_j, psi_j (dc:150), cpart (dc:156), SS_j (dc:169), ps_j, omega_j
    //      + the guard of the SS identity (as k_lambda's, lambda.h): kappa_j = max(yy_j + (1 + c_j) |w|^2 / ps_j
    //      + sum_r Plam_jr x_r^2 / ps_j + 2 sum_r |x_r C_jr|,  (sqrt(yy_j) + sum_r |x_r| sqrt(E_rr))^2) / SS_j,
    //      c_j = max_r Q_rr / L_rr^2; a row beyond kappa_max (or SS_j <= 0) flags its 32-row tile, whose
    //      ps, omega k_resid_flagged then takes from dc:169's residual
    double ssr = 0.0, mag = 0.0, ww = 0.0, sab = 0.0, cs = 1.0;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int r = lane + 64 * h;
        const double xv = (r < K) ? vx[r] : 0.0;
        double psir = 0.0;
        if (r < K) {
            const double scale = 1.0 / (d.df * 0.5 + 0.5 * (xv * xv * ein[2][r]));
            psir = scale * ein[1][r];
            psi[rowoff + r] = psir;
            const double w = vb[r], px = ein[4][r] * xv * xv, xc = xv * ein[3][r];
            ssr += fma(w, w, -px) / psj - 2.0 * xc;
            ww = fma(w, w, ww);
            mag += px / psj + 2.0 * fabs(xc);
            const double e = edg[r], ik = udg[r];
            sab = e > 0.0 ? fma(fabs(xv), e * __builtin_amdgcn_rsq(e), sab) : sab;
            cs = fmax(cs, fma(psj, e, ein[4][r]) * ik * ik);
        }
        Lam[rowoff + r] = xv;
        cpart[rowoff + r] = psir * (xv * xv);          // mat = psijh .* Lambda.^2 (dc:156)
    }
    // wave sums: DPP within the 16-lane rows, then the four row totals by readlane in a fixed order
    // (a butterfly of lane shuffles here cost ~9 us per c4 launch: six LDS-latency rounds per row)
    auto wsum = [](double v) {
        v = rowsum16(v);
        return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
    };
    ssr = wsum(ssr);
    mag = wsum(mag);
    ww = wsum(ww);
    sab = wsum(sab);
    cs = fmax(cs, dpp_d<0xB1>(cs));
    cs = fmax(cs, dpp_d<0x4E>(cs));
    cs = fmax(cs, dpp_d<0x124>(cs));
    cs = fmax(cs, dpp_d<0x128>(cs));
    cs = fmax(fmax(readlane_d(cs, 0), readlane_d(cs, 16)), fmax(readlane_d(cs, 32), readlane_d(cs, 48)));
    if (lane == 0) {
        const double SS = yyj + ssr;
        const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps;      // dc:170
        ps[(size_t)m * d.PP + j] = psn;
        omega[(size_t)m * d.PP + j] = 1.0 / psn;                 // dc:171 (Q1)
        if (rflag) {
            const double rt = 1.01 * (yyj * __builtin_amdgcn_rsq(yyj) + sab);
            const double num = fmax(rt * rt, 1.01 * (yyj + mag + (1.0 + cs) * ww / psj));
            if (!(SS > 0.0 && num <= kappa_max * SS)) rflag[m * (d.PP / 32) + j / 32] = 1;
        }
    }
}

// ============================================================================
// block = (shard m, 32 columns); 8 row groups x 4 independent accumulators each.
template <int KW>
__global__ __launch_bounds__(256) void k_colsum(Dims d, const double *__restrict__ cpart, double *__restrict__ sloc) {
    __shared__ double part[8][32];
    const int m = blockIdx.x, k = 32 * blockIdx.y + (threadIdx.x & 31), grp = threadIdx.x >> 5;
    const double *cp = cpart + (size_t)m * d.PP * KW + k;
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    int j = grp;
    for (; j + 24 < d.P; j += 32) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s4[u] += cp[(size_t)(j + 8 * u) * KW];
    }
    for (; j < d.P; j += 8) s4[0] += cp[(size_t)j * KW];
    part[grp][threadIdx.x & 31] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    __syncthreads();
    if (threadIdx.x < 32) {
        double tt = 0.0;
#pragma unroll
        for (int g2 = 0; g2 < 8; ++g2) tt += part[g2][threadIdx.x];
        sloc[(size_t)m * KW + k] = tt;
    }
}

// ============================================================================
// k_delta: multiplicative-gamma-process chain for K in 33..128 (NV = KW/64
// factors per lane: index l + 64 s).  Same algebra as the narrow kernel: every
// shard's h >= 2 step reads shard 1's already-updated delta_h (quirk Q4), the
// recomputed cumprod is the scalar factor F_h (dc:155-165).  (K == 1, quirk Q5,
// is narrow-only.)
// ============================================================================
template <int NV>
__device__ __forceinline__ void suffix_sum_nv(double (&v)[NV], int l) {
    v[NV - 1] = wave_suffix_sum(v[NV - 1], l);
    if (NV == 2) v[0] = wave_suffix_sum(v[0], l) + readlane_d(v[NV - 1], 0);
}
template <int NV>
__device__ __forceinline__ void scan_prod_nv(double (&v)[NV], int l) {
    v[0] = wave_scan_prod(v[0], l);
    if (NV == 2) v[NV - 1] = wave_scan_prod(v[NV - 1], l) * readlane_d(v[0], 63);
}
// The chain over h as the narrow kernel runs it (kernels.hip delta_chain): with y_h = 1 / F_h the
// recurrence is affine, y_{h+1} = alpha_h y_h + beta_h, alpha_h = b_h dold_h / G_h, beta_h = c_h dold_h /
// G_h, c_h = (0.5 / dref_h) T_h, and dn_h = G_h y_h / (b_h y_h + c_h); the maps compose by a wave scan
// (log2 steps) instead of K dependent steps of lane reads (measured 48.7 us per iteration at c4, a
// serial chain on the critical path).  NV = 2: index l + 64 of the second slice composes with the
// first slice's total map (lane 63).  Every term is positive: the reassociation moves the result
// by a few ulps only (dc:157-163).
__device__ __forceinline__ void affine_scan(double &A, double &B, int l) {   // inclusive, lane 0 first
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double Ap = __shfl_up(A, o, 64), Bp = __shfl_up(B, o, 64);
        if (l >= o) {
            B = fma(A, Bp, B);
            A = A * Ap;
        }
    }
}
template <int NV>
__device__ __forceinline__ void delta_chain_nv(const Dims &d, int l, const double (&T)[NV], const double (&G)[NV],
                               const double (&idold)[NV], const double (&idref)[NV], double (&dnew)[NV]) {
    double bh[NV], c[NV], A[NV], B[NV];
    bool act[NV];
#pragma unroll
    for (int s = 0; s < NV; ++s) {
        const int idx = l + 64 * s;
        act[s] = idx < d.K;
        bh[s] = (idx == 0) ? d.bd1 : d.bd2;
        c[s] = (0.5 * idref[s]) * T[s];
        const double inv = 1.0 / (idold[s] * G[s]);              // dold_h / G_h
        A[s] = act[s] ? bh[s] * inv : 1.0;                        // identity map on idle indices
        B[s] = act[s] ? c[s] * inv : 0.0;
        affine_scan(A[s], B[s], l);
    }
    if (NV == 2) {   // the second slice after the whole first one
        const double A0 = readlane_d(A[0], 63), B0 = readlane_d(B[0], 63);
        B[NV - 1] = fma(A[NV - 1], B0, B[NV - 1]);
        A[NV - 1] = A[NV - 1] * A0;
    }
    double yin[NV];
#pragma unroll
    for (int s = 0; s < NV; ++s) yin[s] = A[s] + B[s];            // y_{idx+1} (y_0 = 1)
#pragma unroll
    for (int s = 0; s < NV; ++s) {
        const double yprev = __shfl_up(yin[s], 1, 64);
        const double y = (l == 0) ? (s == 0 ? 1.0 : readlane_d(yin[0], 63)) : yprev;   // y_idx
        dnew[s] = act[s] ? G[s] * y / fma(bh[s], y, c[s]) : 1.0;
    }
}

// one wave = global shard m, lane t (< 64 active)
template <int KW>
__device__ __forceinline__ void delta_shard_w(const Dims &d, const double *__restrict__ sall,
                                              const double *__restrict__ delta_in, const double *__restrict__ tau_in,
                                              double *__restrict__ delta_out, double *__restrict__ tau_out,
                                              const DrawsDev &dr, int64_t iter, int m, int t) {
    constexpr int NV = KW / 64;
    if (t < 64) {
        const int l = t;
        double d0[NV], T0[NV], G0[NV], id0[NV], d0new[NV];
#pragma unroll
        for (int s = 0; s < NV; ++s) {
            const int idx = l + 64 * s;
            const bool act = idx < d.K;
            d0[s] = act ? delta_in[idx] : 1.0;
            T0[s] = act ? tau_in[idx] * sall[idx] : 0.0;
            G0[s] = act ? delta_G(d, dr, iter, 0, idx) : 1.0;
            id0[s] = 1.0 / d0[s];
        }
        suffix_sum_nv<NV>(T0, l);
        delta_chain_nv<NV>(d, l, T0, G0, id0, id0, d0new);   // shard 1, its own pre-update delta_h
        double dm[NV];
#pragma unroll
        for (int s = 0; s < NV; ++s) dm[s] = d0new[s];
        if (m != 0) {
            double Tm[NV], Gm[NV], idold[NV], idref[NV];
#pragma unroll
            for (int s = 0; s < NV; ++s) {
                const int idx = l + 64 * s;
                const bool act = idx < d.K;
                const size_t o = (size_t)m * KW + idx;
                const double dold = act ? delta_in[o] : 1.0;
                Tm[s] = act ? tau_in[o] * sall[o] : 0.0;
                Gm[s] = act ? delta_G(d, dr, iter, m, idx) : 1.0;
                idold[s] = 1.0 / dold;
                idref[s] = (idx == 0) ? idold[s] : 1.0 / d0new[s];   // delta(1,:,m) | delta(h) (Q4)
            }
            suffix_sum_nv<NV>(Tm, l);
            delta_chain_nv<NV>(d, l, Tm, Gm, idold, idref, dm);
        }
        double tm[NV];
#pragma unroll
        for (int s = 0; s < NV; ++s) tm[s] = (l + 64 * s < d.K) ? dm[s] : 1.0;
        scan_prod_nv<NV>(tm, l);                                     // tauh = cumprod(delta)
#pragma unroll
        for (int s = 0; s < NV; ++s) {
            const int idx = l + 64 * s;
            const bool act = idx < d.K;
            const size_t o = (size_t)m * KW + idx;
            delta_out[o] = act ? dm[s] : delta_in[o];
            tau_out[o] = act ? tm[s] : tau_in[o];
        }
    }
}

template <int KW>
__global__ __launch_bounds__(64) void k_delta(Dims d, const double *__restrict__ sall,
                                               const double *__restrict__ delta_in, const double *__restrict__ tau_in,
                                               double *__restrict__ delta_out, double *__restrict__ tau_out,
                                               DrawsDev dr, int64_t iter) {
    delta_shard_w<KW>(d, sall, delta_in, tau_in, delta_out, tau_out, dr, iter, blockIdx.x, threadIdx.x);
}

// ============================================================================
// launchers (kernels.hip dispatches here when d.kp != 32)
// ============================================================================
#define WIDE_DISPATCH(KWV, CALL)        \
    do {                                \
        if ((KWV) == 64) {              \
            constexpr int KW = 64;      \
            CALL;                       \
        } else {                        \
            constexpr int KW = 128;     \
            CALL;                       \
        }                               \
    } while (0)

void launch_prep(const Dims &d, const Bufs &b, hipStream_t s) {
    WIDE_DISPATCH(d.kp, {
        hipLaunchKernelGGL(k_gram<KW>, dim3((KW / 32) * (KW / 32), d.G), dim3(64 * GRAM_WAVES), 0, s, d, b.Lam, b.omega,
                           b.A);
        hipLaunchKernelGGL(k_prep<KW>, dim3(d.G), dim3(TILE_THREADS), 0, s, d, b.A, b.ZM);
    });
}
void launch_xchol(const Dims &d, const Bufs &b, hipStream_t s) {
    WIDE_DISPATCH(d.kp, hipLaunchKernelGGL(k_xchol<KW>, dim3(1), dim3(TILE_THREADS), 0, s, d,
                                           d.coll ? b.xa_all : b.xa, b.XM));
}
// f(std::integral_constant<int, ceil(K / 8)>) for the wide widths (KW = 64: 5..8, KW = 128: 9..16)
template <int KW, class F, int... I>
static void dispatch_tk_impl(int tk, F &&f, std::integer_sequence<int, I...>) {
    ((tk == KW / 16 + 1 + I ? (f(std::integral_constant<int, KW / 16 + 1 + I>{}), 0) : 0), ...);
}
template <int KW, class F>
static void dispatch_tk(int K, F &&f) {   // tk in KW / 16 + 1 .. KW / 8
    dispatch_tk_impl<KW>((K + 7) / 8, f, std::make_integer_sequence<int, KW / 16>{});
}
void launch_zdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    WIDE_DISPATCH(d.kp, dispatch_tk<KW>(d.K, [&](auto T) {
        hipLaunchKernelGGL((k_zdraw<KW, decltype(T)::value>), dim3((d.NP / (16 * ZD_RT)) * d.G), dim3(256), 0, s, d, b.W,
                           b.A, b.ZM, b.X, b.Z, b.Sp, dr, iter);
    }));
}
void launch_xdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    WIDE_DISPATCH(d.kp, dispatch_tk<KW>(d.K, [&](auto T) {
        hipLaunchKernelGGL((k_xdraw<KW, decltype(T)::value>), dim3(cdiv(d.n, 16)), dim3(64 * xd_waves<KW>()), 0, s, d,
                           b.xall, b.XM, b.X, dr, iter);
    }));
}
void launch_lambda(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, const double *tau_cur,
                   const double *plam_src, hipStream_t s, double kappa_max) {
    const dim3 grid(d.P, d.G);
    int *rflag = std::isinf(kappa_max) ? nullptr : b.rflag;   // exact mode: k_resid redoes every row
#define LT(KWV, NBV)                                                                                             \
    hipLaunchKernelGGL((k_lambda_w<KWV, NBV>), grid, dim3(64), 0, s, d, b.C, b.E, b.yy, tau_cur, plam_src, b.Lam, \
                       b.psi, b.ps, b.omega, b.cpart, dr, iter, kappa_max, rflag)
    switch ((d.K + 15) / 16) {            // K = 33..128: 3..8 tile rows
    case 3: LT(64, 3); break;
    case 4: LT(64, 4); break;
    case 5: LT(128, 5); break;
    case 6: LT(128, 6); break;
    case 7: LT(128, 7); break;
    default: LT(128, 8); break;
    }
#undef LT
}
void launch_delta(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, const double *delta_in,
                  const double *tau_in, double *delta_out, double *tau_out, hipStream_t s) {
    WIDE_DISPATCH(d.kp, hipLaunchKernelGGL(k_delta<KW>, dim3(d.g), dim3(64), 0, s, d, b.sall, delta_in, tau_in,
                                           delta_out, tau_out, dr, iter));
}
#undef WIDE_DISPATCH

}  // namespace wide
}  // namespace dcfm
