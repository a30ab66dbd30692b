// Hand-written CDNA4 (gfx950) kernels for one Gibbs iteration of the
// divide-and-conquer factor model (reference divideconquer.m:90-196) and the
// covariance assembly.  fp64 throughout (the reference is double precision).
//
// Kernel map (per iteration, in order)                         reference lines
//   fused chain (K <= 32), one stream:
//   k_wcol     [Z operators A_m -> M1, M2, U, NA (dc:98-107) | column sums of t-1 (dc:156) |
//              shard sum of A, one rank: Xprec = g I + rho sum A, Rx (dc:112-118)] beside
//              the W pass W_m = Y_m (w o Lambda_m) whose tiles draw Z from their registers
//              and write Z and the shard X message (dc:101-107,121-123), and behind it the
//              loading-row variates of t (dc:142,150,170) for k_lambda
//   several ranks: k_xred (local sum of the X messages) + ONE RCCL all-gather of
//              [column sums | A sum | X message]
//   k_xdraw    X rows (dc:119-128) [+ several ranks: Xprec, Rx from the ranks' A sums] +
//              the delta / tau chain of t-1 (dc:155-165)
//   k_cpass    C_m = Y_m' eta_m, E_m = eta_m' eta_m  fp64 MFMA, Y pass 2   dc:133,138,141
//   k_lambda   per loading row: Q, chol, 3 solves, Lambda_j; psi_j;        dc:140-145,150,
//              SS_j via identity, ps_j, omega_j; psi o L^2 per row         dc:156,169-171
//   side-stream layouts (K > 32, DCFM_FLAG_UNFUSED):
//   k_prep / k_xchol (side stream), k_wpass, k_zdraw, k_xred [+ all-gather], k_xdraw,
//   k_cpass, k_lambda, k_colsum [+ all-gather], k_delta
//   (Plam = psi o tau' of dc:175-177 is formed where it is read: in the next
//    k_lambda, from the psi and tau arrays — the same single product)
//   saved iterations: k_save; per batch on the assembly stream (overlapping
//   the following iterations): [RCCL all-gather], k_assemble            dc:180-195
//
// The residual pass of dc:169-170 needs no third read of Y: with C_j = eta'Y_j
// and E = eta'eta already computed for the loading draw,
//   SS_j = sum_i (Y_ij - eta_i Lambda_j')^2 = yy_j - 2 Lambda_j.C_j + Lambda_j E Lambda_j'.
#include "dcfm_internal.h"
#include "philox.h"
#include "linalg.h"
#include "lambda.h"

#include <algorithm>

namespace dcfm {

#ifdef DCFM_WSTAMPS   // dev build: per-block [start, end] (s_memrealtime, 100 MHz) of the last full k_wcol,
                      // and inside the block [2] OPS: A_m out / W tile: pass done, [3] OPS: U out / W tile:
                      // operators arrived, [4] W tile: operators staged, [5] W tile: first 16-row draw done
__device__ unsigned long long g_wstamps[8192][8];
extern "C" int dcfm_debug_wstamps(unsigned long long *out, int nblocks) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wstamps), (size_t)nblocks * 64, 0, hipMemcpyDeviceToHost);
}
#define WSTAMP(s) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_wstamps[blockIdx.x][s] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define WSTAMP(s) do { } while (0)
#endif

// device helpers (MFMA, lane broadcast, rsqrt, register Cholesky): linalg.h

// ============================================================================
// k_prep: A_m = (w o Lambda_m)' Lambda_m and the Z-draw operators of shard m    dc:98-107
//   L = chol(Zprec) lower, Zprec = eye(K) + (1-rho) A_m (cholcov's R = L')
//   U = L^{-1} = R^{-T},  T = U U' = R^{-T} R^{-1}   (quirk Q2: the reference's mean
//   R'\(R\bz) is T bz, its noise R'\z is U z), so with bz = sqrt(1-rho)(W - sqrt(rho) A x):
//     Z = M1 W + M2 x + U eps,   M1 = sqrt(1-rho) T,  M2 = -sqrt(1-rho) sqrt(rho) T A
//     S = W + NA Z,              NA = -sqrt(1-rho) A
// ZM[m] = {M1, M2, U, NA}.  4 waves split the j reduction of A (fp64 MFMA 2x2 tiles).
// ============================================================================
constexpr int PREP_SMEM = 4 * KP * (KP + 1) + 3 * TS16;
// prep_gram: A_m (to HBM and LDS part[0]), NA, and Zprec's upper triangle into the
// lower triangle of part[2]; prep_ops: the Z-draw operators from the LDS image.
// PUB: A_m, NA and (prep_ops) the Z operators are published with agent-scope stores (read by other
// blocks of the same launch, k_wcol)
template <bool PUB = false>
__device__ __forceinline__ void prep_gram(const Dims &d, const double *__restrict__ Lam,
                                          const double *__restrict__ omega, double *__restrict__ A,
                                          double *__restrict__ ZM, int m, double *smem) {
    // partial A per wave; later A, U, Zprec/T, scratch
    double (*part)[KP][KP + 1] = reinterpret_cast<double (*)[KP][KP + 1]>(smem);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int r = lane & 15, q = lane >> 4;
    const double *L = Lam + (size_t)m * d.PP * KP;
    const double *w = omega + (size_t)m * d.PP;
    d4 a00 = {0, 0, 0, 0}, a01 = a00, a10 = a00, a11 = a00;
    // rows j, j+1 of chunk tt: (w_j Lambda_ja) is the A operand [Zmsg, dc:98], Lambda_jb the B operand
    auto ld = [&](int tt, d2 &wj, double (&l)[4]) {
        const int j = 8 * tt + 2 * q;
        wj = *reinterpret_cast<const d2 *>(w + j);
        l[0] = L[j * KP + r]; l[1] = L[j * KP + 16 + r];
        l[2] = L[(j + 1) * KP + r]; l[3] = L[(j + 1) * KP + 16 + r];
    };
    auto mm = [&](const d2 &wj, const double (&l)[4]) {
        const double wl0 = l[0] * wj.x, wh0 = l[1] * wj.x, wl1 = l[2] * wj.y, wh1 = l[3] * wj.y;
        a00 = mfma16x16x4(wl0, l[0], a00); a01 = mfma16x16x4(wl0, l[1], a01);
        a10 = mfma16x16x4(wh0, l[0], a10); a11 = mfma16x16x4(wh0, l[1], a11);
        a00 = mfma16x16x4(wl1, l[2], a00); a01 = mfma16x16x4(wl1, l[3], a01);
        a10 = mfma16x16x4(wh1, l[2], a10); a11 = mfma16x16x4(wh1, l[3], a11);
    };
    const int nt = d.PP >> 3;
    int tt = wave;
    for (; tt + 12 < nt; tt += 16) {       // 4 chunks' loads in flight (latency-bound otherwise;
                                           // one round of 10 measured slower: c3 -1.5%)
        d2 wj[4];
        double l[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ld(tt + 4 * u, wj[u], l[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) mm(wj[u], l[u]);
    }
    for (; tt < nt; tt += 4) {
        d2 wj;
        double l[4];
        ld(tt, wj, l);
        mm(wj, l);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int a = q + 4 * g;
        part[wave][a][r] = a00[g];
        part[wave][a][16 + r] = a01[g];
        part[wave][16 + a][r] = a10[g];
        part[wave][16 + a][16 + r] = a11[g];
    }
    __syncthreads();
    double *Am = A + (size_t)m * KP * KP;
    double *Zm = ZM + (size_t)m * 4 * KP * KP;
    double av[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = t + 256 * u, a = e / KP, b = e % KP;
        av[u] = (part[0][a][b] + part[1][a][b]) + (part[2][a][b] + part[3][a][b]);
        if (PUB) st_agent(Am + e, av[u]);
        else Am[e] = av[u];
        if (PUB) st_agent(Zm + 3 * KP * KP + e, -d.s1r * av[u]);   // NA
        else Zm[3 * KP * KP + e] = -d.s1r * av[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = t + 256 * u;
        const int a = e / KP, b = e % KP;
        part[0][a][b] = av[u];                                      // A
        // cholcov reads the upper triangle: lower of Sm = (Zprec upper)'
        if (a <= b) part[2][b][a] = (a == b ? 1.0 : 0.0) + (1.0 - d.rho) * av[u];
    }
    __syncthreads();
}

// the LDS image prep_gram leaves, from A_m in HBM (the operators run in a later launch)
__device__ __forceinline__ void prep_load(const Dims &d, const double *__restrict__ A, int m, double *smem) {
    double (*part)[KP][KP + 1] = reinterpret_cast<double (*)[KP][KP + 1]>(smem);
    const double *Am = A + (size_t)m * KP * KP;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = threadIdx.x + 256 * u;
        const int a = e / KP, b = e % KP;
        const double v = Am[e];
        part[0][a][b] = v;
        if (a <= b) part[2][b][a] = (a == b ? 1.0 : 0.0) + (1.0 - d.rho) * v;
    }
    __syncthreads();
}

template <bool PUB = false>
__device__ __forceinline__ void prep_ops(const Dims &d, double *__restrict__ ZM, int m, double *smem) {
    double (*part)[KP][KP + 1] = reinterpret_cast<double (*)[KP][KP + 1]>(smem);
    double *lds_l = smem + 4 * KP * (KP + 1), *lds_u = lds_l + 2 * TS16;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    double *Zm = ZM + (size_t)m * 4 * KP * KP;
    if (wave == 0) {                                                // U = L^{-1} -> part[1]
        chol_inv32(part[2], part[1], part[3], lds_l, lds_u, lane);
    }
    __syncthreads();
    if (PUB) WSTAMP(3);
    {   // T = U U' (fp64 MFMA, one 16x16 tile per wave) -> part[2]; M1 = s1r T; U
        const int ti = wave >> 1, tj = wave & 1, j = lane & 15, q = lane >> 4;
        const d4 T = mfma_tile32<true>(part[1], part[1], ti, tj, lane);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int a = 16 * ti + q + 4 * g, c = 16 * tj + j;
            part[2][a][c] = T[g];
            if (PUB) {
                st_agent(Zm + a * KP + c, d.s1r * T[g]);
                st_agent(Zm + 2 * KP * KP + a * KP + c, part[1][a][c]);
            } else {
                Zm[a * KP + c] = d.s1r * T[g];                      // M1
                Zm[2 * KP * KP + a * KP + c] = part[1][a][c];       // U
            }
        }
    }
    __syncthreads();
    {   // M2 = -s1r sr T A (fp64 MFMA)
        const int ti = wave >> 1, tj = wave & 1, j = lane & 15, q = lane >> 4;
        const d4 M = mfma_tile32<false>(part[2], part[0], ti, tj, lane);
        const double s2 = -d.s1r * d.sr;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            double *o = Zm + KP * KP + (16 * ti + q + 4 * g) * KP + 16 * tj + j;
            if (PUB) st_agent(o, s2 * M[g]);
            else *o = s2 * M[g];
        }
    }
}

__device__ __forceinline__ void prep_shard(const Dims &d, const double *__restrict__ Lam,
                                           const double *__restrict__ omega, double *__restrict__ A,
                                           double *__restrict__ ZM, int m, double *smem) {
    prep_gram(d, Lam, omega, A, ZM, m, smem);
    prep_ops(d, ZM, m, smem);
}

__global__ __launch_bounds__(256) void k_prep(Dims d, const double *__restrict__ Lam,
                                              const double *__restrict__ omega,
                                              double *__restrict__ A, double *__restrict__ ZM) {
    __shared__ double smem[PREP_SMEM];
    prep_shard(d, Lam, omega, A, ZM, blockIdx.x, smem);
}

#ifndef DCFM_WP_RING
#define DCFM_WP_RING 3
#endif
constexpr int WP_RING = DCFM_WP_RING;   // W pass register ring depth (chunks)
#ifndef DCFM_WP_RING_WIDE
#define DCFM_WP_RING_WIDE 4
#endif
// the wide layouts' pass (k_wpass<64 / 128>: 2 waves per SIMD at c4) takes one chunk more in flight
// (c4: 152 -> 127 us; ab_rg in profiles/r06_ab_summary.txt); the same products in the same order
constexpr int WP_RING_WIDE = DCFM_WP_RING_WIDE;
// ============================================================================
// k_wpass: W_m[i][k] = sum_j Y_m[i][j] (w_j Lambda_m[j][k])   fp64 MFMA, Y pass 1
// one wave = (shard m, 16 MT rows i = MT M-tiles) x 32 k (even / odd k tiles) of
// column tile kt (KW/32 tiles, adjacent in the 1-D grid so the wide layouts re-read Y from L2),
// reduction over j in chunks of 8: lane (r, q) holds Y[i0+r][8t+2q .. +1] (16 B);
// k-step 2t uses element 0, 2t+1 element 1; the (w_j L[j][2r], w_j L[j][2r+1]) values use the
// same j <-> (q, e) map.  The product is formed transposed, W' = (w o L)' Y' (the Lambda values
// the A operand, Y the B operand: the same products in the same order per element), so lane
// (r, q) ends with W[i0 + 16a + r][8g + 2q + tb] in acc[a][tb][g] — row = lane & 15, the layout
// the Z draw takes its W operand in (zdraw_rows; k_wcol draws Z from these registers).
// Register prefetch 3 chunks ahead (ring of 4).
// MT = 1 (64-row blocks, twice the blocks) where the launch would not fill the chip (a few
// shards per rank): each element's reduction order is the same for both, so the choice
// changes no bit of W.
// ============================================================================
// Register ring of R chunks: chunk t + R - 1 is requested while chunk t multiplies, so R - 1
// chunks are in flight behind the MFMAs.  pre() runs once the first R - 1 chunks' loads are
// issued (VALU work hidden behind their latency).
template <int KW, int MT, int R = (KW > KP ? WP_RING_WIDE : WP_RING), class Pre>
__device__ __forceinline__ void wpass_acc(const Dims &d, const double *__restrict__ Y, const double *__restrict__ Lam,
                                          const double *__restrict__ omega, int m, int i0, int kt, d4 (&acc)[MT][2],
                                          Pre &&pre) {
    const int lane = threadIdx.x & 63;
    const int r = lane & 15, q = lane >> 4;
    const double *Y0 = Y + ((size_t)m * d.NP + i0 + r) * d.PP + 2 * q;
    const double *Y1 = Y0 + (size_t)16 * (MT - 1) * d.PP;
    const double *L = Lam + (size_t)m * d.PP * KW + 32 * kt + 2 * r;
    const double *wp = omega + (size_t)m * d.PP + 2 * q;
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int nch = d.PP >> 3;
    d2 y0[R], y1[R], ww[R], l0[R], l1[R];
    auto load = [&](int t, int k) {
        const int j = 8 * t;
        y0[k] = *reinterpret_cast<const d2 *>(Y0 + j);
        if (MT == 2) y1[k] = *reinterpret_cast<const d2 *>(Y1 + j);
        ww[k] = *reinterpret_cast<const d2 *>(wp + j);
        l0[k] = *reinterpret_cast<const d2 *>(L + (size_t)(j + 2 * q) * KW);
        l1[k] = *reinterpret_cast<const d2 *>(L + (size_t)(j + 2 * q + 1) * KW);
    };
    // the two k-steps of a chunk accumulate into separate sets (8 independent MFMA chains per wave
    // instead of 4), added at the end: W = (sum over even j) + (sum over odd j)
    d4 acc2[MT][2];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc2[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    auto mma = [&](int k) {
        const double b00 = ww[k].x * l0[k].x, b01 = ww[k].x * l0[k].y;
        const double b10 = ww[k].y * l1[k].x, b11 = ww[k].y * l1[k].y;
        acc[0][0] = mfma16x16x4(b00, y0[k].x, acc[0][0]);
        acc[0][1] = mfma16x16x4(b01, y0[k].x, acc[0][1]);
        if (MT == 2) {
            acc[MT - 1][0] = mfma16x16x4(b00, y1[k].x, acc[MT - 1][0]);
            acc[MT - 1][1] = mfma16x16x4(b01, y1[k].x, acc[MT - 1][1]);
        }
        acc2[0][0] = mfma16x16x4(b10, y0[k].y, acc2[0][0]);
        acc2[0][1] = mfma16x16x4(b11, y0[k].y, acc2[0][1]);
        if (MT == 2) {
            acc2[MT - 1][0] = mfma16x16x4(b10, y1[k].y, acc2[MT - 1][0]);
            acc2[MT - 1][1] = mfma16x16x4(b11, y1[k].y, acc2[MT - 1][1]);
        }
    };
#pragma unroll
    for (int k = 0; k < R - 1; ++k)
        if (k < nch) load(k, k);
    pre();
    for (int t = 0; t < nch; t += R) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            if (t + k + R - 1 < nch) load(t + k + R - 1, (k + R - 1) % R);
            if (t + k < nch) mma(k);
        }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] += acc2[a][b];
}

template <int KW, int MT = 2>
__device__ __forceinline__ void wpass_tile(const Dims &d, const double *__restrict__ Y,
                                           const double *__restrict__ Lam, const double *__restrict__ omega,
                                           double *__restrict__ W, int w, int kt) {
    const int nrb = d.NP / (64 * MT);                // row blocks per shard
    const int m = w / nrb, rb = w % nrb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i0 = rb * 64 * MT + wave * 16 * MT;
    const int r = lane & 15, q = lane >> 4;
    d4 acc[MT][2];
    wpass_acc<KW, MT>(d, Y, Lam, omega, m, i0, kt, acc, [] {});
    // acc[a][tb][g] = W[i0 + 16a + r][32 kt + 8g + 2q + tb]: one 16-byte pair per (a, g)
#pragma unroll
    for (int a = 0; a < MT; ++a) {
        double *Wt = W + ((size_t)m * d.NP + i0 + 16 * a + r) * KW + 32 * kt + 2 * q;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            d2 v;
            v.x = acc[a][0][g];
            v.y = acc[a][1][g];
            *reinterpret_cast<d2 *>(Wt + 8 * g) = v;
        }
    }
}

template <int KW>
__global__ __launch_bounds__(256) void k_wpass(Dims d, const double *__restrict__ Y,
                                               const double *__restrict__ Lam,
                                               const double *__restrict__ omega,
                                               double *__restrict__ W) {
    // 1-D grid, the KW/32 column tiles of one 128-row block adjacent (same XCD: Y from L2)
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    wpass_tile<KW>(d, Y, Lam, omega, W, w / (KW / 32), w % (KW / 32));
}

// ============================================================================
// k_zdraw: Z draw and per-shard X message as fp64 MFMA chains.   dc:101-107,121-123
//   Z' = M1 W' + M2 X' + U eps'      (k_prep operators; columns = rows i)
//   S' = W' + NA Z'                  (S_i = Xmsg'(Y_i - sqrt(1-rho) L Z_i))
// block = (shard m, 128 rows), 8 waves, one 16-row tile per wave.  Operand lane map:
// lane (c = lane&15, q = lane>>4) holds W[i0+c][8t+2q .. +1] (k-steps 2t+e); the three
// products of Z' accumulate in separate registers (6 independent MFMA chains per wave,
// 4 waves per SIMD: fp64 MFMA needs many chains in flight) and are added at the end
// ((M1 W' + M2 X') + U eps').  The f64 C/D layout of Z' (row = q + 4r) is directly the B
// operand of the NA Z' product (k-step r), so nothing crosses LDS.
// ============================================================================
constexpr int ZDRAW_SMEM = 4 * KP * (KP + 1);
constexpr int ZROWS = 128, ZTHREADS = 512;     // rows and threads per k_zdraw block

// The draw of 16 rows from the operand registers — lane (c, q) holds row i = (its tile's row c):
// wv[t] = W[i][8t+2q .. +1], xv[t] = X[i][..], ev[t] = eps[i][..] (k-steps 2t + e) — and the
// shard's operators Ms = {M1, M2, U, NA} in LDS.  The S' = W' + NA Z' product takes its A rows
// in the order pi(16 mt + c) = 8 (c >> 2) + 2 (c & 3) + mt, so its C/D registers hold exactly the
// features of wv (the accumulators start from W without a reload, and a lane stores S_i[8g+2q ..
// +1] as one 16-byte pair); every element keeps its products and their order, so the values
// are those of the unpermuted product.  Shared by k_zdraw (W from HBM) and k_wcol's
// fused W pass (W' still in the W-pass accumulators), which therefore give the same bits.
__device__ __forceinline__ void zdraw_rows(const Dims &d, const double (*Ms)[KP][KP + 1], const d2 (&wv)[4],
                                           const d2 (&xv)[4], const d2 (&ev)[4], double *__restrict__ Zr,
                                           double *__restrict__ Sr, bool live, int c, int q) {
    d4 zw[2], zx[2], ze[2], as[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) zw[mt] = zx[mt] = ze[mt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        double mo[2][3][2];   // this chunk's operator values, read before its 12 MFMAs
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int mat = 0; mat < 3; ++mat)
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) mo[e][mat][mt] = Ms[mat][16 * mt + c][8 * t + 2 * q + e];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const double we = e ? wv[t].y : wv[t].x, xe = e ? xv[t].y : xv[t].x;
            const double ee = e ? ev[t].y : ev[t].x;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                zw[mt] = mfma16x16x4(mo[e][0][mt], we, zw[mt]);
                zx[mt] = mfma16x16x4(mo[e][1][mt], xe, zx[mt]);
                ze[mt] = mfma16x16x4(mo[e][2][mt], ee, ze[mt]);
            }
        }
    }
    d4 az[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        az[mt] = (zw[mt] + zx[mt]) + ze[mt];
#pragma unroll
        for (int g = 0; g < 4; ++g) as[mt][g] = mt ? wv[g].y : wv[g].x;     // W[i][8g + 2q + mt]
    }
    // S' = W' + NA Z' (rows of NA in the order pi)
    const int prow = 8 * (c >> 2) + 2 * (c & 3);
#pragma unroll
    for (int mt2 = 0; mt2 < 2; ++mt2)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int kk = 16 * mt2 + 4 * g + q;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) as[mt] = mfma16x16x4(Ms[3][prow + mt][kk], az[mt2][g], as[mt]);
        }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int k = 16 * mt + q + 4 * g;
            if (live) Zr[k] = (k < d.K) ? az[mt][g] : 0.0;
        }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        d2 v;
        v.x = live ? as[0][g] : 0.0;
        v.y = live ? as[1][g] : 0.0;
        *reinterpret_cast<d2 *>(Sr + 8 * g + 2 * q) = v;
    }
}
// eps[i][kk], kk = 8t + 2q + e of the Z draw (dc:104 normrnd): the injected draw buffer, or
// generated here — Philox pair 4t + q of (SITE_Z, shard, row i) = normals kk, kk + 1
__device__ __forceinline__ void z_eps(const Dims &d, const DrawsDev &dr, int64_t iter, int mg, int i, bool live, int q,
                                      d2 (&ev)[4]) {
    if (d.inject) {
        const double *nz = dr.NZ + (((size_t)(iter - dr.first_iter) * d.g + mg) * d.n + (live ? i : 0)) * d.K;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int kk = 8 * t + 2 * q;
            ev[t].x = (live && kk < d.K) ? nz[kk] : 0.0;
            ev[t].y = (live && kk + 1 < d.K) ? nz[kk + 1] : 0.0;
        }
    } else {
        const Rng rng(d.seed);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int kk = 8 * t + 2 * q;
            double n0 = 0.0, n1 = 0.0;
#ifndef DCFM_DEV_NO_ZNORM   // timing-only dev build: zero normals
            if (live && kk < d.K) rng.normal2(SITE_Z, (uint32_t)mg, (uint32_t)i, (uint32_t)(4 * t + q), (uint32_t)iter, n0, n1);
#endif
            ev[t].x = n0;
            ev[t].y = (kk + 1 < d.K) ? n1 : 0.0;
        }
    }
}

// ZT threads = ZT / 4 rows per block: 256 (64-row blocks) where 128-row ones would leave CUs
// idle (a few shards per rank); rows are independent, so the choice changes no bit
template <int ZT = ZTHREADS>
__device__ __forceinline__ void zdraw_tile(const Dims &d, const double *__restrict__ W,
                                           const double *__restrict__ ZM, const double *__restrict__ X,
                                           double *__restrict__ Z, double *__restrict__ Sp, const DrawsDev &dr,
                                           int64_t iter, int w, double *smem) {
    double (*Ms)[KP][KP + 1] = reinterpret_cast<double (*)[KP][KP + 1]>(smem);   // M1, M2, U, NA
    const int nrb = d.NP / (ZT / 4);
    const int m = w / nrb, rb = w % nrb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, q = lane >> 4;
    const int mg = d.shard0 + m;
    const int i0 = rb * (ZT / 4) + wave * 16;
    const int i = i0 + c;
    const bool live = i < d.n;
    // this wave's operands first (in flight while the block stages the operators)
    const double *Wi = W + ((size_t)m * d.NP + i) * KP + 2 * q;
    const double *Xi = X + (size_t)i * KP + 2 * q;
    d2 wv[4], xv[4], ev[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        wv[t] = *reinterpret_cast<const d2 *>(Wi + 8 * t);
        xv[t] = *reinterpret_cast<const d2 *>(Xi + 8 * t);
    }
    // the block's share of the shard's operators, in flight during the draws below (stored to
    // LDS after them: a store per load made the compiler wait for each load in turn)
    constexpr int NU = 4 * KP * KP / ZT;
    double zv[NU];
    {
        const double *Zm = ZM + (size_t)m * 4 * KP * KP;
#pragma unroll
        for (int u = 0; u < NU; ++u) zv[u] = Zm[threadIdx.x + ZT * u];
    }
    z_eps(d, dr, iter, mg, i, live, q, ev);
    {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = threadIdx.x + ZT * u;
            const int mat = e / (KP * KP), rem = e % (KP * KP);
            Ms[mat][rem / KP][rem % KP] = zv[u];
        }
    }
    __syncthreads();
    zdraw_rows(d, Ms, wv, xv, ev, Z + ((size_t)m * d.NP + i) * KP, Sp + ((size_t)m * d.NP + i) * KP, live, c, q);
}

// ZT = 256 holds twice the operator staging registers per thread: 2 waves per SIMD (it runs
// only where the launch leaves SIMDs idle anyway) instead of a 128-VGPR cap that spilled
template <int ZT>
__global__ __launch_bounds__(ZT) __attribute__((amdgpu_waves_per_eu(ZT == ZTHREADS ? 4 : 2))) void k_zdraw(Dims d, const double *__restrict__ W,
                                               const double *__restrict__ ZM,
                                               const double *__restrict__ X,
                                               double *__restrict__ Z, double *__restrict__ Sp,
                                               DrawsDev dr, int64_t iter) {
    __shared__ double smem[ZDRAW_SMEM];
    zdraw_tile<ZT>(d, W, ZM, X, Z, Sp, dr, iter, xcd_remap(blockIdx.x, gridDim.x), smem);
}

// ============================================================================
// k_xred: xin[i][k] = sum_m Sp[m][i][k]  (local shards, canonical tree)  dc:120-124
// ============================================================================
__global__ __launch_bounds__(256) void k_xred(Dims d, const double *__restrict__ Sp,
                                              double *__restrict__ xin) {
    const size_t total = (size_t)d.NP * d.kp;
    const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (e >= total) return;
    xin[e] = tree_sum(Sp + e, d.G, total);
}

// ============================================================================
// k_asum: xa = sum_m A_m over local shards (canonical tree), one thread per element.  dc:113-116
// ============================================================================
__global__ __launch_bounds__(256) void k_asum(Dims d, const double *__restrict__ A,
                                              double *__restrict__ xa) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int kk = d.kp * d.kp;
    if (e >= kk) return;
    xa[e] = tree_sum(A + e, d.G, (size_t)kk);
}

// ============================================================================
// k_xchol: Xprec = g*I + rho*sum A (dc:117) and Rx = cholcov(Xprec) (dc:118), on the
// side stream.  Sums the per-rank sums xa_all (k_asum, all-gathered) in the canonical tree
// and writes the X-draw operators XM = {Tx = sqrt(rho) Ux Ux', Ux = Rx^{-T}} (Tx by MFMA).
// ============================================================================
constexpr int XCHOL_SMEM = 2 * KP * (KP + 1) + TS16 * (KP + 1) + 3 * TS16 + 2;
// smem = {Sm, Us, Wk, lds_l, lds_u, flag}; Sm (lower) holds Xprec's upper triangle on entry
// PUB: XM is published with agent-scope stores (read by other blocks of the same launch, k_xdraw)
template <bool PUB = false>
__device__ __forceinline__ void xchol_factor(const Dims &d, double *__restrict__ XM, double *smem) {
    double (*Sm)[KP + 1] = reinterpret_cast<double (*)[KP + 1]>(smem);
    double (*Us)[KP + 1] = Sm + KP;
    double (*Wk)[KP + 1] = Us + KP;
    double *lds_l = smem + 2 * KP * (KP + 1) + TS16 * (KP + 1), *lds_u = lds_l + 2 * TS16;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (wave == 0) {                       // Ux = Lx^{-1} = Rx^{-T}
        chol_inv32(Sm, Us, Wk, lds_l, lds_u, lane);
    }
    __syncthreads();
    if (wave >= 4) return;                 // blocks of more than 4 waves: the 4 tiles below
    // X = Rx^{-T}(Rx^{-1} sqrt(rho) S + eps) = Tx S + Ux eps,  Tx = sqrt(rho) Ux Ux'
    const int ti = wave >> 1, tj = wave & 1, j = lane & 15, q = lane >> 4;
    const d4 T = mfma_tile32<true>(Us, Us, ti, tj, lane);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int a = 16 * ti + q + 4 * g, c = 16 * tj + j;
        if (PUB) {
            st_agent(XM + a * KP + c, d.sr * T[g]);
            st_agent(XM + KP * KP + a * KP + c, Us[a][c]);
        } else {
            XM[a * KP + c] = d.sr * T[g];
            XM[KP * KP + a * KP + c] = Us[a][c];
        }
    }
}

// Xprec's upper triangle, transposed into the lower triangle of Sm: g I + rho sum A   dc:117
__device__ __forceinline__ void xprec_store(const Dims &d, double *smem, int e, double v) {
    double (*Sm)[KP + 1] = reinterpret_cast<double (*)[KP + 1]>(smem);
    const int a = e / KP, b = e % KP;
    if (a <= b) Sm[b][a] = (a == b ? (double)d.g : 0.0) + d.rho * v;
}

__global__ __launch_bounds__(256) void k_xchol(Dims d, const double *__restrict__ xa_all,
                                               double *__restrict__ XM) {
    __shared__ double smem[XCHOL_SMEM];
    for (int e = threadIdx.x; e < KP * KP; e += 256) {
        xprec_store(d, smem, e, tree_sum(xa_all + e, d.nranks, (size_t)d.xstride));
    }
    __syncthreads();
    xchol_factor(d, XM, smem);
}

// ============================================================================
// k_draws: every standard variate one iteration consumes, from
// the counter-based Philox stream, into buffers with the injected-draw layout
// (T = 1).  ALU-bound; it runs on the side stream one iteration ahead, overlapping
// the HBM-bound Y passes, so the sweep kernels only load their variates.
// Segments (wave-aligned): NZ pairs (local shards), NX pairs, NL pairs (local),
// Gpsi (local), Gps (local), Gdelta (all g shards: every rank runs every chain).
// Pointers are indexed by GLOBAL shard mg (as the injected full-g arrays are).
// ============================================================================
// Block plan of k_draws: every segment gets whole blocks, and a block covers
// 256 / LR rows of one shard with LR in {16, 32, 64} lanes per row (the smallest that
// holds a row's pairs / gammas, K <= 128), so a thread's (shard, row, index) comes
// from shifts and one block-uniform division — no per-element integer division.
// The rejection-sampled gammas (delta: one per thread; ps: one per thread) come first
// in block order so their longer threads start early; the bulk normals follow.
struct DrawPlan {
    int lrn, lrg;                    // lanes per row: normal pairs, gamma row (Gpsi)
    int nrb_n, nrb_p, nrb_g, nrb_s;  // row-blocks per shard: n rows, P rows (normals), P rows (Gpsi), Gps
    int b_gdel, b_gps, b_gpsi, b_nz, b_nx, total;  // segment end blocks (cumulative); NL last
};
__host__ __device__ inline int lanes_for(int c) { return c <= 16 ? 16 : (c <= 32 ? 32 : 64); }
__host__ __device__ inline DrawPlan draw_plan(const Dims &d) {
    DrawPlan pl;
    const int kp2 = (d.K + 1) / 2;
    pl.lrn = lanes_for(kp2);
    pl.lrg = lanes_for(d.K);
    const int rpn = 256 / pl.lrn, rpg = 256 / pl.lrg;
    pl.nrb_n = (d.n + rpn - 1) / rpn;
    pl.nrb_p = (d.P + rpn - 1) / rpn;
    pl.nrb_g = (d.P + rpg - 1) / rpg;
    pl.nrb_s = (d.P + 255) / 256;
    pl.b_gdel = (d.g * d.K + 255) / 256;          // Gdelta of all g shards
    pl.b_gps = pl.b_gdel + d.G * pl.nrb_s;
    pl.b_gpsi = pl.b_gps + d.G * pl.nrb_g;
    pl.b_nz = pl.b_gpsi + d.G * pl.nrb_n;
    pl.b_nx = pl.b_nz + pl.nrb_n;
    pl.total = pl.b_nx + d.G * pl.nrb_p;
    return pl;
}

// normals of one row: lane pair index pr = 0..kp2-1 -> out[2 pr], out[2 pr + 1]
__device__ __forceinline__ void draw_normal_row(const Rng &rng, uint32_t site, uint32_t mg, uint32_t row,
                                                uint32_t it, int K, int lane, int lr, double *out) {
    const int kp2 = (K + 1) / 2;
    for (int pr = lane; pr < kp2; pr += lr) {
        double n0, n1;
        rng.normal2(site, mg, row, (uint32_t)pr, it, n0, n1);
        out[2 * pr] = n0;
        if (2 * pr + 1 < K) out[2 * pr + 1] = n1;
    }
}

// two launches per iteration: the gamma segments (rejection loops, more registers)
// and the normal segments (high occupancy); b_off = first block of the launch
// block b of the draw plan (256 threads)
template <bool GAMMAS>
__device__ __forceinline__ void draws_block(const Dims &d, const DrawsDev &dr, int64_t iter, const DrawPlan &pl,
                                            int b) {
    const Rng rng(d.seed);
    const uint32_t it = (uint32_t)iter;
    const int t = threadIdx.x, K = d.K;
    if (GAMMAS) {
    if (b < pl.b_gdel) {                               // dc:158,163 delta, K x g, all shards
        const int x = b * 256 + t;
        if (x >= d.g * K) return;
        const int h = x % K, mg = x / K;
        const double shape = (h == 0) ? d.ad1 + 0.5 * d.P * d.K : d.ad2 + 0.5 * d.P * (d.K - h);
        const_cast<double *>(dr.Gdelta)[(size_t)mg * K + h] = rng.gamma(shape, SITE_DELTA, (uint32_t)mg, 0, (uint32_t)h, it);
        return;
    }
    if (b < pl.b_gps) {                                // dc:170 ps, P x g, shape as + n/2
        const int bb = b - pl.b_gdel, m = bb / pl.nrb_s, j = (bb % pl.nrb_s) * 256 + t;
        if (j >= d.P) return;
        const uint32_t mg = (uint32_t)(d.shard0 + m);
        const_cast<double *>(dr.Gps)[(size_t)mg * d.P + j] = rng.gamma(d.as_ + 0.5 * d.n, SITE_PS, mg, (uint32_t)j, 0, it);
        return;
    }
    if (b < pl.b_gpsi) {                               // dc:150 psi, device layout [g][P][K]
        const int bb = b - pl.b_gps, m = bb / pl.nrb_g, rb = bb % pl.nrb_g;
        const int sh = pl.lrg == 16 ? 4 : (pl.lrg == 32 ? 5 : 6);
        const int j = rb * (256 / pl.lrg) + (t >> sh), lane = t & (pl.lrg - 1);
        if (j >= d.P) return;
        const uint32_t mg = (uint32_t)(d.shard0 + m);
        double *o = const_cast<double *>(dr.Gpsi) + ((size_t)mg * d.P + j) * K;
        const double shape = d.df * 0.5 + 0.5;
        for (int k = lane; k < K; k += pl.lrg) o[k] = rng.gamma(shape, SITE_PSI, mg, (uint32_t)j, (uint32_t)k, it);
        return;
    }
    return;
    }
    const int sh = pl.lrn == 16 ? 4 : (pl.lrn == 32 ? 5 : 6), lane = t & (pl.lrn - 1), rsub = t >> sh;
    if (b < pl.b_nx) {                                 // dc:104 Z (K x n x g), dc:126 X (K x n)
        const bool xs = b >= pl.b_nz;
        const int bb = xs ? b - pl.b_nz : b - pl.b_gpsi;
        const int m = xs ? 0 : bb / pl.nrb_n, rb = xs ? bb : bb % pl.nrb_n;
        const int i = rb * (256 / pl.lrn) + rsub;
        if (i >= d.n) return;
        const uint32_t mg = xs ? 0u : (uint32_t)(d.shard0 + m);
        double *o = xs ? const_cast<double *>(dr.NX) + (size_t)i * K
                       : const_cast<double *>(dr.NZ) + ((size_t)mg * d.n + i) * K;
        draw_normal_row(rng, xs ? SITE_X : SITE_Z, mg, (uint32_t)i, it, K, lane, pl.lrn, o);
        return;
    }
    {                                                  // dc:142 Lambda (K x P x g)
        const int bb = b - pl.b_nx, m = bb / pl.nrb_p, rb = bb % pl.nrb_p;
        const int j = rb * (256 / pl.lrn) + rsub;
        if (j >= d.P) return;
        const uint32_t mg = (uint32_t)(d.shard0 + m);
        draw_normal_row(rng, SITE_LAMBDA, mg, (uint32_t)j, it, K, lane, pl.lrn,
                        const_cast<double *>(dr.NL) + ((size_t)mg * d.P + j) * K);
    }
}
// hand-off between blocks of one launch (k_wcol, k_xdraw): payload by agent-scope stores,
// s_waitcnt vmcnt(0), then a relaxed fetch-add on a monotonic 64-bit counter; consumers poll
// it (s_sleep) up to the launch's target and read the payload with agent-scope loads.
// Hardware assumption (not the HIP memory model's release / acquire, which on gfx950 costs an
// L2 write-back + invalidate per hand-off, +25 us per k_wcol in round 1): this is the guide's
// cross-XCD hand-off recipe -- (1) every payload store is an agent-scope (sc1) atomic store that
// bypasses the non-coherent per-XCD L2 copy, (2) the storing threads wait for those stores
// (s_waitcnt vmcnt(0)) and meet at the workgroup barrier before one thread signals, (3) the
// polled counter is an atomic, (4) every consumer load of the payload is an agent-scope (sc1)
// load issued after the poll returned.  An ISA without sc1 coherence for relaxed agent-scope
// atomics would break it; tests/test_gpu_loopback.py and the parity tests run these paths.
__device__ __forceinline__ void signal_count(unsigned long long *ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this thread's agent-scope stores are done
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wait_count(unsigned long long *ctr, unsigned long long target) {
    if (threadIdx.x == 0)
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
}

// ============================================================================
// k_xdraw: X' = Tx S' + Ux eps' as fp64 MFMA (operators from k_xchol).  S is the sum of
// nsrc [NP][KP] slices in the canonical tree order (TreeSum): the ranks' gathered sums
// (xall), or — one rank, fused chain — the G shard messages Sp themselves, which makes
// k_xred's launch unnecessary.  16 rows per block, 16 waves: wave (t, s) sums source chunk
// s (a power-of-two run of slices, a canonical subtree; xdraw_chunks) of columns
// 8t .. 8t+7 (lane (c, q): row i0 + c, columns 8t + 2q, +1) — the sum is latency-bound, so
// the block keeps 16 waves of loads in flight; wave 0 adds the chunk sums (the tree over the
// chunks) and runs the MFMAs.                                              dc:119-128
// ============================================================================
// source chunks of the X message sum: nch <= 4 runs of `chunk` slices, chunk a power of two
__device__ __forceinline__ void xdraw_chunks(int nsrc, int &nch, int &chunk) {
    chunk = 1;
    while (nsrc / chunk > 4 && (nsrc / chunk) % 2 == 0) chunk *= 2;
    nch = nsrc / chunk;
    if (nch > 4) { nch = 1; chunk = nsrc; }
}
// one wave = one global shard m of the delta / tau chain (defined with k_delta below)
template <bool COH = false>
__device__ __forceinline__ void delta_shard(const Dims &d, const double *__restrict__ sall,
                                            const double *__restrict__ delta_in, const double *__restrict__ tau_in,
                                            double *__restrict__ delta_out, double *__restrict__ tau_out,
                                            const DrawsDev &dr, int64_t iter, int m, int t);
struct DeltaArgs {
    const double *delta_in, *tau_in;
    double *delta_out, *tau_out;
    int64_t iter;                          // iteration whose delta / tau the chain updates
};
// Roles (xroles & 1, several ranks): block 0 factors Xprec from the ranks' A sums and publishes
// XM; the row blocks sum their messages first and wait for XM only before the MFMAs.  Row
// blocks of XD_ROWS rows (the MFMA's other columns padding), every lane summing one part of a
// source chunk: the shard-message sums are bound by the memory parallelism of the CUs that
// issue them (phase stamps: 9 of 14 us with 63 blocks of 16 rows at c3).
constexpr int XD_ROWS = 4;
constexpr int XD_SMEM = (2 * KP * (KP + 1) + 4 * 4 * 64 * 2) > XCHOL_SMEM ? (2 * KP * (KP + 1) + 4 * 4 * 64 * 2)
                                                                          : XCHOL_SMEM;
__global__ __launch_bounds__(1024) void k_xdraw(Dims d, const double *__restrict__ src, int nsrc, size_t sstride,
                                                double *__restrict__ XM,
                                                double *__restrict__ X, DrawsDev dr, int64_t iter, int xroles,
                                                const double *__restrict__ xa, unsigned long long *xm_ctr,
                                                unsigned long long xm_target) {
    __shared__ double smem[XD_SMEM];
    int blk = blockIdx.x;
    if (xroles & 1) {   // producer of XM
        if (blk == 0) {
            for (int e = threadIdx.x; e < KP * KP; e += 1024)   // several ranks: their sums, canonical tree
                xprec_store(d, smem, e, d.nranks > 1 ? tree_sum(xa + e, d.nranks, (size_t)d.xstride) : xa[e]);
            __syncthreads();
            xchol_factor<true>(d, XM, smem);
            signal_count(xm_ctr);
            return;
        }
        blk -= 1;
    }
    double (*Ms)[KP][KP + 1] = reinterpret_cast<double (*)[KP][KP + 1]>(smem);
    d2 (*part)[4][64] = reinterpret_cast<d2 (*)[4][64]>(smem + 2 * KP * (KP + 1));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, q = lane >> 4;
    const int tw = w & 3, sw = w >> 2;                 // column group, source chunk
    const int i0 = blk * XD_ROWS, i = i0 + c;
    const bool live = c < XD_ROWS && i < d.n;          // lanes c >= XD_ROWS pad the MFMA's 16 columns
    const size_t stride = sstride;
    int nch, chunk;
    xdraw_chunks(nsrc, nch, chunk);     // chunk < 1024 (TreeSum levels below); dcfm_create caps g
    d2 sv[4], ev[4];
    if (w == 0 && d.inject) {   // eps of dc:126 (injected draw buffer), in flight during the sum
        const double *nx = dr.NX + ((size_t)(iter - dr.first_iter) * d.n + (live ? i : 0)) * d.K;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int kk = 8 * t + 2 * q;
            ev[t].x = (live && kk < d.K) ? nx[kk] : 0.0;
            ev[t].y = (live && kk + 1 < d.K) ? nx[kk + 1] : 0.0;
        }
    } else if (w == 0) {        // generated here (SITE_X, row i): Philox pair 4t + q
        const Rng rng(d.seed);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int kk = 8 * t + 2 * q;
            double n0 = 0.0, n1 = 0.0;
            if (live && kk < d.K) rng.normal2(SITE_X, 0u, (uint32_t)i, (uint32_t)(4 * t + q), (uint32_t)iter, n0, n1);
            ev[t].x = n0;
            ev[t].y = (kk + 1 < d.K) ? n1 : 0.0;
        }
    }
    // one rank: the operators are already out (k_wcol's last arrival): their loads go out before
    // the sums' (two per thread), the LDS stores after
    double xmv[2] = {0.0, 0.0};
    if (!(xroles & 1)) {
#pragma unroll
        for (int u = 0; u < 2; ++u) xmv[u] = XM[threadIdx.x + 1024 * u];
    }
    if (sw < nch) {
        if (chunk >= 2) {   // lane c sums part c / XD_ROWS (a canonical subtree) of the chunk for row c % XD_ROWS
            // the parts split only a power-of-two chunk (np | chunk, each part a canonical
            // subtree); a chunk of any other size (xdraw_chunks: nch = 1, chunk = nsrc, e.g.
            // g = 5 or 10 shards) is summed whole by the h == 0 lanes
            constexpr int NPART = 16 / XD_ROWS;
            const int np = (chunk & (chunk - 1)) ? 1 : (chunk < NPART ? chunk : NPART), per = chunk / np;
            const int rr = c % XD_ROWS, h = c / XD_ROWS;
            const bool rl = i0 + rr < d.n && h < np;
            const double *p = src + (size_t)(sw * chunk + (h < np ? h : 0) * per) * stride +
                              (size_t)(i0 + rr < d.n ? i0 + rr : i0) * KP + 8 * tw + 2 * q;
            d2 v = rl ? tree_sum_f<d2, 8, 10>(per, [&](int rk) { return *reinterpret_cast<const d2 *>(p + (size_t)rk * stride); })
                      : d2{0.0, 0.0};
            for (int o = 1; o < np; o <<= 1) {   // adjacent parts pairwise: the canonical tree over the parts
                d2 u;
                u.x = __shfl_down(v.x, o * XD_ROWS, 16);
                u.y = __shfl_down(v.y, o * XD_ROWS, 16);
                v.x = v.x + u.x;
                v.y = v.y + u.y;
            }
            part[sw][tw][lane] = h == 0 ? v : d2{0.0, 0.0};
        } else {
            const double *p = src + (size_t)sw * chunk * stride + (size_t)(live ? i : i0) * KP + 8 * tw + 2 * q;
            part[sw][tw][lane] = live ? *reinterpret_cast<const d2 *>(p) : d2{0.0, 0.0};
        }
    }
    if (xroles & 1) {
        wait_count(xm_ctr, xm_target);       // XM of this launch's block 0
#pragma unroll
        for (int u = 0; u < 2; ++u) xmv[u] = ld_agent(XM + threadIdx.x + 1024 * u);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = threadIdx.x + 1024 * u;
        const int mat = e / (KP * KP), rem = e % (KP * KP);
        Ms[mat][rem / KP][rem % KP] = xmv[u];
    }
    __syncthreads();
    if (w > 0) return;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        TreeSum<d2, 3> ts;
        for (int k = 0; k < nch; ++k) ts.push(part[k][t][lane]);
        sv[t] = ts.total();
    }
    d4 ax[2];
    ax[0] = ax[1] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int kk = 8 * t + 2 * q + e;
            const double se = e ? sv[t].y : sv[t].x, ee = e ? ev[t].y : ev[t].x;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                ax[mt] = mfma16x16x4(Ms[0][16 * mt + c][kk], se, ax[mt]);
                ax[mt] = mfma16x16x4(Ms[1][16 * mt + c][kk], ee, ax[mt]);
            }
        }
    if (!live) return;
    double *Xr = X + (size_t)i * KP;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int k = 16 * mt + q + 4 * g;
            Xr[k] = (k < d.K) ? ax[mt][g] : 0.0;
        }
}

// ============================================================================
// k_cpass: [C_m | E_m] = [Y_m | eta_m]' eta_m    fp64 MFMA, Y pass 2      dc:133,138,141
// block = (shard m, 32-column tile of [Y | eta]) x (32-column tile kt of eta, the
// fastest index of the 1-D grid); its CP_WAVES waves split the reduction over rows i, partial
// 32x32 tiles summed in LDS in a fixed order (the canonical tree).  The wave count fixes the
// summation order, so it cannot follow the shard count per rank (N ranks reproduce one rank's
// bits); 8 waves measured g = 8 share 18.2 -> 16.8 us but c3 45.5 -> 49.8 us: 4 it is.
// Lane (r, q) loads 16 B: Y[i][c0+2r .. +1] and eta[i][2r .. +1] (formed on the
// fly from X and Z), i = 4s + q, so the MFMA tiles are even/odd columns x
// even/odd k.  Register double-buffered prefetch, 4 k-steps per batch (a ring of 3: same
// time at c3 and c4, 180 VGPRs).
// ============================================================================
// IS_E: the A operand is eta itself, columns te*32.. (Yp = nullptr; Xa/Za point at
// them); SAME_T: te == kt, so the A operand is the B operand (no extra loads).
// PS: the block computes only the k columns of parity par (acc[.][0]); same per-element order
// ETA (wide): Xp / Xa point at eta itself (formed once per iteration by k_eta into the free W buffer,
// with the same eta_of), Zp / Za unused: one load per operand instead of two
template <int KW, bool IS_E, bool SAME_T, bool PS = false, bool ETA = false>
__device__ __forceinline__ void cpass_wave(const Dims &d, const double *__restrict__ Yp,
                                           const double *__restrict__ Xp,
                                           const double *__restrict__ Zp,
                                           const double *__restrict__ Xa,
                                           const double *__restrict__ Za, int s0, int nsw,
                                           int q, d4 (&acc)[2][2], int par = 0) {
    constexpr bool EXTRA = IS_E && !SAME_T;
    d2 yA[4], xA[4], zA[4], yB[4], xB[4], zB[4];
    auto load = [&](int s, d2 (&y)[4], d2 (&x)[4], d2 (&z)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = 4 * (s + u) + q;
            x[u] = *reinterpret_cast<const d2 *>(Xp + (size_t)i * KW);
            if (!ETA) z[u] = *reinterpret_cast<const d2 *>(Zp + (size_t)i * KW);
            if (!IS_E) {
                y[u] = *reinterpret_cast<const d2 *>(Yp + (size_t)i * d.PP);
            } else if (EXTRA) {   // eta of tile te, formed into y
                const d2 xa = *reinterpret_cast<const d2 *>(Xa + (size_t)i * KW);
                if (ETA) {
                    y[u] = xa;
                } else {
                    const d2 za = *reinterpret_cast<const d2 *>(Za + (size_t)i * KW);
                    y[u].x = eta_of(d.sr, d.s1r, xa.x, za.x);
                    y[u].y = eta_of(d.sr, d.s1r, xa.y, za.y);
                }
            }
        }
    };
    auto mma = [&](d2 (&y)[4], d2 (&x)[4], d2 (&z)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double e0 = ETA ? x[u].x : eta_of(d.sr, d.s1r, x[u].x, z[u].x);
            const double e1 = ETA ? x[u].y : eta_of(d.sr, d.s1r, x[u].y, z[u].y);
            const double a0 = (IS_E && SAME_T) ? e0 : y[u].x, a1 = (IS_E && SAME_T) ? e1 : y[u].y;
            if constexpr (PS) {
                const double ep = par ? e1 : e0;
                acc[0][0] = mfma16x16x4(a0, ep, acc[0][0]);
                acc[1][0] = mfma16x16x4(a1, ep, acc[1][0]);
            } else {
                acc[0][0] = mfma16x16x4(a0, e0, acc[0][0]);
                acc[0][1] = mfma16x16x4(a0, e1, acc[0][1]);
                acc[1][0] = mfma16x16x4(a1, e0, acc[1][0]);
                acc[1][1] = mfma16x16x4(a1, e1, acc[1][1]);
            }
        }
    };
    const int nb = nsw >> 2;
    load(s0, yA, xA, zA);
    for (int b = 0; b < nb; b += 2) {
        if (b + 1 < nb) load(s0 + 4 * (b + 1), yB, xB, zB);
        mma(yA, xA, zA);
        if (b + 2 < nb) load(s0 + 4 * (b + 2), yA, xA, zA);
        if (b + 1 < nb) mma(yB, xB, zB);
    }
}

template <int KW> constexpr int cp_waves() { return 4; }
#ifndef DCFM_WIDE_ETA
#define DCFM_WIDE_ETA 1
#endif
// PS (K <= 32, where the launch would leave CUs idle): each block computes one parity of its
// 32 k columns (twice the blocks, the pair adjacent: Y from L2); per-element order unchanged
// ndel > 0 (fused K <= 32 chain): the last ndel blocks run the previous iteration's delta / tau
// chain (one wave per shard, dc:155-165) beside the pass — it needs only the column sums k_wcol
// (and, several ranks, the packed gather) left, and its ~12 us chain of dependent steps would
// otherwise be the long pole of k_xdraw
// waves_per_eu(3): 164 VGPRs and no AGPRs (without it hipcc took 168 + 32 AGPRs, 2 waves per
// SIMD); measured neutral at c3 and c4 (42.4 vs 42.9 us, 132 vs 135 us), kept for the
// occupancy headroom
template <int KW, bool PS = false>
__global__ __launch_bounds__(64 * cp_waves<KW>()) __attribute__((amdgpu_waves_per_eu(3))) void k_cpass(Dims d, const double *__restrict__ Y,
                                                              const double *__restrict__ X,
                                                              const double *__restrict__ Z,
                                                              double *__restrict__ C, double *__restrict__ E,
                                                              DrawsDev dr, const double *__restrict__ sall,
                                                              DeltaArgs da, int ndel) {
    constexpr int NWV = cp_waves<KW>();
    __shared__ double red[NWV][32][33];
    const int nbc = gridDim.x - ndel;
    if ((int)blockIdx.x >= nbc) {
        const int m = (blockIdx.x - nbc) * NWV + (threadIdx.x >> 6);
        if (m < d.g)
            delta_shard(d, sall, da.delta_in, da.tau_in, da.delta_out, da.tau_out, dr, da.iter, m, threadIdx.x & 63);
        return;
    }
    // 1-D grid, the KW/32 eta column tiles of one [Y | eta] tile adjacent (same XCD,
    // so the Y tile is fetched once and re-read from L2)
    const int nt = (d.PP + KW) >> 5, nkt = KW / 32;
    int w = xcd_remap(blockIdx.x, nbc);
    const int par = PS ? (w & 1) : 0;
    if (PS) w >>= 1;
    const int kt = w % nkt, m = (w / nkt) / nt, tile = (w / nkt) % nt;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c0 = tile * 32;
    const bool isE = c0 >= d.PP;
    const int te = isE ? (c0 - d.PP) >> 5 : 0;
    const int r = lane & 15, q = lane >> 4;
    const double *Yp = Y + (size_t)m * d.NP * d.PP + c0 + 2 * r;
    // wide: X is eta [G][NP][KW] (k_eta, launch_cpass), so the shard's rows
    constexpr bool ETA = KW > KP && DCFM_WIDE_ETA;
    const double *Xs = ETA ? X + (size_t)m * d.NP * KW : X;
    const double *Xp = Xs + 32 * kt + 2 * r;
    const double *Zp = Z + (size_t)m * d.NP * KW + 32 * kt + 2 * r;
    const double *Xa = Xs + 32 * te + 2 * r;
    const double *Za = Z + (size_t)m * d.NP * KW + 32 * te + 2 * r;
    const int nsw = d.NP / (4 * NWV);          // k-steps (4 rows each) per wave
    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    if (!isE) cpass_wave<KW, false, false, PS, ETA>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc, par);
    else if (te == kt) cpass_wave<KW, true, true, PS, ETA>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc, par);
    else cpass_wave<KW, true, false, PS, ETA>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc, par);
    // D row rho = q + 4g -> column c0 + 2 rho + ta;  D col r -> k = 2r + tb
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int rho = q + 4 * g;
#pragma unroll
        for (int ta = 0; ta < 2; ++ta) {
            if (PS) {
                red[wave][2 * rho + ta][2 * r + par] = acc[ta][0][g];
            } else {
#pragma unroll
                for (int tb = 0; tb < 2; ++tb) red[wave][2 * rho + ta][2 * r + tb] = acc[ta][tb][g];
            }
        }
    }
    __syncthreads();
    auto tsum = [&](int a, int b) {
        if constexpr (NWV == 8)
            return ((red[0][a][b] + red[1][a][b]) + (red[2][a][b] + red[3][a][b])) +
                   ((red[4][a][b] + red[5][a][b]) + (red[6][a][b] + red[7][a][b]));
        else
            return (red[0][a][b] + red[1][a][b]) + (red[2][a][b] + red[3][a][b]);
    };
    if (KW > KP && isE) {   // wide: E_m in the loading-row kernel's tile layout (etile_index), upper tiles
        double *Em = E + (size_t)m * KW * KW;
        for (int e = threadIdx.x; e < 32 * 32; e += 64 * NWV) {
            const int a = e >> 5, b = e & 31, R = 32 * te + a, Cc = 32 * kt + b;
            if ((R >> 4) <= (Cc >> 4)) Em[etile_index(KW / 16, R, Cc)] = tsum(a, b);
        }
        return;
    }
    double *out = isE ? (E + (size_t)m * KW * KW + (size_t)(32 * te) * KW + 32 * kt)
                      : (C + ((size_t)m * d.PP + c0) * KW + 32 * kt);
    if (PS) {   // this block's parity of the columns
        for (int e = threadIdx.x; e < 32 * 16; e += 64 * NWV) {
            const int a = e >> 4, b = 2 * (e & 15) + par;
            out[(size_t)a * KW + b] = tsum(a, b);
        }
        return;
    }
    for (int e = threadIdx.x; e < 32 * 32; e += 64 * NWV) {
        const int a = e >> 5, b = e & 31;
        out[(size_t)a * KW + b] = tsum(a, b);
    }
}

// k_lambda (loading rows, dc:140-145,150,156,169-171): lambda.h

// ============================================================================
// k_colsum: sloc[m][k] = sum_{j<P} cpart[m][j][k], fixed order            dc:156 sum(mat)
// block = (shard m, 32 columns); 8 row groups x 4 independent accumulators each.
// ============================================================================
template <int KW, bool PUB = false>
__device__ __forceinline__ void colsum_tile(const Dims &d, const double *__restrict__ cpart,
                                            double *__restrict__ sloc, int m, int kt, double *smem) {
    double (*part)[32] = reinterpret_cast<double (*)[32]>(smem);
    const int k = 32 * kt + (threadIdx.x & 31), grp = threadIdx.x >> 5;
    const double *cp = cpart + (size_t)m * d.PP * KW + k;
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    // rows j = grp + 8 i: every load of a 320-row band in flight at once (one latency round
    // per band instead of one per few rows), summed into 4 accumulators in row order
    constexpr int RB = 40;
    for (int j0 = 0; j0 < d.P; j0 += 8 * RB) {
        double v[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int j = j0 + grp + 8 * i;
            v[i] = j < d.P ? cp[(size_t)j * KW] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) s4[i & 3] += v[i];
    }
    part[grp][threadIdx.x & 31] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    __syncthreads();
    if (threadIdx.x < 32) {
        double tt = 0.0;
#pragma unroll
        for (int g2 = 0; g2 < 8; ++g2) tt += part[g2][threadIdx.x];
        if (PUB) st_agent(sloc + (size_t)m * KW + k, tt);
        else sloc[(size_t)m * KW + k] = tt;
    }
}
template <int KW>
__global__ __launch_bounds__(256) void k_colsum(Dims d, const double *__restrict__ cpart, double *__restrict__ sloc) {
    __shared__ double smem[8 * 32];
    colsum_tile<KW>(d, cpart, sloc, blockIdx.x, blockIdx.y, smem);
}

// ============================================================================
// k_delta: multiplicative-gamma-process chain                      dc:154-165, 174-177
//   K >= 2: every shard's h>=2 step reads shard 1's ALREADY-updated delta_h (Q4);
//           each block re-runs shard 1's chain first (deterministic, identical).
//   K == 1: cumprod over the K x 1 x g array runs along shards (Q5):
//           tau_used(m) = prod_{m'<m} delta_new(m') * delta_old(m).
// The chain over h is scalar: with T_h = sum_{l>=h} tau_l s_l of the incoming
// tau, the reference's recomputed cumprod gives dot_h = F_h T_h where
// F_h = prod_{h'<h} delta_new(h')/delta_old(h')  (exact; rounding-level only).
// grid = all g shards (delta/tau replicated on every rank); local blocks also
// (formerly) refresh Plam — now formed lazily in k_lambda.
// ============================================================================

// lane l < K holds T_l, G_l, 1/delta_old_l and 1/dref_l; returns delta_new_l.
// The chain  bd_h = b_h + (0.5 / dref_h) F_h T_h,  dn_h = G_h / bd_h,  F_{h+1} = F_h dn_h / dold_h
// (F_0 = 1, b_0 = bd1, b_h = bd2) is a linear recurrence in y_h = 1 / F_h:
//   y_{h+1} = alpha_h y_h + beta_h,  alpha_h = b_h dold_h / G_h,  beta_h = (0.5 / dref_h) T_h dold_h / G_h,
// and dn_h = G_h y_h / (b_h y_h + c_h), c_h = (0.5 / dref_h) T_h.  The affine maps compose by a
// wave scan (log2 steps) instead of K dependent steps; every term is positive, so the
// reassociation moves the result by a few ulps only (dc:157-163).
__device__ __forceinline__ double delta_chain(const Dims &d, int l, double T, double G, double idold, double idref) {
    const bool act = l < d.K;
    const double bh = (l == 0) ? d.bd1 : d.bd2;
    const double c = (0.5 * idref) * T;
    const double inv = 1.0 / (idold * G);            // dold_h / G_h
    double A = act ? bh * inv : 1.0, B = act ? c * inv : 0.0;   // identity map on idle lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {                // inclusive scan: (A,B)_l o ... o (A,B)_0
        const double Ap = __shfl_up(A, o, 64), Bp = __shfl_up(B, o, 64);
        if (l >= o) {
            B = fma(A, Bp, B);
            A = A * Ap;
        }
    }
    const double yin = A + B;                         // y_{l+1} (y_0 = 1)
    const double yprev = __shfl_up(yin, 1, 64);
    const double y = (l == 0) ? 1.0 : yprev;          // y_l
    return act ? G * y / fma(bh, y, c) : 1.0;
}

// column sums of global shard mg in the gathered buffer (rank blocks padded by d.sgap)
__device__ __forceinline__ size_t sall_off(const Dims &d, int mg) {
    return (size_t)mg * KP + (d.sgap ? (size_t)(mg / d.G) * d.sgap : 0);
}

// one wave = one global shard m, lane l.  COH: sall was published by other blocks of the
// same launch (k_wcol) and is read with agent-scope loads
template <bool COH>
__device__ __forceinline__ void delta_shard(const Dims &d, const double *__restrict__ sall,
                                            const double *__restrict__ delta_in, const double *__restrict__ tau_in,
                                            double *__restrict__ delta_out, double *__restrict__ tau_out,
                                            const DrawsDev &dr, int64_t iter, int m, int t) {
    if (t < 64) {
        const int l = t;
        const int lk = l < KP ? l : 0;
        const bool act = l < d.K;
        if (d.K >= 2) {
            // shard 1 (index 0) with its own pre-update delta_h
            const double d0 = act ? delta_in[lk] : 1.0;
            const double s0 = act ? (COH ? ld_agent(sall + sall_off(d, 0) + lk) : sall[sall_off(d, 0) + lk]) : 0.0;
            const double T0 = wave_suffix_sum(act ? tau_in[lk] * s0 : 0.0, l);
            const double G0 = act ? delta_G(d, dr, iter, 0, l) : 1.0;
            const double id0 = 1.0 / d0;
            const double d0new = delta_chain(d, l, T0, G0, id0, id0);
            double dm = d0new;
            if (m != 0) {
                const size_t o = (size_t)m * KP + lk;
                const double dold = act ? delta_in[o] : 1.0;
                const double sm = act ? (COH ? ld_agent(sall + sall_off(d, m) + lk) : sall[sall_off(d, m) + lk]) : 0.0;
                const double Tm = wave_suffix_sum(act ? tau_in[o] * sm : 0.0, l);
                const double Gm = act ? delta_G(d, dr, iter, m, l) : 1.0;
                const double idold = 1.0 / dold;
                const double idref = (l == 0) ? idold : 1.0 / d0new;   // delta(1,:,m) | delta(h) (Q4)
                dm = delta_chain(d, l, Tm, Gm, idold, idref);
            }
            const double tm = wave_scan_prod(act ? dm : 1.0, l);         // tauh = cumprod(delta)
            if (l < KP) {
                delta_out[(size_t)m * KP + l] = act ? dm : delta_in[(size_t)m * KP + l];
                tau_out[(size_t)m * KP + l] = act ? tm : tau_in[(size_t)m * KP + l];
            }
        } else {
            if (l == 0) {
                double prefix = 1.0, dnew = 0.0;
                for (int mm = 0; mm <= m; ++mm) {
                    const double dold = delta_in[(size_t)mm * KP];
                    const double tused = prefix * dold;
                    const double smm = COH ? ld_agent(sall + sall_off(d, mm)) : sall[sall_off(d, mm)];
                    const double bd = d.bd1 + (0.5 * (1.0 / dold)) * (tused * smm);
                    dnew = (1.0 / bd) * delta_G(d, dr, iter, mm, 0);
                    prefix = prefix * dnew;
                }
                delta_out[(size_t)m * KP] = dnew;
                tau_out[(size_t)m * KP] = prefix;
            }
            if (l >= 1 && l < KP) {
                delta_out[(size_t)m * KP + l] = delta_in[(size_t)m * KP + l];
                tau_out[(size_t)m * KP + l] = tau_in[(size_t)m * KP + l];
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_delta(Dims d, const double *__restrict__ sall,
                                               const double *__restrict__ delta_in,
                                               const double *__restrict__ tau_in,
                                               double *__restrict__ delta_out,
                                               double *__restrict__ tau_out,
                                               DrawsDev dr,
                                               int64_t iter) {
    delta_shard(d, sall, delta_in, tau_in, delta_out, tau_out, dr, iter, blockIdx.x, threadIdx.x);
}

// ============================================================================
// Fused single-stream launches (K <= 32).  Cross-stream event hand-offs cost ~6 us each
// on the critical path, and latency-bound work slows ~2x when it shares CUs with the
// MFMA-bound Y passes, so the small per-shard K x K work rides in the launches of the
// Y passes (k_wcol, k_xdraw) as extra roles (dcfm_run names the plan).
// ============================================================================
// The chunk sums are handed to the last arrival with agent-scope relaxed atomics (sc1:
// coherent across the XCDs' L2s without write-back / invalidate), ordered by the stores'
// completion before the ticket — __threadfence's buffer_wbl2 / buffer_inv flush the XCD's
// whole L2 and drop what co-resident blocks cache (measured +20 us next to a Y pass).
__device__ __forceinline__ bool last_arrival(unsigned *ticket, unsigned count, double *smem) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this thread's agent-scope stores are done
    __syncthreads();
    unsigned *flag = reinterpret_cast<unsigned *>(smem);
    if (threadIdx.x == 0) {
        const bool last =
            __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == count - 1;
        if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
        *flag = last ? 1u : 0u;
    }
    __syncthreads();
    const bool last = *flag != 0u;
    __syncthreads();
    return last;
}

// ============================================================================
// k_wcol (one rank, K <= 32): the small per-iteration work that feeds the Z / X draws rides
// in the Y pass's launch.  As separate launches these latency-bound pieces (K x K
// factorisations, shard sums, column sums) cost ~25 us per iteration on the critical path;
// inside k_wpass's launch they run beside the pass.  Roles, in block order (a consumer's
// producers always have lower block ids, so they are dispatched first and a spinning
// consumer can never hold back its producer):
//   OPS    [0, G)      prep_shard(m): A_m (published agent-coherent) and the Z operators ZM_m
//                      of THIS iteration (from the incoming Lambda, omega)           dc:98-107
//   COLSUM [.., +G)    column sums of the PREVIOUS iteration's psi o Lambda^2 (dc:156) for
//                      the delta chain, which runs in the next launch (k_xdraw)
//   OPS    [.., +nxs)  wait for every A_m; chunk j's tree sum (a canonical subtree) -> xpart;
//                      the last arrival sums the chunks (canonical tree) into xa (dc:117);
//                      (several ranks: k_xdraw's block 0 factors Xprec from the ranks' sums) dc:112-118
//   WPASS  [.., +nw)   W_m = Y_m (w o Lambda_m) tiles, each drawing Z for its rows and writing
//                      the shard's X message (wpass_z_tile)       dc:101-107,121-123
//   LAMGEN [.., +nlg)  the generated chain's loading-row variates of this iteration for the
//                      k_lambda that follows (lam_draws; VALU work in the slots and issue
//                      cycles the streaming W tiles leave free)      dc:142,150,170
// Hand-off: payload by agent-scope stores, s_waitcnt vmcnt(0), then a relaxed fetch-add on a
// monotonic 64-bit counter; consumers poll it (s_sleep) up to the launch's target and read
// the payload with agent-scope loads.
// ============================================================================
// ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7)): the canonical tree of 8 (TreeSum), and of
// any power-of-two n <= 8 when v[n..8) are zero (x + 0 = x)
__device__ __forceinline__ double tree8(const double (&v)[8]) {
    return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}

// k_wcol's W pass with the Z draw of its rows (fused chain, K <= 32; dc:101-107,121-123): the
// wave's W' tile stays in the accumulators (wpass_acc) and feeds zdraw_rows directly — no W
// round trip through HBM and no k_zdraw launch.  The rows' normals are drawn while the first Y
// chunks are in flight; the shard's operators come from its OPS block of the same launch
// (agent-scope stores, counter SYNC_ZM + m, epoch = the launch's ops epoch), staged once per
// block in LDS after the pass.
template <int MT>
__device__ __forceinline__ void wpass_z_tile(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, int w,
                                             unsigned long long zm_epoch, double *smem) {
    double (*Ms)[KP][KP + 1] = reinterpret_cast<double (*)[KP][KP + 1]>(smem);   // M1, M2, U, NA
    const int nrb = d.NP / (64 * MT);
    const int m = w / nrb, rb = w % nrb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, q = lane >> 4;
    const int mg = d.shard0 + m;
    const int i0 = rb * 64 * MT + wave * 16 * MT;
    d4 acc[MT][2];
    wpass_acc<KP, MT>(d, b.Y, b.Lam, b.omega, m, i0, 0, acc, [] {});
    WSTAMP(2);
    // the operators are normally out long before the pass ends; their loads and the rows' X are
    // issued first, the first tile's normals drawn while they are in flight
    wait_count(b.sync + SYNC_ZM + m, zm_epoch);
    WSTAMP(3);
    constexpr int NU = 4 * KP * KP / 256;
    double zv[NU];
    {
        const double *Zm = b.ZM + (size_t)m * 4 * KP * KP;
#pragma unroll
        for (int u = 0; u < NU; ++u) zv[u] = ld_agent(Zm + threadIdx.x + 256 * u);
    }
    // each tile's X rows after its normals (tile 0's during the operators' staging, tile 1's at its
    // own draw): held across the normals and tile 0's draw they spilled (12 VGPRs at waves_per_eu(3))
    d2 xv[MT][4], ev[MT][4];
    auto load_x = [&](int a) {
        const double *Xi = b.X + (size_t)(i0 + 16 * a + c) * KP + 2 * q;
#pragma unroll
        for (int t = 0; t < 4; ++t) xv[a][t] = *reinterpret_cast<const d2 *>(Xi + 8 * t);
    };
    z_eps(d, dr, iter, mg, i0 + c, i0 + c < d.n, q, ev[0]);   // tile 1's after tile 0's draw (registers)
    load_x(0);                                                  // in flight during the operators' staging
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int e = threadIdx.x + 256 * u;
        const int mat = e / (KP * KP), rem = e % (KP * KP);
        Ms[mat][rem / KP][rem % KP] = zv[u];
    }
    __syncthreads();
    WSTAMP(4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int a = 0; a < MT; ++a) {
        const int i = i0 + 16 * a + c;
        if (a > 0) {
            load_x(a);
            z_eps(d, dr, iter, mg, i, i < d.n, q, ev[a]);
        }
        d2 wv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            wv[g].x = acc[a][0][g];
            wv[g].y = acc[a][1][g];
        }
        zdraw_rows(d, Ms, wv, xv[a], ev[a], b.Z + ((size_t)m * d.NP + i) * KP, b.Sp + ((size_t)m * d.NP + i) * KP,
                   i < d.n, c, q);
        if (a == 0) WSTAMP(5);
        __builtin_amdgcn_sched_barrier(0);   // one tile's draw at a time (registers)
    }
}

__device__ __forceinline__ void wcol_body(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, int ops, int colsum,
                                          int wpass, unsigned long long ops_epoch, int xchol, const LamGen &lg,
                                          double *smem);
#ifndef DCFM_WCOL_WPE
#define DCFM_WCOL_WPE 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DCFM_WCOL_WPE))) void k_wcol(Dims d, Bufs b, DrawsDev dr, int64_t iter, int ops, int colsum,
                                              int wpass, unsigned long long ops_epoch, int xchol, LamGen lg) {
    __shared__ double smem[PREP_SMEM];
#ifdef DCFM_WSTAMPS
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_readcyclecounter();
#endif
    wcol_body(d, b, dr, iter, ops, colsum, wpass, ops_epoch, xchol, lg, smem);
#ifdef DCFM_WSTAMPS
    if (wpass && threadIdx.x == 0 && blockIdx.x < 8192) {
        g_wstamps[blockIdx.x][0] = t0;
        g_wstamps[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
        g_wstamps[blockIdx.x][6] = c0;                                 // shader clock: the block's mean frequency
        g_wstamps[blockIdx.x][7] = __builtin_readcyclecounter();
    }
#endif
}
__device__ __forceinline__ void wcol_body(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, int ops, int colsum,
                                          int wpass, unsigned long long ops_epoch, int xchol, const LamGen &lg,
                                          double *smem) {
    const int G = d.G, nxs = xsum_blocks(G), chunk = G / nxs;
    unsigned long long *chunk_ctr = b.sync + 2;   // per chunk of shards: A_m published
    int blk = blockIdx.x;
    if (ops) {
        if (blk < G) {
            prep_gram<true>(d, b.Lam, b.omega, b.A, b.ZM, blk, smem);
            WSTAMP(2);
            signal_count(chunk_ctr + blk / chunk);   // A_m is out; the operators follow
            prep_ops<true>(d, b.ZM, blk, smem);
            signal_count(b.sync + SYNC_ZM + blk);    // the Z operators are out (the W tiles draw Z)
            return;
        }
        blk -= G;
    }
    if (colsum) {
        if (blk < G) {
            colsum_tile<KP>(d, b.cpart, b.sloc, blk, 0, smem);
            return;
        }
        blk -= G;
    }
    if (ops) {
        if (blk < nxs) {   // chunk j of the shard sum of A, then (last arrival) Xprec and its factors
            const int t = threadIdx.x, j = blk, m0 = j * chunk;   // chunk: a canonical subtree
            constexpr int NU = KP * KP / 256;
            wait_count(chunk_ctr + j, ops_epoch * (unsigned long long)chunk);
            double vs[NU];
            if (chunk <= 8) {                                      // one round: the whole chunk
                double v[NU][8];
#pragma unroll
                for (int u = 0; u < NU; ++u)
#pragma unroll
                    for (int U = 0; U < 8; ++U)
                        v[u][U] = (U < chunk) ? ld_agent(b.A + (size_t)(m0 + U) * KP * KP + t + 256 * u) : 0.0;
#pragma unroll
                for (int u = 0; u < NU; ++u) vs[u] = tree8(v[u]);   // chunk a power of two, or G <= 8
            } else {                                               // groups of 8 (subtrees), then their tree
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    TreeSum<double, 6> ts;
                    for (int k = 0; k < chunk; k += 8) {
                        double v[8];
#pragma unroll
                        for (int U = 0; U < 8; ++U) v[U] = ld_agent(b.A + (size_t)(m0 + k + U) * KP * KP + t + 256 * u);
                        ts.push(tree8(v));
                    }
                    vs[u] = ts.total();
                }
            }
            if (nxs > 1) {   // several chunks: publish, the last arrival goes on
#pragma unroll
                for (int u = 0; u < NU; ++u) st_agent(b.xpart + (size_t)j * KP * KP + t + 256 * u, vs[u]);
                if (!last_arrival(b.ticket, (unsigned)nxs, smem)) return;
            }
            double xs[NU];
            if (nxs <= 8) {   // canonical tree over the chunk sums: every load in flight at once
                              // (a round trip per u cost ~1.3 us each); tree8 with zeros past nxs
                              // is TreeSum's order for any nxs <= 8
                double v[NU][8];
#pragma unroll
                for (int u = 0; u < NU; ++u)
#pragma unroll
                    for (int U = 0; U < 8; ++U)
                        v[u][U] = (U < nxs) ? (U == j ? vs[u] : ld_agent(b.xpart + (size_t)U * KP * KP + t + 256 * u))
                                            : 0.0;
#pragma unroll
                for (int u = 0; u < NU; ++u) xs[u] = tree8(v[u]);
            } else {   // a non-power-of-two G: the chunks are single shards and nxs = G exceeds
                       // 8: groups of 8 into a TreeSum
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    TreeSum<double, 8> ts;
                    for (int k = 0; k < nxs; k += 8) {
                        double v[8];
#pragma unroll
                        for (int U = 0; U < 8; ++U)
                            v[U] = (k + U < nxs) ? (k + U == j ? vs[u] : ld_agent(b.xpart + (size_t)(k + U) * KP * KP + t + 256 * u))
                                                 : 0.0;
                        static_for<8>([&](auto U) { if (k + U < nxs) ts.push(v[U]); });
                    }
                    xs[u] = ts.total();
                }
            }
            if (!xchol) {   // several ranks: the local sum into the packed message (all-gathered next)
#pragma unroll
                for (int u = 0; u < NU; ++u) b.xa[t + 256 * u] = xs[u];
                return;
            }
            __syncthreads();                          // smem (last_arrival's flag) is reused below
#pragma unroll
            for (int u = 0; u < NU; ++u) xprec_store(d, smem, t + 256 * u, xs[u]);
            __syncthreads();
            xchol_factor(d, b.XM, smem);              // Xprec = g I + rho sum A (dc:117), Rx (dc:118)
            return;
        }
        blk -= nxs;
    }
    if (wpass) {   // 1: 128-row blocks, 2: 64-row blocks (wcol_wpass_mode); W' -> the Z draw
        const int nw = (d.NP / (64 * (3 - wpass))) * d.G;
        if (blk < nw) {
            if (wpass == 2) wpass_z_tile<1>(d, b, dr, iter, xcd_remap(blk, nw), ops_epoch, smem);
            else wpass_z_tile<2>(d, b, dr, iter, xcd_remap(blk, nw), ops_epoch, smem);
            return;
        }
        blk -= nw;
    }
    // the loading-row variates of this iteration (generated chain), behind every other role
#ifdef DCFM_DEV_NO_LAMGEN   // timing-only dev build: the variates of iterations > 3 are not drawn (stale, finite)
    if (iter > 3) return;
#endif
    if (blk < lg.b_total) lam_draws(d, lg, iter, blk * LAM_GEN_THREADS + (int)threadIdx.x, lg.b_total * LAM_GEN_THREADS);
}

// ============================================================================
// saved samples: Lb[(mg*P + j)][slot*K + k] = Lambda, wsum += omega         dc:180-186
// ============================================================================
__global__ __launch_bounds__(256) void k_save(Dims d, const double *__restrict__ Lam,
                                              const double *__restrict__ omega,
                                              double *__restrict__ Lb, double *__restrict__ wsum,
                                              int LDB, int slot) {
    const size_t total = (size_t)d.G * d.P * d.K;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
         e += (size_t)gridDim.x * blockDim.x) {
        const int k = e % d.K;
        const size_t jm = e / d.K;
        const int j = jm % d.P, m = jm / d.P;
        const size_t a = (size_t)(d.shard0 + m) * d.P + j;
        Lb[a * LDB + (size_t)slot * d.K + k] = Lam[((size_t)m * d.PP + j) * d.kp + k];
        if (k == 0) wsum[a] += omega[(size_t)m * d.PP + j];
    }
}

// ============================================================================
// k_assemble: Sigma[a][b] += (coef(a,b)/effsamp) sum_kk Lb[a][kk] Lb[b][kk]
//                            + [a==b] wsum[a]/effsamp                       dc:184-195
// coef = 1 inside a diagonal shard block (Lambda_r Lambda_r' + Omega_r), rho
// across blocks (rho Lambda_r Lambda_c').  Lower-triangle 128x128 tiles only, in
// 8 x 8-tile supertiles (dcfm_create), XCD-contiguous (xcd_remap): the tiles an XCD
// has in flight share 8 row and 8 column panels of Lb in its L2.  The tile's place
// in the rank's packed Sigma block comes from (ti, tj).
// Cross-shard tiles (no row and column of the same shard: coef = rho everywhere, ~95% of
// the tiles at c3) start their accumulators FROM the old Sigma values, loaded with the
// first panel chunk, and stage the row panel scaled by rho / effsamp: the epilogue is
// plain stores, so the read half of the read-modify-write never waits at the end of the
// tile.  Tiles with same-shard pairs (and the diagonal) keep the epilogue update.  Sigma is
// streamed with nontemporal loads / stores (read and written once per flush): it no longer
// evicts the Lb panels the XCD's co-resident tiles share from L2 (driver flush 1,176 -> 1,137 us;
// a second register set prefetching the panels two chunks ahead measured no gain).
// 4 waves in 2x2, each 64x64 = 4x4 tiles of v_mfma_f64_16x16x4.  The k extent
// (batch x K) runs in chunks of 16 through double-buffered LDS, stored k-major
// with a 144-double pitch: an MFMA operand read (16 consecutive rows x 4 k) is a
// conflict-free ds_read_b64, and the next chunk's global loads are in flight
// during the current chunk's 64 MFMAs per wave.  One barrier per chunk.
// ============================================================================
constexpr int AKC = ASM_KC, ALD = ASM_TILE + 16, ASM_THREADS = 256;

__device__ __forceinline__ void assemble_tile(const Dims &d, const double *__restrict__ Lb, int LDB, int kext,
                                              const double *__restrict__ wsum, double inv_eff, int2 T, int T0,
                                              double *__restrict__ Sig, double (*As)[AKC][ALD],
                                              double (*Bs)[AKC][ALD], int (*shard_of)[ASM_TILE]) {
    double *__restrict__ St = Sig + (size_t)(tri(T.x) - tri(T0) + T.y) * ASM_TILE * ASM_TILE;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    shard_of[t >> 7][t & 127] = ((t < ASM_TILE ? T.x : T.y) * ASM_TILE + (t & 127)) / d.P;
    const int r = lane & 15, q = lane >> 4;
    const int p = d.p;
    const int wa = (wave >> 1) * 64, wb = (wave & 1) * 64;
    // cross-shard tile: the rows' shards all lie below the columns' (tj < ti, rows >= columns)
    const int clast = min(p, T.y * ASM_TILE + ASM_TILE) - 1;
    const bool cross = (T.x * ASM_TILE) / d.P > clast / d.P;
    const double sA = cross ? d.rho * inv_eff : 1.0;     // row-panel scale while staging
    // global -> LDS: thread t stages row (t >> 1) of both panels, k = 8 (t & 1) .. +7
    const int srow = t >> 1, shalf = t & 1;
    const int ga = T.x * ASM_TILE + srow, gb = T.y * ASM_TILE + srow;
    const bool va = ga < p, vb = gb < p;
    const double *pa = Lb + (size_t)(va ? ga : 0) * LDB + 8 * shalf;
    const double *pb = Lb + (size_t)(vb ? gb : 0) * LDB + 8 * shalf;
    const d2 zero2 = {0.0, 0.0};
    d2 ra[4], rb[4];
    auto gload = [&](int kc) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ra[i] = va ? *reinterpret_cast<const d2 *>(pa + kc + 2 * i) : zero2;
            rb[i] = vb ? *reinterpret_cast<const d2 *>(pb + kc + 2 * i) : zero2;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = 8 * shalf + 2 * i;
            As[buf][k][srow] = sA * ra[i].x;
            As[buf][k + 1][srow] = sA * ra[i].y;
            Bs[buf][k][srow] = rb[i].x;
            Bs[buf][k + 1][srow] = rb[i].y;
        }
    };
    gload(0);      // ahead of the tile's Sigma loads: staging chunk 0 waits only for its panels
    d4 acc[4][4];
    // the tile's values of this wave's accumulators: slice (u, v, h) = 64 lanes x 16 B, contiguous
    auto sl = [&](int u, int v, int h) { return reinterpret_cast<d2 *>(St + sig_tile_off(u, v, 2 * h, wave, lane)); };
    if (cross) {   // acc = the tile's old values (C/D layout: row q + 4g of 16-row tile u)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const d2 o = __builtin_nontemporal_load(sl(u, v, h));
                    acc[u][v][2 * h] = o.x;
                    acc[u][v][2 * h + 1] = o.y;
                }
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[u][v] = d4{0.0, 0.0, 0.0, 0.0};
    }
    lstore(0);
    __syncthreads();
    for (int kc = 0, buf = 0; kc < kext; kc += AKC, buf ^= 1) {
        const bool more = kc + AKC < kext;
        if (more) gload(kc + AKC);
        const int nk4 = min(AKC, kext - kc);   // k extent of this chunk (a multiple of 4)
#pragma unroll
        for (int s4 = 0; s4 < AKC / 4; ++s4) {
            if (4 * s4 >= nk4) break;            // block-uniform: the last chunk may be partial
            double a[4], b[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = As[buf][4 * s4 + q][wa + 16 * u + r];
#pragma unroll
            for (int v = 0; v < 4; ++v) b[v] = Bs[buf][4 * s4 + q][wb + 16 * v + r];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] = mfma16x16x4(a[u], b[v], acc[u][v]);
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
    }
    if (cross) {   // acc = old + (rho / effsamp) L_a L_b': plain stores (the whole tile is below the diagonal)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    d2 o;
                    o.x = acc[u][v][2 * h];
                    o.y = acc[u][v][2 * h + 1];
                    __builtin_nontemporal_store(o, sl(u, v, h));
                }
        return;
    }
    // epilogue: lower-triangle read-modify-write of the tile (tile-packed, accumulator order inside),
    // loads issued together (predicated, no branches around them), shard test from the LDS table
    const int a0 = T.x * ASM_TILE + wa, b0 = T.y * ASM_TILE + wb;
    int sb[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) sb[v] = shard_of[1][wb + 16 * v + r];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        double old[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int a = a0 + 16 * u + q + 4 * g;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int b = b0 + 16 * v + r;
                const bool live = a < p && b <= a;
                old[g][v] = live ? __builtin_nontemporal_load(&St[sig_tile_off(u, v, g, wave, lane)]) : 0.0;
            }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int a = a0 + 16 * u + q + 4 * g;
            const int sa = shard_of[0][wa + 16 * u + q + 4 * g];
            const double dg = (a < p) ? wsum[a] * inv_eff : 0.0;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int b = b0 + 16 * v + r;
                if (a < p && b <= a) {
                    const double coef = (sb[v] == sa) ? 1.0 : d.rho;
                    double val = coef * acc[u][v][g] * inv_eff;
                    if (a == b) val += dg;
                    __builtin_nontemporal_store(old[g][v] + val, &St[sig_tile_off(u, v, g, wave, lane)]);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256, 2) void k_assemble(Dims d, const double *__restrict__ Lb, int LDB,
                                                     int kext, const double *__restrict__ wsum,
                                                     double inv_eff, const int2 *__restrict__ tiles, int T0,
                                                     double *__restrict__ Sig) {
    __shared__ double As[2][AKC][ALD], Bs[2][AKC][ALD];
    __shared__ int shard_of[2][ASM_TILE];      // shard of the tile's rows / columns (epilogue coef)
    assemble_tile(d, Lb, LDB, kext, wsum, inv_eff, tiles[xcd_remap(blockIdx.x, gridDim.x)], T0, Sig, As, Bs,
                  shard_of);
}

// Column stripe [c0, c0 + nc) of the symmetric Sigmaout from this rank's tile-packed block
// of the lower triangle (tile rows [T0, T1), rows [R0, R1)), written as the rank's packed
// windows: column c holds rows [win_lo(c), R1) at out + win_off(c) (dc:194-195 output, Q9:
// the symmetrisation is this mirror).  One rank owns everything: the windows are then the
// dense p x nc column-major stripe.  32x32 tiles: Sigma(r, c) = S(r, c) for r >= c (read
// along c, transposed through LDS), S(c, r) for r < c (read along r).
__global__ __launch_bounds__(256) void k_sigma_pack(const double *__restrict__ S, int p, int T0, int T1, int c0,
                                                    int nc, double *__restrict__ out) {
    __shared__ double lo[32][33];
    const int R0 = min(p, T0 * ASM_TILE), R1 = min(p, T1 * ASM_TILE);
    const int r0 = blockIdx.x * 32, cb = c0 + blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const bool need_lo = r0 + 31 >= cb;            // some r >= c in the tile
    const bool need_up = r0 < cb + 31;             // some r < c
    if (need_lo) {
        for (int yy = ty; yy < 32; yy += 8) {      // rows r = r0 + yy, columns c = cb + tx
            const int r = r0 + yy, c = cb + tx;
            lo[yy][tx] = (r >= R0 && r < R1 && c < c0 + nc && r >= c) ? S[sig_off(r, c, T0)] : 0.0;
        }
    }
    __syncthreads();
    for (int yy = ty; yy < 32; yy += 8) {          // output column c = cb + yy, rows r = r0 + tx
        const int c = cb + yy, r = r0 + tx;
        if (c >= c0 + nc || r >= R1) continue;
        const long long wl = win_lo(c, R0, R1);
        if (r < wl) continue;
        const double v = (r >= c) ? lo[tx][yy] : (need_up ? S[sig_off(c, r, T0)] : 0.0);
        out[win_off(c, c0, R0, R1) + (r - wl)] = v;
    }
}

// Root of the striped gather: out (dense p x nc, column-major) from the ranks' packed
// windows.  Element (r, c) lives on the owner of tile row max(r, c) / 128.
__global__ __launch_bounds__(256) void k_sigma_unpack(const double *__restrict__ recv, int p, int c0, int cbeg,
                                                      const int *__restrict__ Tb,
                                                      const long long *__restrict__ base, int nranks,
                                                      double *__restrict__ out) {
    const int c = cbeg + blockIdx.y;
    for (int r = blockIdx.x * 256 + threadIdx.x; r < p; r += gridDim.x * 256) {
        const int t = max(r, c) / ASM_TILE;
        int k = 0;
        while (k + 1 < nranks && Tb[k + 1] <= t) ++k;
        const long long R0 = min(p, Tb[k] * ASM_TILE), R1 = min(p, Tb[k + 1] * ASM_TILE);
        out[(size_t)(c - c0) * p + r] = recv[base[k] + win_off(c, c0, R0, R1) + (r - win_lo(c, R0, R1))];
    }
}

__global__ __launch_bounds__(256) void k_eta(Dims d, const double *__restrict__ X,
                                             const double *__restrict__ Z, double *__restrict__ eta) {
    const size_t total = (size_t)d.G * d.NP * d.kp;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
         e += (size_t)gridDim.x * blockDim.x) {
        const size_t ik = e % ((size_t)d.NP * d.kp);
        eta[e] = eta_of(d.sr, d.s1r, X[ik], Z[e]);
    }
}

template <bool GAMMAS>
__global__ __launch_bounds__(256) void k_draws(Dims d, DrawsDev dr, int64_t iter) {
    const DrawPlan pl = draw_plan(d);
    draws_block<GAMMAS>(d, dr, iter, pl, blockIdx.x + (GAMMAS ? 0 : pl.b_gpsi));
}

// variate e at counter (site, shard, row = e / width, index = e % width, iter)
__global__ __launch_bounds__(256) void k_rng_fill(uint64_t seed, int kind, double shape, int site,
                                                  int shard, int64_t iter, int64_t count, int width,
                                                  double *__restrict__ out) {
    const Rng rng(seed);
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < count;
         e += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t row = (uint32_t)(e / width), k = (uint32_t)(e % width);
        out[e] = kind == 0 ? rng.normal(site, shard, row, k, (uint32_t)iter)
                           : rng.gamma(shape, site, shard, row, k, (uint32_t)iter);
    }
}

// ============================================================================
// launchers
// ============================================================================
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// kp == 32: the register-blocked narrow kernels of this file; kp = 64 / 128: the
// wide kernels of kernels_wide.hip (wide::).  Layout-generic kernels are templated.
void launch_prep(const Dims &d, const Bufs &b, hipStream_t s) {
    if (d.kp != KP) return wide::launch_prep(d, b, s);
    hipLaunchKernelGGL(k_prep, dim3(d.G), dim3(256), 0, s, d, b.Lam, b.omega, b.A, b.ZM);
}
void launch_wpass(const Dims &d, const Bufs &b, hipStream_t s) {
    const dim3 grid((d.NP / 128) * d.G * (d.kp / 32));
    switch (d.kp) {
    case 32: hipLaunchKernelGGL(k_wpass<32>, grid, dim3(256), 0, s, d, b.Y, b.Lam, b.omega, b.W); break;
    case 64: hipLaunchKernelGGL(k_wpass<64>, grid, dim3(256), 0, s, d, b.Y, b.Lam, b.omega, b.W); break;
    default: hipLaunchKernelGGL(k_wpass<128>, grid, dim3(256), 0, s, d, b.Y, b.Lam, b.omega, b.W); break;
    }
}
void launch_zdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    if (d.kp != KP) return wide::launch_zdraw(d, b, dr, iter, s);
    if ((d.NP / ZROWS) * d.G < 256)   // 64-row blocks (zdraw_tile)
        hipLaunchKernelGGL(k_zdraw<256>, dim3((d.NP / 64) * d.G), dim3(256), 0, s, d, b.W, b.ZM, b.X, b.Z, b.Sp, dr, iter);
    else
        hipLaunchKernelGGL(k_zdraw<ZTHREADS>, dim3((d.NP / ZROWS) * d.G), dim3(ZTHREADS), 0, s, d, b.W, b.ZM, b.X, b.Z,
                           b.Sp, dr, iter);
}
// k_wcol launch (K <= 32)
void launch_wcol(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, bool ops, bool colsum, bool wpass,
                 unsigned long long ops_epoch, hipStream_t s, bool lamgen) {
    static_assert(LAM_GEN_THREADS == 256, "k_wcol blocks are 256 threads");
    LamGen lg = {};
    if (lamgen && b.ldraw) lg = lam_gen_plan(d, b.ldraw);
    // W pass tiles: 64-row blocks up to one 128-row block per CU (the g = 32 share of c3: 256
    // blocks; 64-row ones measured 2.8 % faster there, 128-row ones faster at c3's 512)
#ifdef DCFM_WCOL_WMODE
    const int wmode = DCFM_WCOL_WMODE;   // dev A/B: forced block height
#else
    const int wmode = (d.NP / 128) * d.G <= 256 ? 2 : 1;
#endif
    const int nb = (ops ? d.G + xsum_blocks(d.G) : 0) + (colsum ? d.G : 0) + (wpass ? (d.NP / (64 * (3 - wmode))) * d.G : 0);
    if (nb + lg.b_total == 0) return;
    hipLaunchKernelGGL(k_wcol, dim3(nb + lg.b_total), dim3(256), 0, s, d, b, dr, iter, ops ? 1 : 0, colsum ? 1 : 0,
                       wpass ? wmode : 0, ops_epoch, d.coll ? 0 : 1, lg);
}
void launch_xred(const Dims &d, const Bufs &b, hipStream_t s) {
    const int total = d.NP * d.kp;
    hipLaunchKernelGGL(k_xred, dim3(cdiv(total, 256)), dim3(256), 0, s, d, b.Sp, b.xin);
}
void launch_asum(const Dims &d, const Bufs &b, hipStream_t s) {
    hipLaunchKernelGGL(k_asum, dim3(cdiv(d.kp * d.kp, 256)), dim3(256), 0, s, d, b.A, b.xa);
}
void launch_xchol(const Dims &d, const Bufs &b, hipStream_t s) {
    if (d.kp != KP) return wide::launch_xchol(d, b, s);
    hipLaunchKernelGGL(k_xchol, dim3(1), dim3(256), 0, s, d, d.coll ? b.xa_all : b.xa, b.XM);
}
void launch_xdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s,
                  bool from_shards) {
    if (d.kp != KP) return wide::launch_xdraw(d, b, dr, iter, s);
    const dim3 grid(cdiv(d.n, XD_ROWS));
    const size_t st = (size_t)d.NP * KP;
    if (from_shards)   // one rank: sum the G shard messages here (no k_xred)
        hipLaunchKernelGGL(k_xdraw, grid, dim3(1024), 0, s, d, b.Sp, d.G, st, b.XM, b.X, dr, iter, 0, nullptr, nullptr,
                           0ull);
    else
        hipLaunchKernelGGL(k_xdraw, grid, dim3(1024), 0, s, d, b.xall, d.nranks, st, b.XM, b.X, dr, iter, 0, nullptr,
                           nullptr, 0ull);
}
void launch_xdraw_mr(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, unsigned long long xm_epoch,
                     hipStream_t s) {
    hipLaunchKernelGGL(k_xdraw, dim3(1 + cdiv(d.n, XD_ROWS)), dim3(1024), 0, s, d, b.xall, d.nranks, (size_t)d.xstride,
                       b.XM, b.X, dr, iter, 1, b.xa_all, b.sync, xm_epoch);
}
void launch_cpass(const Dims &d, const Bufs &b, hipStream_t s, const DrawsDev &dr, const double *delta_in,
                  const double *tau_in, double *delta_out, double *tau_out, int64_t delta_iter) {
    const dim3 grid(((d.PP + d.kp) / 32) * d.G * (d.kp / 32));
    DeltaArgs da;
    da.delta_in = delta_in; da.tau_in = tau_in; da.delta_out = delta_out; da.tau_out = tau_out;
    da.iter = delta_iter;
    const int ndel = (delta_in && d.kp == KP) ? cdiv(d.g, cp_waves<32>()) : 0;
    switch (d.kp) {
    case 32:
        // a few shards per rank: split the k columns by parity (k_cpass PS) below 128 blocks
        // (c3's g = 8 share, 88 blocks: +7 %; the g = 16 / 32 shares, 176 / 352: -4 / -2 %)
        if (grid.x < 128)
            hipLaunchKernelGGL((k_cpass<32, true>), dim3(2 * grid.x + ndel), dim3(64 * cp_waves<32>()), 0, s, d, b.Y,
                               b.X, b.Z, b.C, b.E, dr, b.sall, da, ndel);
        else
            hipLaunchKernelGGL((k_cpass<32, false>), dim3(grid.x + ndel), dim3(64 * cp_waves<32>()), 0, s, d, b.Y, b.X,
                               b.Z, b.C, b.E, dr, b.sall, da, ndel);
        break;
    // wide: eta formed once (k_eta into W, free after k_zdraw) instead of in each of the shard's column
    // tiles from X and Z: their two 2 MB panels shared the XCD's L2 with the Y stream (c4: 358 MB)
    case 64:
        if (DCFM_WIDE_ETA) launch_eta(d, b, b.W, s);
        hipLaunchKernelGGL(k_cpass<64>, grid, dim3(256), 0, s, d, b.Y, DCFM_WIDE_ETA ? b.W : b.X, b.Z, b.C, b.E, dr,
                           b.sall, da, 0);
        break;
    default:
        if (DCFM_WIDE_ETA) launch_eta(d, b, b.W, s);
        hipLaunchKernelGGL(k_cpass<128>, grid, dim3(256), 0, s, d, b.Y, DCFM_WIDE_ETA ? b.W : b.X, b.Z, b.C, b.E, dr,
                           b.sall, da, 0);
        break;
    }
}
void launch_lambda(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter,
                   const double *tau_cur, const double *plam_src, hipStream_t s, bool gen, double kappa_max) {
    if (d.kp != KP) return wide::launch_lambda(d, b, dr, iter, tau_cur, plam_src, s, kappa_max);
    LamDraws ld;
    if (gen) {   // this iteration's variates, drawn by k_wcol's LAMGEN blocks (lam_draws)
        const LamGen g = lam_gen_plan(d, b.ldraw);
        ld.NL = g.NL; ld.Gpsi = g.Gpsi; ld.Gps = g.Gps;
    } else {     // [T][g][P][K] / [T][g][P] draw buffers: this iteration, this rank's first shard
        const size_t row0 = ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
        ld.NL = dr.NL + row0 * d.K;
        ld.Gpsi = dr.Gpsi + row0 * d.K;
        ld.Gps = dr.Gps + row0;
    }
    const dim3 grid(cdiv(d.P, LAM_ROWS), d.G);
#define LAUNCH_LAM(KE)                                                                                       \
    hipLaunchKernelGGL(k_lambda<KE>, grid, dim3(64), 0, s, d, b.C, b.E, b.yy, tau_cur, b.Lam, b.psi, plam_src, \
                       b.ps, b.omega, b.cpart, ld, b.Y, b.X, b.Z, kappa_max)
    // the factor width rounded up to an instantiated one (rows >= K are identity padding)
    if (d.K <= 8) LAUNCH_LAM(8);
    else if (d.K <= 16) LAUNCH_LAM(16);
    else if (d.K <= 20) LAUNCH_LAM(20);
    else if (d.K <= 24) LAUNCH_LAM(24);
    else if (d.K <= 30) LAUNCH_LAM(30);
    else LAUNCH_LAM(32);
#undef LAUNCH_LAM
}
void launch_colsum(const Dims &d, const Bufs &b, hipStream_t s) {
    const dim3 grid(d.G, d.kp / 32);
    switch (d.kp) {
    case 32: hipLaunchKernelGGL(k_colsum<32>, grid, dim3(256), 0, s, d, b.cpart, b.sloc); break;
    case 64: hipLaunchKernelGGL(k_colsum<64>, grid, dim3(256), 0, s, d, b.cpart, b.sloc); break;
    default: hipLaunchKernelGGL(k_colsum<128>, grid, dim3(256), 0, s, d, b.cpart, b.sloc); break;
    }
}
void launch_delta(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter,
                  const double *delta_in, const double *tau_in, double *delta_out, double *tau_out,
                  hipStream_t s) {
    if (d.kp != KP) return wide::launch_delta(d, b, dr, iter, delta_in, tau_in, delta_out, tau_out, s);
    hipLaunchKernelGGL(k_delta, dim3(d.g), dim3(64), 0, s, d, b.sall, delta_in, tau_in, delta_out,
                       tau_out, dr, iter);
}
void launch_save(const Dims &d, const Bufs &b, double *Lb, double *wsum, int slot, hipStream_t s) {
    const size_t total = (size_t)d.G * d.P * d.K;
    const int grid = (int)std::min<size_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_save, dim3(grid), dim3(256), 0, s, d, b.Lam, b.omega, Lb, wsum, b.LDB, slot);
}
void launch_assemble(const Dims &d, const Bufs &b, const double *Lb, const double *wsum, int kext,
                     double inv_eff, hipStream_t s) {
    if (b.ntiles == 0) return;
    hipLaunchKernelGGL(k_assemble, dim3(b.ntiles), dim3(ASM_THREADS), 0, s, d, Lb, b.LDB, kext, wsum, inv_eff,
                       b.tiles, b.T0, b.Sigma);
}
void launch_sigma_pack(const double *S, int p, int T0, int T1, int c0, int nc, double *out, hipStream_t s) {
    const int R1 = std::min(p, T1 * ASM_TILE);
    if (nc <= 0 || R1 <= 0 || T1 <= T0) return;
    hipLaunchKernelGGL(k_sigma_pack, dim3(cdiv(R1, 32), cdiv(nc, 32)), dim3(256), 0, s, S, p, T0, T1, c0, nc, out);
}
void launch_sigma_unpack(const double *recv, int p, int c0, int nc, const int *Tb, const long long *base,
                         int nranks, double *out, hipStream_t s) {
    for (int j = 0; j < nc; j += 32768) {   // grid.y <= 32768 columns per launch
        const int w = std::min(32768, nc - j);
        hipLaunchKernelGGL(k_sigma_unpack, dim3(std::min(cdiv(p, 256), 16), w), dim3(256), 0, s, recv, p, c0, c0 + j,
                           Tb, base, nranks, out);
    }
}
void launch_eta(const Dims &d, const Bufs &b, double *eta_out, hipStream_t s) {
    const size_t total = (size_t)d.G * d.NP * d.kp;
    const int grid = (int)std::min<size_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_eta, dim3(grid), dim3(256), 0, s, d, b.X, b.Z, eta_out);
}
void launch_draws(const Dims &d, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    const DrawPlan pl = draw_plan(d);
    hipLaunchKernelGGL(k_draws<true>, dim3(pl.b_gpsi), dim3(256), 0, s, d, dr, iter);
    hipLaunchKernelGGL(k_draws<false>, dim3(pl.total - pl.b_gpsi), dim3(256), 0, s, d, dr, iter);
}
// NaN / Inf sentinel (DCFM_ERR_NUMERIC): after a dcfm_run, every non-finite value of the
// state a later iteration reads (Lambda, ps, omega, X, tau) sets *flag (sticky until the
// next set_state / init_state).  A NaN anywhere in a sweep reaches these within one
// iteration (SS_j -> ps_j -> omega_j; X -> eta -> Lambda).  One pass over ~6 MB at c3.
__device__ __forceinline__ bool bad(double v) { return !(fabs(v) <= 1.7976931348623157e308); }
__global__ __launch_bounds__(256) void k_finite(Dims d, const double *__restrict__ Lam,
                                                const double *__restrict__ ps, const double *__restrict__ omega,
                                                const double *__restrict__ X, const double *__restrict__ tau,
                                                int *__restrict__ flag) {
    const size_t nL = (size_t)d.G * d.PP * d.kp, nP = (size_t)d.G * d.PP, nX = (size_t)d.NP * d.kp,
                 nT = (size_t)d.g * d.kp;
    bool any = false;
    for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < nL; e += (size_t)gridDim.x * 256) any |= bad(Lam[e]);
    for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < nP; e += (size_t)gridDim.x * 256)
        any |= bad(ps[e]) || bad(omega[e]);
    for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < nX; e += (size_t)gridDim.x * 256) any |= bad(X[e]);
    for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < nT; e += (size_t)gridDim.x * 256) any |= bad(tau[e]);
    if (any) *flag = 1;   // benign race: every writer stores 1
}
void launch_finite(const Dims &d, const Bufs &b, const double *tau_cur, int *flag, hipStream_t s) {
    hipLaunchKernelGGL(k_finite, dim3(128), dim3(256), 0, s, d, b.Lam, b.ps, b.omega, b.X, tau_cur, flag);
}

__global__ __launch_bounds__(256) void k_sum_slices(const double *__restrict__ src, int ns, size_t count,
                                                   double *__restrict__ dst) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) {
        double v = 0.0;
        for (int k = 0; k < ns; ++k) v += src[(size_t)k * count + i];
        dst[i] = v;
    }
}
void launch_sum_slices(const double *src, int ns, size_t count, double *dst, hipStream_t s) {
    const int grid = (int)std::min<size_t>((count + 255) / 256, 8192);
    hipLaunchKernelGGL(k_sum_slices, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, src, ns, count, dst);
}
void launch_rng_fill(uint64_t seed, int kind, double shape, int site, int shard, int64_t iter,
                     int64_t count, int width, double *out, hipStream_t s) {
    const int grid = (int)std::min<int64_t>((count + 255) / 256, 8192);
    hipLaunchKernelGGL(k_rng_fill, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, seed, kind, shape, site,
                       shard, iter, count, width, out);
}

}  // namespace dcfm
