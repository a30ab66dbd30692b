// Hand-written CDNA4 (gfx950) kernels for one Gibbs iteration of the
// divide-and-conquer factor model (reference divideconquer.m:90-196) and the
// covariance assembly.  fp64 throughout (the reference is double precision).
//
// Kernel map (per iteration, in order)                         reference lines
//   k_prep     A_m = Lambda' diag(w) Lambda (MFMA), R_m = cholcov(I+(1-rho)A_m)  dc:98-100,114-115
//   k_wpass    W_m = Y_m (w o Lambda_m)           fp64 MFMA, Y pass 1      dc:102-103,122-123
//   k_zdraw    Z rows: R\ , R'\ , noise; per-shard (W - s1r A Z')          dc:101-107,121-124
//   k_xred     sum over local shards (+ sum_m A_m)                         dc:112-116,120-124
//   [RCCL all-gather across ranks]
//   k_xdraw    Xprec = gI + rho sum A, cholcov, X rows                     dc:117-128
//   k_cpass    C_m = Y_m' eta_m, E_m = eta_m' eta_m  fp64 MFMA, Y pass 2   dc:133,138,141
//   k_lambda   per loading row: Q, chol, 3 solves, Lambda_j; psi_j;        dc:140-145,150,
//              SS_j via identity, ps_j, omega_j; column sums of psi o L^2  dc:156,169-171
//   k_colsum   per-shard column sums                                       dc:156
//   [RCCL all-gather across ranks]
//   k_delta    MGP chain (quirks Q4/Q5) for all shards, Plam refresh       dc:155-165,175-177
//   saved iterations: k_save (+ RCCL all-gather at flush), k_assemble      dc:180-195
//
// The residual pass of dc:169-170 needs no third read of Y: with C_j = eta'Y_j
// and E = eta'eta already computed for the loading draw,
//   SS_j = sum_i (Y_ij - eta_i Lambda_j')^2 = yy_j - 2 Lambda_j.C_j + Lambda_j E Lambda_j'.
#include "dcfm_internal.h"
#include "philox.h"

#include <algorithm>

namespace dcfm {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d4 mfma16x16x4(double a, double b, d4 c) {
    // v_mfma_f64_16x16x4_f64: A[i=lane&15][k=lane>>4], B[k=lane>>4][j=lane&15],
    // C/D: col = lane&15, row = (lane>>4) + 4*reg
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double readlane_d(double x, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}

// value of x held by lane c of this lane's half-wave
__device__ __forceinline__ double readsel(double x, int c, bool upper) {
    const double lo = readlane_d(x, c);
    const double hi = readlane_d(x, 32 + c);
    return upper ? hi : lo;
}

// 1/sqrt(x) to full fp64 precision: hardware estimate + 2 Newton steps
__device__ __forceinline__ double rsqrt_f64(double x) {
    double y = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double e = fma(-x * y, y, 1.0);
        y = fma(0.5 * y, e, y);
    }
    return y;
}

// eta = sqrt(rho) X + sqrt(1-rho) Z    (dc:81,133) — one definition for every use
__device__ __forceinline__ double eta_of(double sr, double s1r, double x, double z) {
    return sr * x + s1r * z;
}

// ----------------------------------------------------------------------------
// Register Cholesky of a KP x KP SPD matrix per half-wave (32 lanes).
// Lane r = lane & 31 holds row r in q[] (entries c <= r are read).  On return
// q[c] = L[r][c] (0 for c > r) and the LDS image Lt[k][c] = L[c][k] (column k
// of L, contiguous) with Lt[k][KP] = 1/L[k][k].  Right-looking; column k is
// broadcast through LDS; the diagonal through readlane.  Both half-waves run
// independent matrices (or the same one, writing identical values).
// ----------------------------------------------------------------------------
constexpr int LS = KP + 2;

__device__ __forceinline__ void chol_rows(double (&q)[KP], double (*Lt)[LS], int r, bool upper) {
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const double dkk = readsel(q[k], k, upper);
        const double ikk = rsqrt_f64(dkk);
        const double lkk = dkk * ikk;
        const double lrk = (r > k) ? q[k] * ikk : (r == k ? lkk : 0.0);
        q[k] = lrk;
        Lt[k][r] = lrk;
        if (r == k) Lt[k][KP] = ikk;
#pragma unroll
        for (int c = k + 1; c < KP; ++c) q[c] -= lrk * Lt[k][c];
        // keep the trailing update eager: without this hipcc sinks each FMA to
        // the step that consumes q[c] and keeps O(K^2) loaded L values live
#pragma unroll
        for (int c = k + 1; c < KP; ++c) asm volatile("" : "+v"(q[c]));
    }
}

// ============================================================================
// k_prep: A_m = (w o Lambda_m)' Lambda_m and R_m = cholcov(eye(K) + (1-rho) A_m)   dc:98-100
// 4 waves split the j reduction (fp64 MFMA 2x2 tiles), LDS sum, wave 0 factors.
// ============================================================================
__global__ __launch_bounds__(256) void k_prep(Dims d, const double *__restrict__ Lam,
                                              const double *__restrict__ omega,
                                              double *__restrict__ A, double *__restrict__ R,
                                              double *__restrict__ Rdi) {
    __shared__ double part[4][KP][KP + 1];
    __shared__ double Lt[KP][LS];
    const int m = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, q = lane >> 4;
    const double *L = Lam + (size_t)m * d.PP * KP;
    const double *w = omega + (size_t)m * d.PP;
    d4 a00 = {0, 0, 0, 0}, a01 = a00, a10 = a00, a11 = a00;
    for (int t = wave; t < (d.PP >> 3); t += 4) {
        const int j = 8 * t + 2 * q;
        const d2 wj = *reinterpret_cast<const d2 *>(w + j);
        const double lo0 = L[j * KP + r], hi0 = L[j * KP + 16 + r];
        const double lo1 = L[(j + 1) * KP + r], hi1 = L[(j + 1) * KP + 16 + r];
        // A operand (w_j Lambda_ja) [Zmsg, dc:98], B operand Lambda_jb
        const double wl0 = lo0 * wj.x, wh0 = hi0 * wj.x, wl1 = lo1 * wj.y, wh1 = hi1 * wj.y;
        a00 = mfma16x16x4(wl0, lo0, a00); a01 = mfma16x16x4(wl0, hi0, a01);
        a10 = mfma16x16x4(wh0, lo0, a10); a11 = mfma16x16x4(wh0, hi0, a11);
        a00 = mfma16x16x4(wl1, lo1, a00); a01 = mfma16x16x4(wl1, hi1, a01);
        a10 = mfma16x16x4(wh1, lo1, a10); a11 = mfma16x16x4(wh1, hi1, a11);
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
    for (int e = threadIdx.x; e < KP * KP; e += 256) {
        const int a = e / KP, b = e % KP;
        const double v = (part[0][a][b] + part[1][a][b]) + (part[2][a][b] + part[3][a][b]);
        Am[e] = v;
        part[0][a][b] = v;
    }
    __syncthreads();
    if (wave != 0) return;
    // cholcov reads the upper triangle: S[rr][c] = Zprec[c][rr] for c <= rr
    const int rr = lane & 31;
    const bool upper = lane >= 32;
    double qq[KP];
#pragma unroll
    for (int c = 0; c < KP; ++c)
        qq[c] = (c <= rr) ? ((c == rr ? 1.0 : 0.0) + (1.0 - d.rho) * part[0][c][rr]) : 0.0;
    chol_rows(qq, Lt, rr, upper);
    double *Rm = R + (size_t)m * KP * KP;
    for (int e = lane; e < KP * KP; e += 64) {
        const int a = e / KP, b = e % KP;
        Rm[e] = (b >= a) ? Lt[a][b] : 0.0;        // R = L', upper, R'R = Zprec
    }
    if (lane < KP) Rdi[(size_t)m * KP + lane] = Lt[lane][KP];
}

// XCD-aware block remap (bijective): hardware deals consecutive block ids
// round-robin over the 8 XCDs; give each XCD a contiguous range of work items
// so that blocks sharing operands (one shard's tiles) share one L2.
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int xcd = b & 7, slot = b >> 3;
    const int q = total >> 3, rem = total & 7;
    return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + slot;
}

// ============================================================================
// k_wpass: W_m[i][k] = sum_j Y_m[i][j] (w_j Lambda_m[j][k])   fp64 MFMA, Y pass 1
// one wave = (shard m, 32 rows i = 2 M-tiles) x 32 k (even / odd k N-tiles),
// reduction over j in chunks of 8: lane (r, q) holds Y[i0+r][8t+2q .. +1] (16 B);
// k-step 2t uses element 0, 2t+1 element 1; the B operand (w_j L[j][2r], w_j L[j][2r+1])
// uses the same j <-> (q, e) map.  Register double-buffered prefetch of 2 chunks.
// ============================================================================
__global__ __launch_bounds__(256) void k_wpass(Dims d, const double *__restrict__ Y,
                                               const double *__restrict__ Lam,
                                               const double *__restrict__ omega,
                                               double *__restrict__ W) {
    const int nrb = d.NP >> 7;                       // 128-row blocks per shard
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int m = w / nrb, rb = w % nrb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i0 = rb * 128 + wave * 32;
    const int r = lane & 15, q = lane >> 4;
    const double *Y0 = Y + ((size_t)m * d.NP + i0 + r) * d.PP + 2 * q;
    const double *Y1 = Y0 + (size_t)16 * d.PP;
    const double *L = Lam + (size_t)m * d.PP * KP + 2 * r;
    const double *wp = omega + (size_t)m * d.PP + 2 * q;
    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int nch = d.PP >> 3;
    d2 yA0, yA1, wA, lA0, lA1, yB0, yB1, wB, lB0, lB1;
#define WP_LOAD(t, y0, y1, ww, l0, l1)                                              \
    {                                                                               \
        const int j = 8 * (t);                                                      \
        y0 = *reinterpret_cast<const d2 *>(Y0 + j);                                 \
        y1 = *reinterpret_cast<const d2 *>(Y1 + j);                                 \
        ww = *reinterpret_cast<const d2 *>(wp + j);                                 \
        l0 = *reinterpret_cast<const d2 *>(L + (size_t)(j + 2 * q) * KP);           \
        l1 = *reinterpret_cast<const d2 *>(L + (size_t)(j + 2 * q + 1) * KP);       \
    }
#define WP_MMA(y0, y1, ww, l0, l1)                                                  \
    {                                                                               \
        const double b00 = ww.x * l0.x, b01 = ww.x * l0.y;                          \
        const double b10 = ww.y * l1.x, b11 = ww.y * l1.y;                          \
        acc[0][0] = mfma16x16x4(y0.x, b00, acc[0][0]);                              \
        acc[0][1] = mfma16x16x4(y0.x, b01, acc[0][1]);                              \
        acc[1][0] = mfma16x16x4(y1.x, b00, acc[1][0]);                              \
        acc[1][1] = mfma16x16x4(y1.x, b01, acc[1][1]);                              \
        acc[0][0] = mfma16x16x4(y0.y, b10, acc[0][0]);                              \
        acc[0][1] = mfma16x16x4(y0.y, b11, acc[0][1]);                              \
        acc[1][0] = mfma16x16x4(y1.y, b10, acc[1][0]);                              \
        acc[1][1] = mfma16x16x4(y1.y, b11, acc[1][1]);                              \
    }
    WP_LOAD(0, yA0, yA1, wA, lA0, lA1);
    for (int t = 0; t < nch; t += 2) {
        if (t + 1 < nch) WP_LOAD(t + 1, yB0, yB1, wB, lB0, lB1);
        WP_MMA(yA0, yA1, wA, lA0, lA1);
        if (t + 2 < nch) WP_LOAD(t + 2, yA0, yA1, wA, lA0, lA1);
        if (t + 1 < nch) WP_MMA(yB0, yB1, wB, lB0, lB1);
    }
#undef WP_LOAD
#undef WP_MMA
    // D row = q + 4g (row i), col = r (k = 2r + tb)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        double *Wt = W + ((size_t)m * d.NP + i0 + 16 * a) * KP + 2 * r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            d2 v;
            v.x = acc[a][0][g];
            v.y = acc[a][1][g];
            *reinterpret_cast<d2 *>(Wt + (size_t)(q + 4 * g) * KP) = v;
        }
    }
}

// ============================================================================
// k_zdraw: per (row i, shard m), lane = row; one shard per block, A_m and R_m
// broadcast from LDS.                                           dc:101-107,121-123
//   bz = sqrt(1-rho) (W_i - sqrt(rho) A X_i)            (= sqrt(1-rho) Zmsg'(Y_i - sqrt(rho) L X_i))
//   v  = R \ bz ;  Z_i = R' \ (v + eps)                 (quirk Q2 order)
//   Sp_m,i = W_i - sqrt(1-rho) A Z_i                     (Xmsg'(Y_i - sqrt(1-rho) L Z_i))
// ============================================================================
__global__ __launch_bounds__(256) void k_zdraw(Dims d, const double *__restrict__ W,
                                               const double *__restrict__ A,
                                               const double *__restrict__ R,
                                               const double *__restrict__ Rdi,
                                               const double *__restrict__ X,
                                               double *__restrict__ Z, double *__restrict__ Sp,
                                               DrawsDev dr, int64_t iter) {
    __shared__ double As[KP][KP], Rs[KP][KP], Rd[KP];
    const int m = blockIdx.y;
    {
        const double *Am = A + (size_t)m * KP * KP;
        const double *Rm = R + (size_t)m * KP * KP;
        for (int e = threadIdx.x; e < KP * KP; e += 256) {
            As[e / KP][e % KP] = Am[e];
            Rs[e / KP][e % KP] = Rm[e];
        }
        if (threadIdx.x < KP) Rd[threadIdx.x] = Rdi[(size_t)m * KP + threadIdx.x];
    }
    __syncthreads();
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= d.NP) return;
    double *Spi = Sp + ((size_t)m * d.NP + i) * KP;
    if (i >= d.n) {
#pragma unroll
        for (int k = 0; k < KP; k += 2) *reinterpret_cast<d2 *>(Spi + k) = d2{0.0, 0.0};
        return;
    }
    const double *Wi = W + ((size_t)m * d.NP + i) * KP;
    const double *Xi = X + (size_t)i * KP;
    double x[KP], t[KP];
#pragma unroll
    for (int k = 0; k < KP; k += 2) {
        const d2 v = *reinterpret_cast<const d2 *>(Xi + k);
        x[k] = v.x;
        x[k + 1] = v.y;
    }
#pragma unroll
    for (int a = 0; a < KP; ++a) {
        double acc = 0.0;
#pragma unroll
        for (int b = 0; b < KP; ++b) acc += As[a][b] * x[b];
        t[a] = d.s1r * (Wi[a] - d.sr * acc);
    }
    // back substitution R v = bz (R upper)
#pragma unroll
    for (int a = KP - 1; a >= 0; --a) {
        double acc = t[a];
#pragma unroll
        for (int b = a + 1; b < KP; ++b) acc -= Rs[a][b] * t[b];
        t[a] = acc * Rd[a];
    }
    // + eps  (dc:104 normrnd(0,1,[K,1]))
    const int mg = d.shard0 + m;
    if (d.inject) {
        const double *nz = dr.NZ + (((size_t)(iter - dr.first_iter) * d.g + mg) * d.n + i) * d.K;
#pragma unroll
        for (int k = 0; k < KP; ++k)
            if (k < d.K) t[k] += nz[k];
    } else {
        const Rng rng(d.seed);
#pragma unroll
        for (int k = 0; k < KP; k += 2) {
            if (k < d.K) {
                double n0, n1;
                rng.normal2(SITE_Z, mg, i, k >> 1, (uint32_t)iter, n0, n1);
                t[k] += n0;
                if (k + 1 < d.K) t[k + 1] += n1;
            }
        }
    }
    // forward substitution R' z = v + eps
#pragma unroll
    for (int a = 0; a < KP; ++a) {
        double acc = t[a];
#pragma unroll
        for (int b = 0; b < a; ++b) acc -= Rs[b][a] * t[b];
        t[a] = acc * Rd[a];
    }
    double *Zi = Z + ((size_t)m * d.NP + i) * KP;
#pragma unroll
    for (int k = 0; k < KP; k += 2) {
        d2 v;
        v.x = (k < d.K) ? t[k] : 0.0;
        v.y = (k + 1 < d.K) ? t[k + 1] : 0.0;
        *reinterpret_cast<d2 *>(Zi + k) = v;
    }
#pragma unroll
    for (int a = 0; a < KP; a += 2) {
        double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
        for (int b = 0; b < KP; ++b) {
            acc0 += As[a][b] * t[b];
            acc1 += As[a + 1][b] * t[b];
        }
        d2 v;
        v.x = Wi[a] - d.s1r * acc0;
        v.y = Wi[a + 1] - d.s1r * acc1;
        *reinterpret_cast<d2 *>(Spi + a) = v;
    }
}

// ============================================================================
// k_xred: xin[i][k] = sum_m Sp[m][i][k];  xin[NP+a][b] = sum_m A_m[a][b]     dc:113-116,121-124
// ============================================================================
__global__ __launch_bounds__(256) void k_xred(Dims d, const double *__restrict__ Sp,
                                              const double *__restrict__ A,
                                              double *__restrict__ xin) {
    const size_t total = (size_t)(d.NP + KP) * KP;
    const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (e >= total) return;
    const size_t row = e / KP;
    double acc = 0.0;
    if (row < (size_t)d.NP) {
        const size_t stride = (size_t)d.NP * KP;
#pragma unroll 8
        for (int m = 0; m < d.G; ++m) acc += Sp[(size_t)m * stride + e];
    } else {
        const size_t off = e - (size_t)d.NP * KP;
#pragma unroll 8
        for (int m = 0; m < d.G; ++m) acc += A[(size_t)m * KP * KP + off];
    }
    xin[e] = acc;
}

// ============================================================================
// k_xdraw: X rows.  Xprec = g*I + rho*sum_m A_m (all ranks), Rx = cholcov,     dc:117-128
//   X_i = Rx' \ (Rx \ (sqrt(rho) S_i) + eps)
// one wave per 64 rows; every block factors the KxK Xprec itself (register Cholesky).
// ============================================================================
__global__ __launch_bounds__(64) void k_xdraw(Dims d, const double *__restrict__ xall,
                                              double *__restrict__ X, DrawsDev dr, int64_t iter) {
    __shared__ double Lt[KP][LS];
    __shared__ double As[KP][KP + 1];
    const int lane = threadIdx.x;
    const int rr = lane & 31;
    const bool upper = lane >= 32;
    const size_t stride = (size_t)(d.NP + KP) * KP;
    // sum_m A_m over all ranks (rank order), staged through LDS by all lanes
    for (int e = lane; e < KP * KP; e += 64) {
        double v = xall[(size_t)d.NP * KP + e];
        for (int rk = 1; rk < d.nranks; ++rk) v += xall[rk * stride + (size_t)d.NP * KP + e];
        As[e / KP][e % KP] = v;
    }
    __syncthreads();
    {
        double qq[KP];
#pragma unroll
        for (int c = 0; c < KP; ++c)   // cholcov reads the upper triangle: S[rr][c] = Xprec[c][rr]
            qq[c] = (c <= rr) ? ((c == rr ? (double)d.g : 0.0) + d.rho * As[c][rr]) : 0.0;
        chol_rows(qq, Lt, rr, upper);
    }
    const int i = blockIdx.x * 64 + lane;
    if (i >= d.n) return;
    double v[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) v[k] = 0.0;
    for (int rk = 0; rk < d.nranks; ++rk) {
        const double *s = xall + rk * stride + (size_t)i * KP;
#pragma unroll
        for (int k = 0; k < KP; k += 2) {
            const d2 u = *reinterpret_cast<const d2 *>(s + k);
            v[k] += u.x;
            v[k + 1] += u.y;
        }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) v[k] = d.sr * v[k];     // bx = sqrt(rho)*sumx2
    // Rx v' = bx; Rx[a][b] = L[b][a] = Lt[a][b]
#pragma unroll
    for (int a = KP - 1; a >= 0; --a) {
        double acc = v[a];
#pragma unroll
        for (int b = a + 1; b < KP; ++b) acc -= Lt[a][b] * v[b];
        v[a] = acc * Lt[a][KP];
    }
    if (d.inject) {
        const double *nx = dr.NX + ((size_t)(iter - dr.first_iter) * d.n + i) * d.K;
#pragma unroll
        for (int k = 0; k < KP; ++k)
            if (k < d.K) v[k] += nx[k];
    } else {
        const Rng rng(d.seed);
#pragma unroll
        for (int k = 0; k < KP; k += 2) {
            if (k < d.K) {
                double n0, n1;
                rng.normal2(SITE_X, 0, i, k >> 1, (uint32_t)iter, n0, n1);
                v[k] += n0;
                if (k + 1 < d.K) v[k + 1] += n1;
            }
        }
    }
    // Rx' x = v + eps; Rx'[a][b] = Lt[b][a]
#pragma unroll
    for (int a = 0; a < KP; ++a) {
        double acc = v[a];
#pragma unroll
        for (int b = 0; b < a; ++b) acc -= Lt[b][a] * v[b];
        v[a] = acc * Lt[a][KP];
    }
    double *Xi = X + (size_t)i * KP;
#pragma unroll
    for (int k = 0; k < KP; k += 2) {
        d2 u;
        u.x = (k < d.K) ? v[k] : 0.0;
        u.y = (k + 1 < d.K) ? v[k + 1] : 0.0;
        *reinterpret_cast<d2 *>(Xi + k) = u;
    }
}

// ============================================================================
// k_cpass: [C_m | E_m] = [Y_m | eta_m]' eta_m    fp64 MFMA, Y pass 2      dc:133,138,141
// block = (shard m, 32-column tile of [Y | eta]); its 4 waves split the
// reduction over rows i, partial 32x32 tiles summed in LDS in a fixed order.
// Lane (r, q) loads 16 B: Y[i][c0+2r .. +1] and eta[i][2r .. +1] (formed on the
// fly from X and Z), i = 4s + q, so the MFMA tiles are even/odd columns x
// even/odd k.  Register double-buffered prefetch, 4 k-steps per batch.
// ============================================================================
template <bool IS_E>
__device__ __forceinline__ void cpass_wave(const Dims &d, const double *__restrict__ Yp,
                                           const double *__restrict__ Xp,
                                           const double *__restrict__ Zp, int s0, int nsw,
                                           int q, d4 (&acc)[2][2]) {
    d2 yA[4], xA[4], zA[4], yB[4], xB[4], zB[4];
    auto load = [&](int s, d2 (&y)[4], d2 (&x)[4], d2 (&z)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = 4 * (s + u) + q;
            x[u] = *reinterpret_cast<const d2 *>(Xp + (size_t)i * KP);
            z[u] = *reinterpret_cast<const d2 *>(Zp + (size_t)i * KP);
            if (!IS_E) y[u] = *reinterpret_cast<const d2 *>(Yp + (size_t)i * d.PP);
        }
    };
    auto mma = [&](d2 (&y)[4], d2 (&x)[4], d2 (&z)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double e0 = eta_of(d.sr, d.s1r, x[u].x, z[u].x);
            const double e1 = eta_of(d.sr, d.s1r, x[u].y, z[u].y);
            const double a0 = IS_E ? e0 : y[u].x, a1 = IS_E ? e1 : y[u].y;
            acc[0][0] = mfma16x16x4(a0, e0, acc[0][0]);
            acc[0][1] = mfma16x16x4(a0, e1, acc[0][1]);
            acc[1][0] = mfma16x16x4(a1, e0, acc[1][0]);
            acc[1][1] = mfma16x16x4(a1, e1, acc[1][1]);
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

__global__ __launch_bounds__(256) void k_cpass(Dims d, const double *__restrict__ Y,
                                               const double *__restrict__ X,
                                               const double *__restrict__ Z,
                                               double *__restrict__ C, double *__restrict__ E) {
    __shared__ double red[4][32][33];
    const int nt = (d.PP + KP) >> 5;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int m = w / nt, tile = w % nt;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c0 = tile * 32;
    const bool isE = c0 >= d.PP;
    const int r = lane & 15, q = lane >> 4;
    const double *Yp = Y + (size_t)m * d.NP * d.PP + c0 + 2 * r;
    const double *Xp = X + 2 * r;
    const double *Zp = Z + (size_t)m * d.NP * KP + 2 * r;
    const int nsw = d.NP >> 4;                 // k-steps (4 rows each) per wave
    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    if (isE) cpass_wave<true>(d, Yp, Xp, Zp, wave * nsw, nsw, q, acc);
    else cpass_wave<false>(d, Yp, Xp, Zp, wave * nsw, nsw, q, acc);
    // D row rho = q + 4g -> column c0 + 2 rho + ta;  D col r -> k = 2r + tb
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int rho = q + 4 * g;
#pragma unroll
        for (int ta = 0; ta < 2; ++ta)
#pragma unroll
            for (int tb = 0; tb < 2; ++tb) red[wave][2 * rho + ta][2 * r + tb] = acc[ta][tb][g];
    }
    __syncthreads();
    double *out = isE ? (E + (size_t)m * KP * KP) : (C + ((size_t)m * d.PP + c0) * KP);
    for (int e = threadIdx.x; e < 32 * KP; e += 256) {
        const int a = e / KP, b = e % KP;
        out[e] = (red[0][a][b] + red[1][a][b]) + (red[2][a][b] + red[3][a][b]);
    }
}

// ----------------------------------------------------------------------------
// Packed variant for k_lambda: per half-wave LDS image Lp = [column-major packed
// lower L (528) | 1/L_kk (32) | broadcast scratch (32)].  The forward solve
// L v = b is fused into the factorisation (b rides along as an extra column),
// and the next pivot is formed from the pivot lane's own registers so the LDS
// column broadcast stays off the serial critical path.
// ----------------------------------------------------------------------------
constexpr int PACK = KP * (KP + 1) / 2;
constexpr int PSTRIDE = PACK + 2 * KP;
__host__ __device__ constexpr int pbase(int k) { return k * KP - (k * (k - 1)) / 2; }

__device__ __forceinline__ void chol_rows_fwd(double (&q)[KP], double *Lp, int r, bool upper,
                                              double bv, double &vr) {
    double piv = readsel(q[0], 0, upper);
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const double ikk = rsqrt_f64(piv);
        const double lkk = piv * ikk;
        const double lrk = (r > k) ? q[k] * ikk : (r == k ? lkk : 0.0);
        q[k] = lrk;
        if (r >= k) Lp[pbase(k) + r - k] = lrk;          // column k of L
        if (r == k) Lp[PACK + k] = ikk;
        const double vk = readsel(bv, k, upper) * ikk;   // v_k = b_k / L_kk
        if (r == k) vr = vk;
        if (r > k) bv -= lrk * vk;
        if (k + 1 < KP) piv = readsel(q[k + 1] - lrk * lrk, k + 1, upper);
#pragma unroll
        for (int c = k + 1; c < KP; ++c) q[c] -= lrk * Lp[pbase(k) + c - k];
#pragma unroll
        for (int c = k + 1; c < KP; ++c) asm volatile("" : "+v"(q[c]));
    }
}

// ============================================================================
// k_lambda: loading rows.  A half-wave (32 lanes) owns one row j; lane r holds
// row r of Q_j = diag(Plam_j) + ps_j E_m in registers.        dc:140-145 (+150,156,169-171)
//   L = chol(Q,'lower'), v = L \ (ps_j C_j)   (chol_rows_fwd)
//   Lambda_j = L' \ (v + z)                    (= ylam + mlam)
//   psi_j  = Gpsi * 1/(df/2 + 0.5 lambda^2 tau)               (dc:150, tau of the previous it.)
//   SS_j   = yy_j - 2 lambda.C_j + lambda' E lambda  ->  ps_j = Gps * 1/(bs + 0.5 SS_j), w = 1/ps
// 8 rows per 256-thread block; per-block column sums of psi o lambda^2 -> cpart.
// ============================================================================
__global__ __launch_bounds__(256) void k_lambda(Dims d, const double *__restrict__ C,
                                                const double *__restrict__ E,
                                                const double *__restrict__ yy,
                                                const double *__restrict__ tau_cur,
                                                double *__restrict__ Lam, double *__restrict__ psi,
                                                double *__restrict__ Plam, double *__restrict__ ps,
                                                double *__restrict__ omega,
                                                double *__restrict__ cpart, DrawsDev dr,
                                                int64_t iter) {
    __shared__ double LP[8][PSTRIDE];
    __shared__ double Es[KP][KP + 1];  // E_m, shared by the block's 8 rows (same shard)
    __shared__ double csum[8][KP];
    const int m = blockIdx.y;
    const int mg = d.shard0 + m;
    const int lane = threadIdx.x & 63;
    const int hw = threadIdx.x >> 5;          // half-wave id 0..7
    const bool upper = (lane >= 32);
    const int r = lane & 31;                  // matrix row
    const int j = blockIdx.x * 8 + hw;
    const bool valid = j < d.P;
    const bool real = r < d.K;
    const size_t rowoff = ((size_t)m * d.PP + (valid ? j : 0)) * KP;
    {
        const double *Em = E + (size_t)m * KP * KP;
        for (int e = threadIdx.x; e < KP * KP; e += 256) Es[e / KP][e % KP] = Em[e];
    }
    __syncthreads();
    // --- build Q row r and rhs
    const double psj = valid ? ps[(size_t)m * d.PP + j] : 0.0;
    double q[KP];
#pragma unroll
    for (int c = 0; c < KP; ++c) q[c] = psj * Es[r][c];
    const double plam = (valid && real) ? Plam[rowoff + r] : 1.0;
#pragma unroll
    for (int c = 0; c < KP; ++c)
        if (c == r) q[c] = (real && valid) ? plam + q[c] : 1.0;
    const double cjr = valid ? C[rowoff + r] : 0.0;

    double *Lp = LP[hw];
    double vr = 0.0;
    chol_rows_fwd(q, Lp, r, upper, psj * cjr, vr);
    // --- + z  (dc:142 normrnd(0,1,K,1))
    double z = 0.0;
    if (real && valid) {
        if (d.inject) {
            z = dr.NL[(((size_t)(iter - dr.first_iter) * d.g + mg) * d.P + j) * d.K + r];
        } else {
            const Rng rng(d.seed);
            z = rng.normal(SITE_LAMBDA, mg, j, r, (uint32_t)iter);
        }
    }
    double wr = vr + z;
    // --- back solve L' x = w;  L[c][r] = Lp[pbase(r) + c - r]
    double xr = 0.0;
    const int br = pbase(r) - r;
#pragma unroll 2
    for (int c = KP - 1; c >= 0; --c) {
        const double xc = readsel(wr, c, upper) * Lp[PACK + c];
        if (r == c) xr = xc;
        if (r < c) wr -= Lp[br + c] * xc;
    }
    if (!real) xr = 0.0;

    // --- SS_j = yy_j + sum_r x_r (E x)_r - 2 x_r C_jr; x broadcast through the scratch slots
    Lp[PACK + KP + r] = xr;
    double ex = 0.0;
#pragma unroll
    for (int c = 0; c < KP; ++c) ex += Es[c][r] * Lp[PACK + KP + c];   // (E x)_r, E symmetric
    double contrib = xr * (ex - 2.0 * cjr);
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) contrib += __shfl_xor(contrib, o, 32);

    // --- psi (dc:150), uses tau of the previous iteration (Q11)
    double psir = 0.0;
    if (real && valid) {
        const double tr = tau_cur[(size_t)mg * KP + r];
        const double scale = 1.0 / (d.df * 0.5 + 0.5 * (xr * xr * tr));
        double G;
        if (d.inject) {
            G = dr.Gpsi[(((size_t)(iter - dr.first_iter) * d.g + mg) * d.K + r) * d.P + j];
        } else {
            const Rng rng(d.seed);
            G = rng.gamma(d.df * 0.5 + 0.5, SITE_PSI, mg, j, r, (uint32_t)iter);
        }
        psir = scale * G;
    }
    csum[hw][r] = psir * (xr * xr);       // mat = psijh .* Lambda.^2 (dc:156)

    if (valid) {
        Lam[rowoff + r] = xr;
        if (real) psi[rowoff + r] = psir;
        if (r == 0) {
            const double SS = yy[(size_t)m * d.PP + j] + contrib;
            double G;
            if (d.inject) {
                G = dr.Gps[((size_t)(iter - dr.first_iter) * d.g + mg) * d.P + j];
            } else {
                const Rng rng(d.seed);
                G = rng.gamma(d.as_ + 0.5 * d.n, SITE_PS, mg, j, 0, (uint32_t)iter);
            }
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * G;   // dc:170
            ps[(size_t)m * d.PP + j] = psn;
            omega[(size_t)m * d.PP + j] = 1.0 / psn;            // dc:171 (Q1)
        }
    }
    __syncthreads();
    if (threadIdx.x < KP) {
        double s = 0.0;
#pragma unroll
        for (int h = 0; h < 8; ++h) s += csum[h][threadIdx.x];
        cpart[((size_t)m * (d.PP >> 3) + blockIdx.x) * KP + threadIdx.x] = s;
    }
}

// ============================================================================
// k_colsum: sloc[m][k] = sum_b cpart[m][b][k]                               dc:156 sum(mat)
// ============================================================================
__global__ __launch_bounds__(256) void k_colsum(Dims d, const double *__restrict__ cpart,
                                                double *__restrict__ sloc) {
    __shared__ double part[8][KP];
    const int m = blockIdx.x, k = threadIdx.x & 31, grp = threadIdx.x >> 5;
    const int nb = (d.P + 7) >> 3;
    double s = 0.0;
    for (int b = grp; b < nb; b += 8) s += cpart[((size_t)m * (d.PP >> 3) + b) * KP + k];
    part[grp][k] = s;
    __syncthreads();
    if (threadIdx.x < KP) {
        double t = 0.0;
#pragma unroll
        for (int g2 = 0; g2 < 8; ++g2) t += part[g2][threadIdx.x];
        sloc[(size_t)m * KP + threadIdx.x] = t;
    }
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
// refresh Plam = psi o tau'.
// ============================================================================
__device__ __forceinline__ double wave_scan_prod(double v, int l) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(v, o, 64);
        if (l >= o) v *= u;
    }
    return v;
}

__device__ __forceinline__ double wave_suffix_sum(double v, int l) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_down(v, o, 64);
        if (l + o < 64) v += u;
    }
    return v;
}

__device__ double delta_G(const Dims &d, const DrawsDev &dr, int64_t iter, int mg, int h) {
    if (d.inject) return dr.Gdelta[((size_t)(iter - dr.first_iter) * d.g + mg) * d.K + h];
    const double shape = (h == 0) ? d.ad1 + 0.5 * d.P * d.K : d.ad2 + 0.5 * d.P * (d.K - h);
    const Rng rng(d.seed);
    return rng.gamma(shape, SITE_DELTA, mg, 0, h, (uint32_t)iter);
}

// lane l < K holds delta_old_l, T_l, G_l, 1/delta_old_l and 1/dref_l; returns delta_new_l
__device__ double delta_chain(const Dims &d, int l, double T, double G, double idold, double idref) {
    double F = 1.0, dnew = 1.0;
    for (int h = 0; h < d.K; ++h) {
        const double Th = readlane_d(T, h), ih = readlane_d(idref, h);
        const double ioh = readlane_d(idold, h), Gh = readlane_d(G, h);
        const double bd = (h == 0 ? d.bd1 : d.bd2) + (0.5 * ih) * (F * Th);   // dc:157,161
        const double dn = (1.0 / bd) * Gh;                                      // dc:158,163
        if (l == h) dnew = dn;
        F = F * (dn * ioh);
    }
    return dnew;
}

__global__ __launch_bounds__(256) void k_delta(Dims d, const double *__restrict__ sall,
                                               const double *__restrict__ delta_in,
                                               const double *__restrict__ tau_in,
                                               double *__restrict__ delta_out,
                                               double *__restrict__ tau_out,
                                               const double *__restrict__ psi,
                                               double *__restrict__ Plam, DrawsDev dr,
                                               int64_t iter) {
    __shared__ double tnew[KP];
    const int m = blockIdx.x;   // global shard
    const int t = threadIdx.x;
    if (t < 64) {
        const int l = t;
        const int lk = l < KP ? l : 0;
        const bool act = l < d.K;
        if (d.K >= 2) {
            // shard 1 (index 0) with its own pre-update delta_h
            const double d0 = act ? delta_in[lk] : 1.0;
            const double T0 = wave_suffix_sum(act ? tau_in[lk] * sall[lk] : 0.0, l);
            const double G0 = act ? delta_G(d, dr, iter, 0, l) : 1.0;
            const double id0 = 1.0 / d0;
            const double d0new = delta_chain(d, l, T0, G0, id0, id0);
            double dm = d0new;
            if (m != 0) {
                const size_t o = (size_t)m * KP + lk;
                const double dold = act ? delta_in[o] : 1.0;
                const double Tm = wave_suffix_sum(act ? tau_in[o] * sall[o] : 0.0, l);
                const double Gm = act ? delta_G(d, dr, iter, m, l) : 1.0;
                const double idold = 1.0 / dold;
                const double idref = (l == 0) ? idold : 1.0 / d0new;   // delta(1,:,m) | delta(h) (Q4)
                dm = delta_chain(d, l, Tm, Gm, idold, idref);
            }
            const double tm = wave_scan_prod(act ? dm : 1.0, l);         // tauh = cumprod(delta)
            if (l < KP) {
                delta_out[(size_t)m * KP + l] = act ? dm : delta_in[(size_t)m * KP + l];
                tau_out[(size_t)m * KP + l] = act ? tm : tau_in[(size_t)m * KP + l];
                tnew[l] = tm;
            }
        } else {
            if (l == 0) {
                double prefix = 1.0, dnew = 0.0;
                for (int mm = 0; mm <= m; ++mm) {
                    const double dold = delta_in[(size_t)mm * KP];
                    const double tused = prefix * dold;
                    const double bd = d.bd1 + (0.5 * (1.0 / dold)) * (tused * sall[(size_t)mm * KP]);
                    dnew = (1.0 / bd) * delta_G(d, dr, iter, mm, 0);
                    prefix = prefix * dnew;
                }
                delta_out[(size_t)m * KP] = dnew;
                tau_out[(size_t)m * KP] = prefix;
                tnew[0] = prefix;
            }
            if (l >= 1 && l < KP) {
                delta_out[(size_t)m * KP + l] = delta_in[(size_t)m * KP + l];
                tau_out[(size_t)m * KP + l] = tau_in[(size_t)m * KP + l];
            }
        }
    }
    __syncthreads();
    const int ml = m - d.shard0;
    if (ml < 0 || ml >= d.G) return;
    const size_t base = (size_t)ml * d.PP * KP;
    for (int e = t; e < d.P * KP; e += 256) {
        const int k = e % KP;
        if (k < d.K) Plam[base + e] = psi[base + e] * tnew[k];   // dc:176
    }
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
        Lb[a * LDB + (size_t)slot * d.K + k] = Lam[((size_t)m * d.PP + j) * KP + k];
        if (k == 0) wsum[a] += omega[(size_t)m * d.PP + j];
    }
}

// ============================================================================
// k_assemble: Sigma[a][b] += (coef(a,b)/effsamp) sum_kk Lb[a][kk] Lb[b][kk]
//                            + [a==b] wsum[a]/effsamp                       dc:184-195
// coef = 1 inside a diagonal shard block (Lambda_r Lambda_r' + Omega_r), rho
// across blocks (rho Lambda_r Lambda_c').  Lower-triangle 128x128 tiles only;
// 4 waves in 2x2, each 64x64 = 4x4 tiles of v_mfma_f64_16x16x4; operands
// streamed from L2 with one chunk (8 k) of register prefetch.
// ============================================================================
__global__ __launch_bounds__(256) void k_assemble(Dims d, const double *__restrict__ Lb, int LDB,
                                                  int kext, const double *__restrict__ wsum,
                                                  double inv_eff, const int2 *__restrict__ tiles,
                                                  double *__restrict__ Sig) {
    const int2 T = tiles[blockIdx.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, q = lane >> 4;
    const int a0 = T.x * ASM_TILE + (wave >> 1) * 64;
    const int b0 = T.y * ASM_TILE + (wave & 1) * 64;
    const int p = d.p;
    const double *pa[4], *pb[4];
    bool va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int ar = a0 + 16 * u + r, br = b0 + 16 * u + r;
        va[u] = ar < p;
        vb[u] = br < p;
        pa[u] = Lb + (size_t)(va[u] ? ar : 0) * LDB + 2 * q;
        pb[u] = Lb + (size_t)(vb[u] ? br : 0) * LDB + 2 * q;
    }
    d4 acc[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = d4{0.0, 0.0, 0.0, 0.0};
    const d2 zero2 = {0.0, 0.0};
    d2 an[4], bn[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        an[u] = va[u] ? *reinterpret_cast<const d2 *>(pa[u]) : zero2;
        bn[u] = vb[u] ? *reinterpret_cast<const d2 *>(pb[u]) : zero2;
    }
    for (int kc = 0; kc < kext; kc += 8) {
        d2 ac[4], bc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { ac[u] = an[u]; bc[u] = bn[u]; }
        if (kc + 8 < kext) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                an[u] = va[u] ? *reinterpret_cast<const d2 *>(pa[u] + kc + 8) : zero2;
                bn[u] = vb[u] ? *reinterpret_cast<const d2 *>(pb[u] + kc + 8) : zero2;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[u][v] = mfma16x16x4(ac[u].x, bc[v].x, acc[u][v]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[u][v] = mfma16x16x4(ac[u].y, bc[v].y, acc[u][v]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int a = a0 + 16 * u + q + 4 * g;
            if (a >= p) continue;
            const int sa = a / d.P;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int b = b0 + 16 * v + r;
                if (b > a || b >= p) continue;
                const double coef = (b / d.P == sa) ? 1.0 : d.rho;
                double val = coef * acc[u][v][g] * inv_eff;
                if (a == b) val += wsum[a] * inv_eff;
                Sig[(size_t)a * p + b] += val;
            }
        }
    }
}

// Sigma[a][b] = Sigma[b][a] for a < b (lower -> upper), 32x32 LDS tiles
__global__ __launch_bounds__(256) void k_mirror(double *__restrict__ S, int p) {
    __shared__ double tile[32][33];
    const int tr = blockIdx.y, tc = blockIdx.x;   // destination tile (upper: tr <= tc)
    if (tr > tc) return;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int yy = ty; yy < 32; yy += 8) {
        const int sr = tc * 32 + yy, sc = tr * 32 + tx;   // source lower tile (tc, tr)
        tile[yy][tx] = (sr < p && sc < p) ? S[(size_t)sr * p + sc] : 0.0;
    }
    __syncthreads();
    for (int yy = ty; yy < 32; yy += 8) {
        const int dr = tr * 32 + yy, dc = tc * 32 + tx;
        if (dr < p && dc < p && dr < dc) S[(size_t)dr * p + dc] = tile[tx][yy];
    }
}

__global__ __launch_bounds__(256) void k_eta(Dims d, const double *__restrict__ X,
                                             const double *__restrict__ Z, double *__restrict__ eta) {
    const size_t total = (size_t)d.G * d.NP * KP;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
         e += (size_t)gridDim.x * blockDim.x) {
        const size_t ik = e % ((size_t)d.NP * KP);
        eta[e] = eta_of(d.sr, d.s1r, X[ik], Z[e]);
    }
}

__global__ __launch_bounds__(256) void k_rng_fill(uint64_t seed, int kind, double shape, int site,
                                                  int shard, int64_t iter, int64_t count,
                                                  double *__restrict__ out) {
    const Rng rng(seed);
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < count;
         e += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t row = (uint32_t)(e / 32), k = (uint32_t)(e % 32);
        out[e] = kind == 0 ? rng.normal(site, shard, row, k, (uint32_t)iter)
                           : rng.gamma(shape, site, shard, row, k, (uint32_t)iter);
    }
}

// ============================================================================
// launchers
// ============================================================================
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

void launch_prep(const Dims &d, const Bufs &b, hipStream_t s) {
    hipLaunchKernelGGL(k_prep, dim3(d.G), dim3(256), 0, s, d, b.Lam, b.omega, b.A, b.R, b.Rdi);
}
void launch_wpass(const Dims &d, const Bufs &b, hipStream_t s) {
    hipLaunchKernelGGL(k_wpass, dim3((d.NP / 128) * d.G), dim3(256), 0, s, d, b.Y, b.Lam, b.omega, b.W);
}
void launch_zdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    hipLaunchKernelGGL(k_zdraw, dim3(cdiv(d.NP, 256), d.G), dim3(256), 0, s, d, b.W, b.A, b.R, b.Rdi, b.X,
                       b.Z, b.Sp, dr, iter);
}
void launch_xred(const Dims &d, const Bufs &b, hipStream_t s) {
    const int total = (d.NP + KP) * KP;
    hipLaunchKernelGGL(k_xred, dim3(cdiv(total, 256)), dim3(256), 0, s, d, b.Sp, b.A, b.xin);
}
void launch_xdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    hipLaunchKernelGGL(k_xdraw, dim3(cdiv(d.n, 64)), dim3(64), 0, s, d, b.xall, b.X, dr, iter);
}
void launch_cpass(const Dims &d, const Bufs &b, hipStream_t s) {
    const int nt = (d.PP + KP) / 32;
    hipLaunchKernelGGL(k_cpass, dim3(nt * d.G), dim3(256), 0, s, d, b.Y, b.X, b.Z, b.C, b.E);
}
void launch_lambda(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter,
                   const double *tau_cur, hipStream_t s) {
    hipLaunchKernelGGL(k_lambda, dim3(cdiv(d.P, 8), d.G), dim3(256), 0, s, d, b.C, b.E, b.yy, tau_cur,
                       b.Lam, b.psi, b.Plam, b.ps, b.omega, b.cpart, dr, iter);
}
void launch_colsum(const Dims &d, const Bufs &b, hipStream_t s) {
    hipLaunchKernelGGL(k_colsum, dim3(d.G), dim3(256), 0, s, d, b.cpart, b.sloc);
}
void launch_delta(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter,
                  const double *delta_in, const double *tau_in, double *delta_out, double *tau_out,
                  hipStream_t s) {
    hipLaunchKernelGGL(k_delta, dim3(d.g), dim3(256), 0, s, d, b.sall, delta_in, tau_in, delta_out,
                       tau_out, b.psi, b.Plam, dr, iter);
}
void launch_save(const Dims &d, const Bufs &b, int slot, hipStream_t s) {
    const size_t total = (size_t)d.G * d.P * d.K;
    const int grid = (int)std::min<size_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_save, dim3(grid), dim3(256), 0, s, d, b.Lam, b.omega, b.Lb, b.wsum, b.LDB, slot);
}
void launch_assemble(const Dims &d, const Bufs &b, int kext, double inv_eff, hipStream_t s) {
    if (b.ntiles == 0) return;
    hipLaunchKernelGGL(k_assemble, dim3(b.ntiles), dim3(256), 0, s, d, b.Lb, b.LDB, kext, b.wsum,
                       inv_eff, b.tiles, b.Sigma);
}
void launch_mirror(double *S, int p, hipStream_t s) {
    const int nt = cdiv(p, 32);
    hipLaunchKernelGGL(k_mirror, dim3(nt, nt), dim3(256), 0, s, S, p);
}
void launch_eta(const Dims &d, const Bufs &b, double *eta_out, hipStream_t s) {
    const size_t total = (size_t)d.G * d.NP * KP;
    const int grid = (int)std::min<size_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_eta, dim3(grid), dim3(256), 0, s, d, b.X, b.Z, eta_out);
}
void launch_rng_fill(uint64_t seed, int kind, double shape, int site, int shard, int64_t iter,
                     int64_t count, double *out, hipStream_t s) {
    const int grid = (int)std::min<int64_t>((count + 255) / 256, 8192);
    hipLaunchKernelGGL(k_rng_fill, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, seed, kind, shape, site,
                       shard, iter, count, out);
}

}  // namespace dcfm
