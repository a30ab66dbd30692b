// Residual-precision update by the reference's own formula for every loading row, as a launch of
// its own after the loading-row kernel (DCFM_FLAG_EXACT_RESIDUAL), or (K > 32, default mode) for the
// 32-row tiles whose SS identity k_lambda_w's guard rejected (k_resid_flagged).  The default K <= 32
// chain runs the same arithmetic per wave inside k_lambda where its guard rejects the identity
// (lambda.h, resid_rows8).
//
// The default chain forms SS_j = sum_i Ytil_ij^2 inside the loading-row kernel by the identity
// yy_j - 2 lambda_j.C_j + lambda_j E lambda_j' (no Y pass).  That sum cancels when SS_j is
// small against its terms: its rounding error grows like kappa_j eps with kappa_j = (yy_j +
// 2 sum_k |lambda_jk C_jk| + |lambda_j| |E| |lambda_j|') / SS_j (measured ~1e6 at the second
// iteration of config c2, where the X excursions make E large: 1.3e-10 relative in SS).  The
// direct residual's error grows like sqrt(kappa_j) eps.  k_resid overwrites ps and omega from the
// direct residual (resid.h): a pass over the tile's Y columns, the reference's own third product.
//
// k_resid<KW>: block = (32-column tile of shard m's loading rows, shard m), resid_tile's 4 waves.
#include <algorithm>

#include "resid.h"

namespace dcfm {

template <int KW>
__global__ __launch_bounds__(256) void k_resid(Dims d, const double *__restrict__ Y, const double *__restrict__ X,
                                               const double *__restrict__ Z, const double *__restrict__ Lam,
                                               const double *__restrict__ Gps, double *__restrict__ ps,
                                               double *__restrict__ omega) {
    __shared__ double red[4][32];
    resid_tile<KW>(d, Y, X, Z, Lam, Gps, ps, omega, blockIdx.y, blockIdx.x * 32, red);
}

// k_resid64 (K <= 32, DCFM_FLAG_EXACT_RESIDUAL): block = (64 loading rows j0 .. j0+63 of shard m) x
// RW waves; wave w takes the 16-row chunks ch = w, w + RW, ... of i.  Per chunk a wave forms Ytil
// for 16 rows x 64 columns as four independent fp64 MFMA chains (column tiles h = 0..3, the Y
// values the accumulator input, -eta the shared A operand: the subtraction of dc:169 inside the
// accumulation), with the next chunk's Y, X and Z loads in flight behind them; lane (c, q) squares
// Ytil for rows i0 + q + 4v of columns j0 + 16h + c into its sums.  The 4 lanes of a column, then
// the RW waves, are summed in a fixed order.  (resid_tile's 32-column tiles ran two chains per
// wave: 65 us at c3 against this kernel's four.)
#ifndef DCFM_RESID_RW
#define DCFM_RESID_RW 4
#endif
#ifndef DCFM_RESID_LDSB
#define DCFM_RESID_LDSB 0
#endif
#ifndef DCFM_RESID_WPE
#define DCFM_RESID_WPE 2
#endif
constexpr int RW = DCFM_RESID_RW;
__global__ __launch_bounds__(64 * RW) __attribute__((amdgpu_waves_per_eu(DCFM_RESID_WPE))) void k_resid64(
    Dims d, const double *__restrict__ Y, const double *__restrict__ X, const double *__restrict__ Z,
    const double *__restrict__ Lam, const double *__restrict__ Gps, double *__restrict__ ps,
    double *__restrict__ omega) {
    __shared__ double red[RW][64];
    __shared__ __attribute__((aligned(16))) double Ls[64][KP + 2];   // Lambda rows j0 .. j0+63 (B operands)
    const int m = blockIdx.y, j0 = blockIdx.x * 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 15, q = lane >> 4;
    for (int e = threadIdx.x; e < 64 * (KP / 2); e += 64 * RW) {
        const int r = e / (KP / 2), k2 = 2 * (e % (KP / 2)), j = j0 + r;
        d2 v = {0.0, 0.0};
        if (j < d.PP) v = *reinterpret_cast<const d2 *>(Lam + ((size_t)m * d.PP + j) * KP + k2);
        *reinterpret_cast<d2 *>(&Ls[r][k2]) = v;
    }
    // column tile h holds columns jc(h) = 32 (h >> 1) + 2c + (h & 1) of the group: a lane's columns of tiles
    // 2hp and 2hp + 1 are adjacent, one 16-byte Y load; PP is a multiple of 32, so a pair is valid whole
    auto jc = [&](int h) { return 32 * (h >> 1) + 2 * c + (h & 1); };
    int ho[2];
#pragma unroll
    for (int hp = 0; hp < 2; ++hp) ho[hp] = (j0 + 32 * hp < d.PP) ? 32 * hp : 0;   // invalid: re-read pair 0
    __syncthreads();
#if !DCFM_RESID_LDSB
    d2 lb[4][4];   // B operands Lambda[j0 + 16h + c][8t + 2q .. +1], register-resident for the block
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int t = 0; t < 4; ++t) lb[h][t] = *reinterpret_cast<const d2 *>(&Ls[jc(h)][8 * t + 2 * q]);
#endif
    // Y of the block as a buffer resource: one 32-bit offset per row, the column tiles as offsets
    // (64-bit addresses per load cost two VGPRs each and made hipcc spill)
    const auto ysrc = __builtin_amdgcn_make_buffer_rsrc((void *)(Y + (size_t)m * d.NP * d.PP + j0), (short)0,
                                                        (int)(((size_t)d.NP * d.PP - j0) * 8), 0x00020000);
    const double *Zm = Z + (size_t)m * d.NP * KP + 2 * q;
    const double *Xq = X + 2 * q;
    double ss[4] = {0.0, 0.0, 0.0, 0.0};
    // Y of the next chunk is loaded a chunk ahead (two register sets); X and Z of the next chunk as soon
    // as this chunk's eta is formed (their registers are free then), so both are in flight behind the MFMAs
    double yA[4][4], yB[4][4];
    d2 xv[4], zv[4];
    auto load_y = [&](int ch, double (&y)[4][4]) {
        const int i0 = 16 * ch;
#pragma unroll
        for (int v = 0; v < 4; ++v) {   // unconditional loads: an invalid column pair (j >= PP) re-reads pair 0
            const uint32_t ro = (uint32_t)((i0 + q + 4 * v) * d.PP + 2 * c) * 8u;
#pragma unroll
            for (int hp = 0; hp < 2; ++hp) {
                const d2 yv = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(ysrc, ro + 8u * ho[hp], 0, 0));
                y[2 * hp][v] = yv.x;
                y[2 * hp + 1][v] = yv.y;
            }
        }
    };
    auto load_xz = [&](int ch) {
        const int i0 = 16 * ch;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            xv[t] = *reinterpret_cast<const d2 *>(Xq + (size_t)(i0 + c) * KP + 8 * t);
            zv[t] = *reinterpret_cast<const d2 *>(Zm + (size_t)(i0 + c) * KP + 8 * t);
        }
    };
    const int nch = d.NP / 16;
    if (w < nch) {
        load_y(w, yA);
        load_xz(w);
    }
#pragma unroll 1
    for (int ch = w; ch < nch; ch += RW) {
        double e[4][2];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            e[t][0] = -eta_of(d.sr, d.s1r, xv[t].x, zv[t].x);
            e[t][1] = -eta_of(d.sr, d.s1r, xv[t].y, zv[t].y);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bool more = ch + RW < nch;
        if (more) {
            load_xz(ch + RW);
            load_y(ch + RW, yB);
        }
        __builtin_amdgcn_sched_barrier(0);
        d4 acc[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) acc[h] = d4{yA[h][0], yA[h][1], yA[h][2], yA[h][3]};   // invalid tiles: unused sums
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#if DCFM_RESID_LDSB   // B operands read from the LDS image per k-step (64 fewer VGPRs: 3 waves per SIMD)
            d2 lt[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) lt[h] = *reinterpret_cast<const d2 *>(&Ls[jc(h)][8 * t + 2 * q]);
#pragma unroll
            for (int h = 0; h < 4; ++h) acc[h] = mfma16x16x4(e[t][0], lt[h].x, acc[h]);
#pragma unroll
            for (int h = 0; h < 4; ++h) acc[h] = mfma16x16x4(e[t][1], lt[h].y, acc[h]);
#else
#pragma unroll
            for (int h = 0; h < 4; ++h) acc[h] = mfma16x16x4(e[t][0], lb[h][t].x, acc[h]);
#pragma unroll
            for (int h = 0; h < 4; ++h) acc[h] = mfma16x16x4(e[t][1], lb[h][t].y, acc[h]);
#endif
        }
        const int i0 = 16 * ch;
#pragma unroll
        for (int h = 0; h < 4; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) ss[h] = (i0 + q + 4 * v < d.n) ? fma(acc[h][v], acc[h][v], ss[h]) : ss[h];
#pragma unroll
        for (int h = 0; h < 4; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) yA[h][v] = yB[h][v];
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) {   // the column's 4 lane rows: (q0 + q1) + (q2 + q3)
        ss[h] += xor16_d(ss[h]);
        ss[h] += xor32_d(ss[h]);
        if (q == 0) red[w][jc(h)] = ss[h];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int t = threadIdx.x, j = j0 + t;
        double SS = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
        if constexpr (RW == 8) SS += (red[4][t] + red[5][t]) + (red[6][t] + red[7][t]);
        if (j < d.P) {
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps[(size_t)m * d.P + j];   // dc:170
            ps[(size_t)m * d.PP + j] = psn;
            omega[(size_t)m * d.PP + j] = 1.0 / psn;                                  // dc:171 (Q1)
        }
    }
}
static_assert(RW == 4 || RW == 8, "k_resid64's wave tree is written for 4 or 8 waves");

// K > 32 default mode: only the 32-row tiles whose guard k_lambda_w tripped (b.rflag); a flag is
// read by every thread before resid_tile's barrier and cleared by thread 0 after it
template <int KW>
__global__ __launch_bounds__(256) void k_resid_flagged(Dims d, const double *__restrict__ Y, const double *__restrict__ X,
                                                       const double *__restrict__ Z, const double *__restrict__ Lam,
                                                       const double *__restrict__ Gps, double *__restrict__ ps,
                                                       double *__restrict__ omega, int *__restrict__ rflag) {
    __shared__ double red[4][32];
    const int nt = d.PP / 32;
    for (int t = blockIdx.x; t < nt; t += gridDim.x) {   // a few blocks per shard walk its tiles
        int *f = rflag + blockIdx.y * nt + t;
        if (*f == 0) continue;                            // block-uniform
        resid_tile<KW>(d, Y, X, Z, Lam, Gps, ps, omega, blockIdx.y, t * 32, red);
        if (threadIdx.x == 0) *f = 0;
        __syncthreads();                                  // red is reused by the next flagged tile
    }
}

void launch_resid_flagged(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    const double *Gps = dr.Gps + ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
    // tiles are flagged rarely (the reference's transients and excursions): 16 blocks per shard walk them
    // (one block per tile cost ~6 us of dispatch per iteration at c4 with every block exiting at once)
    const dim3 grid(std::min(d.PP / 32, 16), d.G);
    switch (d.kp) {
    case 64: hipLaunchKernelGGL(k_resid_flagged<64>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega, b.rflag); break;
    default: hipLaunchKernelGGL(k_resid_flagged<128>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega, b.rflag); break;
    }
}

void launch_resid(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s, bool gen) {
    const double *Gps;
    if (gen) Gps = lam_gen_plan(d, b.ldraw).Gps;   // the generated fused chain: k_wcol's buffer
    else Gps = dr.Gps + ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
    if (d.kp == KP && (size_t)d.NP * d.PP * 8 < ((size_t)1 << 31)) {   // k_resid64's buffer offsets are 32-bit
        hipLaunchKernelGGL(k_resid64, dim3((d.PP + 63) / 64, d.G), dim3(64 * RW), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps,
                           b.ps, b.omega);
        return;
    }
    const dim3 grid(d.PP / 32, d.G);
    switch (d.kp) {
    case 32: hipLaunchKernelGGL(k_resid<32>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    case 64: hipLaunchKernelGGL(k_resid<64>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    default: hipLaunchKernelGGL(k_resid<128>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    }
}

}  // namespace dcfm
