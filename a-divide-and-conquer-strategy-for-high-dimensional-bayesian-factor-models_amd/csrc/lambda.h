// Loading-row kernel of the narrow (K <= 32) chain and the generator of its variates
// (divideconquer.m:140-145, 150, 156, 169-171), included by kernels.hip.
#pragma once
#include "dcfm_internal.h"
#include "philox.h"
#include "linalg.h"

namespace dcfm {

// The loading-row variates of one iteration (dc:142 zlam, dc:150 psi gammas, dc:170 ps
// gamma) into k_lambda's buffer layout, at the counters every other path draws them from
// (k_draws, dcfm_rng_fill).  Runs as extra blocks of k_wcol (behind the W tiles) so the
// loading-row kernel reads its variates instead of drawing them.  Thread gtid of gthreads walks
// each index range — ps gammas (m, j), psi gammas (m, j, k), normal pairs (m, j, pair) — grid-
// stride, LAM_ILP independent variates per step: one variate is a chain of dependent Philox
// rounds and transcendental steps, so a thread drawing them one after another is latency-bound
// (block stamps at c3: 160 such blocks took 35 us alone, the long pole of k_wcol); the
// branch-free shapes (psi gammas of integer shape, Box-Muller pairs) run LAM_ILP chains side by
// side.  Every variate keeps its counter and formula: the same values as rng.gamma / normal2.
#ifndef DCFM_LAM_ILP
#define DCFM_LAM_ILP 4
#endif
constexpr int LAM_ILP = DCFM_LAM_ILP;
__device__ __forceinline__ void lam_draws(const Dims &d, const LamGen &lg, int64_t iter, int gtid, int gthreads) {
    const Rng rng(d.seed);
    const uint32_t it = (uint32_t)iter;
    const int kp2 = (d.K + 1) / 2;
    for (int x = gtid; x < lg.n_ps; x += gthreads) {   // (m, j): Marsaglia-Tsang, rejection loop
        const int m = x / d.P, j = x - m * d.P;
        lg.Gps[x] = rng.gamma(d.as_ + 0.5 * d.n, SITE_PS, (uint32_t)(d.shard0 + m), (uint32_t)j, 0u, it);
    }
    const double sh = d.df * 0.5 + 0.5;
    const int npsi = lg.n_psi - lg.n_ps;
    if (sh == 1.0 || sh == 2.0) {   // rng.gamma's integer-shape branch: -log(u1 [* u2]), no rejection
        for (int y0 = gtid; y0 < npsi; y0 += LAM_ILP * gthreads) {
            double u[LAM_ILP];
#pragma unroll
            for (int t = 0; t < LAM_ILP; ++t) {
                const int y = y0 + t * gthreads, yc = y < npsi ? y : 0;
                const int mj = yc / d.K, k = yc - mj * d.K, m = mj / d.P, j = mj - m * d.P;
                const u32x4 a = rng.raw(SITE_PSI, (uint32_t)(d.shard0 + m), (uint32_t)j,
                                        0x80000000u | (((uint32_t)k & 0x7FFFFFu) << 8), it);
                const double u1 = u01_53(a.x, a.y);
                u[t] = sh == 1.0 ? u1 : u1 * u01_53(a.z, a.w);
            }
#pragma unroll
            for (int t = 0; t < LAM_ILP; ++t) {
                const int y = y0 + t * gthreads;
                const double gv = -log_u01(u[t]);
                if (y < npsi) lg.Gpsi[y] = gv;
            }
        }
    } else {
        for (int y = gtid; y < npsi; y += gthreads) {   // (m, j, k)
            const int mj = y / d.K, k = y - mj * d.K, m = mj / d.P, j = mj - m * d.P;
            lg.Gpsi[y] = rng.gamma(sh, SITE_PSI, (uint32_t)(d.shard0 + m), (uint32_t)j, (uint32_t)k, it);
        }
    }
    const int nnp = lg.n_all - lg.n_psi;
    for (int y0 = gtid; y0 < nnp; y0 += LAM_ILP * gthreads) {   // (m, j, pair)
        double n0[LAM_ILP], n1[LAM_ILP];
#pragma unroll
        for (int t = 0; t < LAM_ILP; ++t) {
            const int y = y0 + t * gthreads, yc = y < nnp ? y : 0;
            const int mj = yc / kp2, q = yc - mj * kp2, m = mj / d.P, j = mj - m * d.P;
            rng.normal2(SITE_LAMBDA, (uint32_t)(d.shard0 + m), (uint32_t)j, (uint32_t)q, it, n0[t], n1[t]);
        }
#pragma unroll
        for (int t = 0; t < LAM_ILP; ++t) {
            const int y = y0 + t * gthreads;
            if (y < nnp) {
                const int mj = y / kp2, q = y - mj * kp2;
                double *o = lg.NL + (size_t)mj * d.K + 2 * q;
                o[0] = n0[t];
                if (2 * q + 1 < d.K) o[1] = n1[t];
            }
        }
    }
}

// ============================================================================
// k_lambda: loading rows.                                   dc:140-145 (+150,156,169-171)
// One wave = 8 loading rows j of shard m; an aligned 8-lane group owns one row's K x K
// system: lane l holds rows r_b = l + 8b of the system in registers, row r_b only up to
// column min(8b + 7, KE - 1) (the lower triangle, compile-time pruned; KE = K rounded up to
// an instantiated width, rows >= K identity padding).
//   * Q_j = ps_j E_m + diag(Plam_j) (dc:141) is factored as ps_j (E_m + diag(Plam_j / ps_j)):
//     L_Q = sqrt(ps_j) L, so E_m enters unscaled (staged once per wave in LDS: 8 dwordx4 global
//     loads per lane, the 8 groups then read it as LDS broadcasts), the rhs of the forward solve
//     is sqrt(ps_j) C_j (= L_Q v = b, dc:143 vlam) and Lambda_j = L^{-T} (v + z) / sqrt(ps_j)
//     (dc:143-144 mlam + ylam).
//   * Pivots two at a time: each group writes the current column pair of its rows (and the
//     rhs) to an LDS image; every lane reads the 2x2 pivot block from it and forms the rank-2
//     update q[c] -= alpha Q[c][k] + beta Q[c][k+1] of its rows from the unnormalised image
//     (one LDS round per pair).  The image is double-buffered: the next pair's columns are
//     updated first and written to the other buffer, so the next pivots' LDS round trip and
//     rsqrt chain overlap the rest of this pair's update, whose image reads are issued a batch
//     of LAM_PIPE columns ahead of their FMAs.
//   * Back solve L' x = w from the bottom, the sums over the group's rows as 8-lane DPP sums.
//   * psi_j (dc:150, tau of the previous iteration), SS_j = yy_j - 2 x.C_j + x'E x with
//     x'E x = (|w|^2 - sum_r Plam_jr x_r^2) / ps_j and ps_j x.C_j = w.v (no third Y pass, no
//     second read of E or C), ps_j and omega_j (dc:169-171), psi o Lambda^2 -> cpart (dc:156).
// Plam_j = psi_j o tau' (dc:176) is formed from the previous iteration's psi and tau unless
// plam_src is given (first iteration after dcfm_set_state).  The row's variates (dc:142, 150,
// 170) come from a draw buffer: the generated chain's k_wcol draws them (lam_draws),
// injected draws and the k_draws batches are read in place.
// ============================================================================
// DPP moves within the aligned 8-lane group (every source lane of these patterns is valid)
template <int CTRL>
__device__ __forceinline__ double dpp8_d(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
// sum over the aligned 8-lane group (identical bits in every lane: each stage adds a
// commutative pair)
__device__ __forceinline__ double rowsum8(double v) {
    v += dpp8_d<0xB1>(v);     // quad_perm [1,0,3,2]
    v += dpp8_d<0x4E>(v);     // quad_perm [2,3,0,1]
    v += dpp8_d<0x141>(v);    // row_half_mirror: the other quad of the 8
    return v;
}

constexpr int LAM_ROWS = 8;   // loading rows per wave

// dc:169-171 as written for the wave's 8 loading rows j0 .. j0+7 (the guard below, or the exact
// mode): Ytil = Yd - eta Lambda' as fp64 MFMA v_mfma_f64_16x16x4 over 16-row chunks of i, the Y
// values as the accumulator input and -eta as the A operand (the subtraction of dc:169 inside the
// accumulation); B = the rows' Lambda from the LDS image Lm (columns 8..15 of the tile zero); lane
// (c, q) holds Ytil for rows i0 + q + 4v of loading row j0 + c and squares them into its sum, the
// 4 lanes of a row then summed in a fixed order.  ps_j, omega_j with the row's gamma variate Gps.
__device__ __forceinline__ void resid_rows8(const Dims &d, const double *__restrict__ Y,
                                            const double *__restrict__ X, const double *__restrict__ Z,
                                            const double (*Lm)[KP + 1], double Gps_c, int m, int j0, int lane,
                                            double *__restrict__ ps, double *__restrict__ omega) {
    constexpr int NT = KP / 8;
    const int c = lane & 15, q = lane >> 4;
    const bool col = c < LAM_ROWS && j0 + c < d.P;
    d2 lb[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        lb[t].x = col ? Lm[c][8 * t + 2 * q] : 0.0;
        lb[t].y = col ? Lm[c][8 * t + 2 * q + 1] : 0.0;
    }
    const double *Ym = Y + (size_t)m * d.NP * d.PP + (col ? j0 + c : 0);
    const double *Zm = Z + (size_t)m * d.NP * KP + 2 * q;
    double ss = 0.0;
    for (int i0 = 0; i0 < d.NP; i0 += 16) {
        d4 acc;
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[v] = col ? Ym[(size_t)(i0 + q + 4 * v) * d.PP] : 0.0;
        const double *xr = X + (size_t)(i0 + c) * KP + 2 * q, *zr = Zm + (size_t)(i0 + c) * KP;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const d2 xa = *reinterpret_cast<const d2 *>(xr + 8 * t);
            const d2 za = *reinterpret_cast<const d2 *>(zr + 8 * t);
            acc = mfma16x16x4_na(eta_of(d.sr, d.s1r, xa.x, za.x), lb[t].x, acc);
            acc = mfma16x16x4_na(eta_of(d.sr, d.s1r, xa.y, za.y), lb[t].y, acc);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) ss = (i0 + q + 4 * v < d.n) ? fma(acc[v], acc[v], ss) : ss;   // data rows only
    }
    ss += xor16_d(ss);   // (q0 + q1) + (q2 + q3)
    ss += xor32_d(ss);
    if (q == 0 && col) {
        const double psn = (1.0 / (d.bs + 0.5 * ss)) * Gps_c;   // dc:170
        ps[(uint32_t)(m * d.PP + j0 + c)] = psn;
        omega[(uint32_t)(m * d.PP + j0 + c)] = 1.0 / psn;        // dc:171 (Q1)
    }
}
constexpr int LAM_PIPE = 4;   // image columns read ahead of their trailing-update FMAs
__host__ __device__ constexpr int lam_ncol(int KE, int b) { return 8 * b + 8 < KE ? 8 * b + 8 : KE; }

// pivot pair (k, k+1) from the image: 2x2 Cholesky block, the forward-solve entries and the
// coefficients the rows' updates need
struct LamPiv { double i00, i11, l10, v0, v1, t10; };
__device__ __forceinline__ LamPiv lam_pivots(d2 pk, d2 pk1, d2 bb) {
    LamPiv p;
    const double a = pk.x, bq = pk1.x, c2 = pk1.y;
    p.i00 = rsqrt_f64(a);
    p.l10 = bq * p.i00;
    const double d11 = c2 - p.l10 * p.l10;
    p.i11 = rsqrt_f64(d11);
    p.v0 = bb.x * p.i00;
    p.v1 = (bb.y - p.l10 * p.v0) * p.i11;
    p.t10 = p.l10 * p.i11;
    return p;
}

template <int KE>
// waves_per_eu(2): the residual fixup's MFMA accumulator must share the row path's 250 VGPRs (left
// alone, hipcc put it in AGPRs: 258 registers, one wave per SIMD)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_lambda(Dims d, const double *__restrict__ C, const double *__restrict__ E,
                                               const double *__restrict__ yy, const double *__restrict__ tau_cur,
                                               double *__restrict__ Lam, double *__restrict__ psi,
                                               const double *__restrict__ plam_src, double *__restrict__ ps,
                                               double *__restrict__ omega, double *__restrict__ cpart,
                                               LamDraws ld, const double *__restrict__ Y,
                                               const double *__restrict__ X, const double *__restrict__ Z,
                                               double kappa_max) {
    static_assert(KE % 2 == 0 && KE >= 2 && KE <= KP, "even factor width");
    constexpr int NB = (KE + 7) / 8;
    // LDS: double-buffered image [2][8 systems][KP + 1 (bank spread)][2] | rhs image [2][8][KP+2] |
    // per system v and 1 / L_kk [8][KP+2] each; E_m is staged (row pitch EP) in the image area first
    constexpr int LSN = 2 * LAM_ROWS * (KP + 1) * 2, BSN = 2 * LAM_ROWS * (KP + 2), VSN = LAM_ROWS * (KP + 2);
    constexpr int EP = KP + 2;
    static_assert(KP * EP <= LSN + BSN, "E staging fits the image area");
    __shared__ __attribute__((aligned(16))) double SM[LSN + BSN + 2 * VSN + KP];   // + sqrt(diag E_m): the guard
    double(*LS)[LAM_ROWS][KP + 1][2] = reinterpret_cast<double(*)[LAM_ROWS][KP + 1][2]>(SM);
    double(*BS)[LAM_ROWS][KP + 2] = reinterpret_cast<double(*)[LAM_ROWS][KP + 2]>(SM + LSN);
    double *Vs = SM + LSN + BSN, *Is = Vs + VSN;
    double *Dg = SM + LSN + BSN + 2 * VSN;          // E_m[k][k]
    double *Es = SM;
    const int m = blockIdx.y, mg = d.shard0 + m;
    const int lane = threadIdx.x, grp = lane >> 3, l = lane & 7;
    Vs += grp * (KP + 2);
    Is += grp * (KP + 2);
    const int j0 = blockIdx.x * LAM_ROWS;   // the wave's first loading row
    const int j = j0 + grp;
    const bool valid = j < d.P;
    const int jj = valid ? j : 0;
    const uint32_t rowoff = (uint32_t)(m * d.PP + jj) * KP, toff = (uint32_t)mg * KP;
    bool rv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) rv[b] = valid && l + 8 * b < d.K;
    {   // E_m rows < 8 NB (every row a lane of the group holds, identity-padding rows >= K included:
        // E is zero there; an unstaged row would leave stale LDS in registers that the back solve
        // multiplies by x = 0, and NaN * 0 is NaN): lane t moves pairs 2t + 128 i
        const double *Em = E + (uint32_t)m * KP * KP;
        constexpr int NI = (8 * NB * KP + 127) / 128;
        d2 e[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) e[i] = *reinterpret_cast<const d2 *>(Em + 2 * lane + 128 * i);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int f = 2 * lane + 128 * i, r = f >> 5, c = f & 31;
            *reinterpret_cast<d2 *>(Es + r * EP + c) = e[i];
        }
    }
    const double psj = valid ? ps[(uint32_t)(m * d.PP + jj)] : 1.0;
    const double isj = rsqrt_f64(psj), sj = psj * isj;     // 1 / sqrt(ps_j), sqrt(ps_j)
    const double ipsj = isj * isj;
    const double *pin = plam_src ? plam_src : psi;
    double dg[4], bv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const double pv = pin[rowoff + l + 8 * b], tv = tau_cur[toff + l + 8 * b], cv = C[rowoff + l + 8 * b];
        dg[b] = rv[b] ? (plam_src ? pv : pv * tv) * ipsj : 1.0;   // Plam_j / ps_j; identity padding
        bv[b] = valid ? sj * cv : 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    double q0[lam_ncol(KE, 0)], q1[NB > 1 ? lam_ncol(KE, 1) : 1], q2[NB > 2 ? lam_ncol(KE, 2) : 1],
        q3[NB > 3 ? lam_ncol(KE, 3) : 1];
    auto qref = [&](auto NBc) -> auto & {
        constexpr int b = decltype(NBc)::value;
        if constexpr (b == 0) return q0;
        else if constexpr (b == 1) return q1;
        else if constexpr (b == 2) return q2;
        else return q3;
    };
    static_for<NB>([&](auto NBc) {
        constexpr int b = decltype(NBc)::value, nc = lam_ncol(KE, b);
        auto &q = qref(NBc);
        const double *Er = Es + (l + 8 * b) * EP;
#pragma unroll
        for (int c = 0; c < nc; c += 2) {
            const d2 e = *reinterpret_cast<const d2 *>(Er + c);
            q[c] = e.x;
            q[c + 1] = e.y;
        }
        // the diagonal entry of this lane's row: selects on the lane, no branch per column (a
        // conditional per column compiled to an exec-mask branch around an LDS store each)
        double e_kk = 0.0;
#pragma unroll
        for (int c = 8 * b; c < nc; ++c) {
            const bool dgl = c == l + 8 * b;
            e_kk = dgl ? q[c] : e_kk;
            q[c] = dgl ? q[c] + dg[b] : q[c];
        }
        if (grp == 0 && l + 8 * b < nc) Dg[l + 8 * b] = e_kk;   // E_m[k][k] (the wave's, whatever the row)
    });
    __builtin_amdgcn_wave_barrier();
    // image of column pair (0, 1) (overwrites E's staging: every read of it is above)
    static_for<NB>([&](auto NBc) {
        constexpr int b = decltype(NBc)::value;
        auto &q = qref(NBc);
        d2 v;
        v.x = q[0];
        v.y = q[1];
        *reinterpret_cast<d2 *>(LS[0][grp][l + 8 * b]) = v;
        BS[0][grp][l + 8 * b] = bv[b];
    });
    __builtin_amdgcn_wave_barrier();
    LamPiv pv = lam_pivots(*reinterpret_cast<const d2 *>(LS[0][grp][0]), *reinterpret_cast<const d2 *>(LS[0][grp][1]),
                           *reinterpret_cast<const d2 *>(&BS[0][grp][0]));
    // ---- factorisation (dc:142 Llam = chol(Qlam,'lower')), forward solve fused
    static_for<KE / 2>([&](auto JC) {
        constexpr int k = 2 * decltype(JC)::value, cur = decltype(JC)::value & 1, nxt = cur ^ 1;
        constexpr int cb = k / 8, kk = k % 8;
        double(*Ls)[2] = LS[cur][grp];
        const LamPiv p = pv;
        {   // every lane of the group stores the same values: no exec-mask branch
            d2 v, iv;
            v.x = p.v0; v.y = p.v1; iv.x = p.i00; iv.y = p.i11;
            *reinterpret_cast<d2 *>(Vs + k) = v;
            *reinterpret_cast<d2 *>(Is + k) = iv;
        }
        // the rows' L entries of the pair, their update coefficients and forward-solve rhs;
        // rows k and k+1 get their own entries from the same formulas (l00 = a i00, l10, l11 =
        // d11 i11), only rows below the pair update their trailing columns
        double al[4] = {0.0, 0.0, 0.0, 0.0}, be[4] = {0.0, 0.0, 0.0, 0.0};
        static_for<NB>([&](auto NBc) {
            constexpr int b = decltype(NBc)::value;
            if constexpr (b >= cb) {
                auto &q = qref(NBc);
                const double lr0 = q[k] * p.i00;
                const double lr1 = (q[k + 1] - lr0 * p.l10) * p.i11;
                const double a_ = p.i00 * fma(-lr1, p.t10, lr0), b_ = lr1 * p.i11;
                bv[b] = fma(-lr1, p.v1, fma(-lr0, p.v0, bv[b]));
                q[k] = lr0;
                if constexpr (b > cb) {
                    q[k + 1] = lr1;
                    al[b] = a_;
                    be[b] = b_;
                } else {
                    const bool below = l > kk + 1;
                    q[k + 1] = (l == kk) ? 0.0 : lr1;
                    al[b] = below ? a_ : 0.0;
                    be[b] = below ? b_ : 0.0;
                }
            }
        });
        if constexpr (k + 2 < KE) {
            constexpr int c0 = k + 2, cb2 = c0 / 8;
            // columns c0, c0+1 first: the next pair's image
            const d2 i2 = *reinterpret_cast<const d2 *>(Ls[c0]);
            const d2 i3 = *reinterpret_cast<const d2 *>(Ls[c0 + 1]);
            static_for<NB>([&](auto NBc) {
                constexpr int b = decltype(NBc)::value;
                if constexpr (b >= cb2) {
                    auto &q = qref(NBc);
                    q[c0] = fma(-be[b], i2.y, fma(-al[b], i2.x, q[c0]));
                    q[c0 + 1] = fma(-be[b], i3.y, fma(-al[b], i3.x, q[c0 + 1]));
                    d2 v;
                    v.x = q[c0];
                    v.y = q[c0 + 1];
                    *reinterpret_cast<d2 *>(LS[nxt][grp][l + 8 * b]) = v;
                    BS[nxt][grp][l + 8 * b] = bv[b];
                }
            });
            __builtin_amdgcn_wave_barrier();
            pv = lam_pivots(*reinterpret_cast<const d2 *>(LS[nxt][grp][c0]),
                            *reinterpret_cast<const d2 *>(LS[nxt][grp][c0 + 1]),
                            *reinterpret_cast<const d2 *>(&BS[nxt][grp][c0]));
            // the rest of the rank-2 update, image reads a batch ahead
            auto upd = [&](int c, d2 ic) {
                static_for<NB>([&](auto NBc) {
                    constexpr int b = decltype(NBc)::value;
                    if constexpr (b >= cb) {
                        auto &q = qref(NBc);
                        constexpr int nq = lam_ncol(KE, b);
                        if (c < nq) {
                            double &x = q[c < nq ? c : 0];
                            x = fma(-be[b], ic.y, fma(-al[b], ic.x, x));
                        }
                    }
                });
            };
            constexpr int cs = c0 + 2, nbt = (KE - cs + LAM_PIPE - 1) / LAM_PIPE;
            d2 buf[2][LAM_PIPE];
            static_for<LAM_PIPE>([&](auto T) {
                constexpr int c = cs + decltype(T)::value;
                if constexpr (c < KE) buf[0][decltype(T)::value] = *reinterpret_cast<const d2 *>(Ls[c]);
            });
            static_for<nbt>([&](auto Bt) {
                constexpr int bt = decltype(Bt)::value, cur_b = bt & 1;
                if constexpr (bt + 1 < nbt) {
                    static_for<LAM_PIPE>([&](auto T) {
                        constexpr int c = cs + (bt + 1) * LAM_PIPE + decltype(T)::value;
                        if constexpr (c < KE) buf[cur_b ^ 1][decltype(T)::value] = *reinterpret_cast<const d2 *>(Ls[c]);
                    });
                }
                __builtin_amdgcn_sched_barrier(0);
                static_for<LAM_PIPE>([&](auto T) {
                    constexpr int c = cs + bt * LAM_PIPE + decltype(T)::value;
                    if constexpr (c < KE) upd(c, buf[cur_b][decltype(T)::value]);
                });
                __builtin_amdgcn_sched_barrier(0);
            });
            // keep the trailing update eager: without this hipcc sinks each FMA to the step that
            // consumes it and keeps the image values live
            static_for<NB>([&](auto NBc) {
                constexpr int b = decltype(NBc)::value;
                if constexpr (b >= cb) {
                    auto &q = qref(NBc);
#pragma unroll
                    for (int c = c0; c < lam_ncol(KE, b); ++c) asm volatile("" : "+v"(q[c]));
                }
            });
        }
    });
    // ---- the row's variates (dc:142 zlam, dc:150, dc:170), Plam_j and tau for the epilogue
    double z[4], G[4], tv[4], pl2[4];
    const uint32_t dro = (uint32_t)(m * d.P + jj), dk = dro * (uint32_t)d.K;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t di = rv[b] ? dk + l + 8 * b : dk;
        z[b] = ld.NL[di];
        G[b] = ld.Gpsi[di];
        const double p2 = pin[rowoff + l + 8 * b];
        tv[b] = tau_cur[toff + l + 8 * b];
        pl2[b] = plam_src ? p2 : p2 * tv[b];
    }
    const double Gps = ld.Gps[dro];
    const double yyj = yy[(uint32_t)(m * d.PP + jj)];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        z[b] = rv[b] ? z[b] : 0.0;
        G[b] = rv[b] ? G[b] : 0.0;
        pl2[b] = rv[b] ? pl2[b] : 0.0;
        tv[b] = rv[b] ? tv[b] : 0.0;
    }
    // ---- back solve L' x = w, w = v + z (dc:143-144), pivots (c, c-1) from the bottom:
    //      x_c = (w_c - sum_{r>c} L[r][c] x_r) / L[c][c], the sums over the group's lanes
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    static_for<KE / 2>([&](auto JC) {
        constexpr int c = KE - 1 - 2 * decltype(JC)::value;     // odd; c and c-1 in block cb
        constexpr int cb = c / 8;
        double pa = 0.0, pb = 0.0;
        static_for<NB>([&](auto NBc) {
            constexpr int b = decltype(NBc)::value;
            if constexpr (b >= cb) {   // block cb: rows above c have x = 0 still
                auto &q = qref(NBc);
                pa = fma(q[c], x[b], pa);
                pb = fma(q[c - 1], x[b], pb);
            }
        });
        pa = rowsum8(pa);
        pb = rowsum8(pb);
        auto &qc = qref(std::integral_constant<int, cb>{});
        const d2 vv = *reinterpret_cast<const d2 *>(Vs + c - 1);
        const d2 iv = *reinterpret_cast<const d2 *>(Is + c - 1);
        const bool isc = l + 8 * cb == c, isc1 = l + 8 * cb == c - 1;
        double xa = (vv.y + z[cb] - pa) * iv.y;
        asm volatile("" : "+v"(xa));      // formed in every lane: hipcc otherwise sinks it into an exec-mask branch
        x[cb] = isc ? xa : x[cb];
        const double t = isc ? qc[c - 1] * xa : 0.0;               // L[c][c-1] x_c
        const double tb = dpp8_d<0x101>(t);                        // row_shl:1: lane c%8 -> c%8 - 1
        const double xb = (vv.x + z[cb] - pb - tb) * iv.x;
        x[cb] = isc1 ? xb : x[cb];
    });
    // ---- SS_j = yy_j - 2 x.C_j + x'E x (dc:169 by identity, no Y pass).  x = L_Q'^{-1} w, so
    //      x'Q_j x = |w|^2 and x'E x = (|w|^2 - sum_r Plam_jr x_r^2) / ps_j: no E re-read;
    //      ps_j x.C_j = x.blam = x.(L_Q v) = (L_Q'x).v = w.v: no C re-read.
    double ww = 0.0, wv = 0.0, wva = 0.0, px = 0.0, cs = 1.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int r = l + 8 * b < KE ? l + 8 * b : 0;
        const double vr = Vs[r];
        const double w = vr + z[b];
        ww = rv[b] ? fma(w, w, ww) : ww;
        wv = rv[b] ? fma(w, vr, wv) : wv;
        wva = rv[b] ? wva + fabs(w * vr) : wva;
        x[b] = rv[b] ? x[b] * isj : 0.0;                           // Lambda_j = L^{-T} w / sqrt(ps_j)
        px = fma(pl2[b] * x[b], x[b], px);
        // the pivot's share of its diagonal, Q_kk / L_kk^2 >= 1 (normalised system E + diag(Plam / ps))
        const double ik = Is[r];
        cs = rv[b] ? fmax(cs, (Dg[r] + pl2[b] * ipsj) * ik * ik) : cs;
    }
    double contrib = (ww - px - 2.0 * wv) * ipsj;
    contrib = valid ? contrib : 0.0;
    contrib = rowsum8(contrib);
    // ---- guard: the identity's rounding error is ~ kappa_j eps, kappa_j = (the magnitudes it sums) / SS_j.
    //      Two bounds on those magnitudes, the larger taken:
    //      * as computed: yy_j + (|w|^2 + sum_r Plam_jr x_r^2 + 2 sum_r |w_r v_r|) / ps_j, with |w|^2 weighted
    //        by 1 + c_j, c_j = max_k Q_kk / L_kk^2 (>= 1, scale-invariant): w = L'x holds only to the back
    //        solve's backward error, which grows with the elimination's loss of the diagonal;
    //      * a priori: yy_j + 2 sum_k |x_k C_jk| + |x|'|E||x| <= (sqrt(yy_j) + s_j)^2, s_j = sum_k |x_k|
    //        sqrt(E_kk) (|C_jk| <= sqrt(E_kk yy_j) and |E_kl| <= sqrt(E_kk E_ll), E a Gram matrix).
    //      Beyond kappa_max (or SS_j <= 0) the wave's 8 rows take dc:169's residual instead (resid_rows8).
    //      Square roots as v * rsq(v) from the hardware estimate (a bound needs no correct rounding; the
    //      factor 1.01 covers its error); a zero yy_j gives NaN, read as "take the residual"
    double sabs = 0.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const double e = Dg[l + 8 * b < KE ? l + 8 * b : 0];
        sabs = (rv[b] && e > 0.0) ? fma(fabs(x[b]), e * __builtin_amdgcn_rsq(e), sabs) : sabs;
    }
    cs = fmax(cs, dpp8_d<0xB1>(cs));
    cs = fmax(cs, dpp8_d<0x4E>(cs));
    cs = fmax(cs, dpp8_d<0x141>(cs));
    double mag = valid ? (fma(cs + 1.0, ww, px) + 2.0 * wva) * ipsj : 0.0;
    sabs = rowsum8(sabs);
    mag = rowsum8(mag);
    bool exact;
    {
        const double SS = yyj + contrib, rt = 1.01 * (yyj * __builtin_amdgcn_rsq(yyj) + sabs);
        const double num = fmax(rt * rt, 1.01 * (yyj + mag));
        exact = __any(valid && !(SS > 0.0 && num <= kappa_max * SS));
    }
    // ---- psi (dc:150, tau of the previous iteration, Q11) and the outputs
    if (valid) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int r = l + 8 * b;
            const double ps_b = rv[b] ? (1.0 / (d.df * 0.5 + 0.5 * (x[b] * x[b] * tv[b]))) * G[b] : 0.0;
            Lam[rowoff + r] = x[b];
            cpart[rowoff + r] = ps_b * (x[b] * x[b]);               // mat = psijh .* Lambda.^2 (dc:156)
            if (rv[b]) psi[rowoff + r] = ps_b;
        }
    }
    if (exact) {   // dc:169 as written for the wave's rows: Ytil = Yd - eta Lambda', sum(Ytil.^2)
        double(*Lm)[KP + 1] = reinterpret_cast<double(*)[KP + 1]>(SM);   // the image area, free now
#pragma unroll
        for (int b = 0; b < 4; ++b) Lm[grp][l + 8 * b] = x[b];
        __builtin_amdgcn_wave_barrier();
        const int cc = lane & 15;
        const double gps_c = ld.Gps[(uint32_t)(m * d.P) + (j0 + cc < d.P && cc < LAM_ROWS ? j0 + cc : 0)];
        resid_rows8(d, Y, X, Z, Lm, gps_c, m, j0, lane, ps, omega);
    } else if (valid && l == 0) {
        const double SS = yyj + contrib;
        const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps;     // dc:170
        ps[(uint32_t)(m * d.PP + j)] = psn;
        omega[(uint32_t)(m * d.PP + j)] = 1.0 / psn;            // dc:171 (Q1)
    }
}

}  // namespace dcfm
