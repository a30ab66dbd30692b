// Dev harness variants of the loading-row kernel (tools/lambench).  Not product code.
#pragma once
#include "linalg.h"
#include "lambda.h"

namespace dcfm {
namespace lv {

template <int CTRL>
__device__ __forceinline__ double dpp8(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsum8(double v) {
    v += dpp8<0xB1>(v);
    v += dpp8<0x4E>(v);
    v += dpp8<0x141>(v);
    return v;
}
template <int B> using IC = std::integral_constant<int, B>;
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
__device__ unsigned long long *g_stamps;

// N1: 8 loading rows per wave (8-lane group per row, lane l holds rows l + 8b, b = 0..3, the
// lower triangle pruned at compile time), variates read from draw buffers, lane-dependent
// selects only in the block holding the pivot pair, double-buffered image of the next pivot
// column pair written before the rest of the trailing update.
template <int LAM = 0>
__global__ __launch_bounds__(64) void k_lam_n1(Dims d, const double *__restrict__ C, const double *__restrict__ E,
                                               const double *__restrict__ yy, const double *__restrict__ tau_cur,
                                               double *__restrict__ Lam, double *__restrict__ psi,
                                               const double *__restrict__ plam_src, double *__restrict__ ps,
                                               double *__restrict__ omega, double *__restrict__ cpart, DrawsDev dr,
                                               int64_t iter) {
    unsigned long long T[6];
    if (LAM) T[0] = stamp();
    __shared__ __attribute__((aligned(16))) double LS[2][8][KP + 1][2];
    __shared__ __attribute__((aligned(16))) double BS[2][8][KP + 2];
    __shared__ __attribute__((aligned(16))) double VS[8][KP + 2];
    __shared__ __attribute__((aligned(16))) double IS[8][KP + 2];
    const int m = blockIdx.y, mg = d.shard0 + m;
    const int lane = threadIdx.x, grp = lane >> 3, l = lane & 7;
    const int j = blockIdx.x * 8 + grp;
    const bool valid = j < d.P;
    const int jj = valid ? j : 0;
    const uint32_t rowoff = (uint32_t)(m * d.PP + jj) * KP, toff = (uint32_t)mg * KP;
    bool rv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) rv[b] = valid && l + 8 * b < d.K;
    const double psj = valid ? ps[(uint32_t)(m * d.PP + jj)] : 1.0;
    const double yyj = (valid && l == 0) ? yy[(uint32_t)(m * d.PP + jj)] : 0.0;
    const double *pin = plam_src ? plam_src : psi;
    double pv[4], tv[4], cv[4], z[4], G[4];
    const uint32_t ti = (uint32_t)(iter - dr.first_iter);
    const uint32_t drow = (ti * (uint32_t)d.g + (uint32_t)mg) * (uint32_t)d.P + (uint32_t)jj;
    const uint32_t dk = drow * (uint32_t)d.K;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        pv[b] = pin[rowoff + l + 8 * b];
        tv[b] = tau_cur[toff + l + 8 * b];
        cv[b] = C[rowoff + l + 8 * b];
        const uint32_t di = rv[b] ? dk + l + 8 * b : dk;
        z[b] = dr.NL[di];
        G[b] = dr.Gpsi[di];
    }
    const double Gps = dr.Gps[drow];
    double q0[8], q1[16], q2[24], q3[32];
    auto load = [&](auto &q, auto NB) {
        constexpr int b = decltype(NB)::value, nc = 8 * b + 8;
        const double *Er = E + ((uint32_t)m * KP + l + 8 * b) * KP;
#pragma unroll
        for (int c = 0; c < nc; c += 2) {
            const d2 e = *reinterpret_cast<const d2 *>(Er + c);
            q[c] = e.x;
            q[c + 1] = e.y;
        }
    };
    load(q0, IC<0>{});
    load(q1, IC<1>{});
    load(q2, IC<2>{});
    load(q3, IC<3>{});
    double plam[4], bv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        plam[b] = rv[b] ? (plam_src ? pv[b] : pv[b] * tv[b]) : 0.0;
        bv[b] = valid ? psj * cv[b] : 0.0;
        z[b] = rv[b] ? z[b] : 0.0;
        G[b] = rv[b] ? G[b] : 0.0;
    }
    auto build = [&](auto &q, auto NB) {
        constexpr int b = decltype(NB)::value, nc = 8 * b + 8;
        const int r = l + 8 * b;
#pragma unroll
        for (int c = 0; c < nc; ++c) q[c] *= psj;
#pragma unroll
        for (int c = 8 * b; c < nc; ++c)
            if (c == r) q[c] = rv[b] ? plam[b] + q[c] : 1.0;
    };
    build(q0, IC<0>{});
    build(q1, IC<1>{});
    build(q2, IC<2>{});
    build(q3, IC<3>{});
    auto qref = [&](auto NB) -> auto & {
        constexpr int b = decltype(NB)::value;
        if constexpr (b == 0) return q0;
        else if constexpr (b == 1) return q1;
        else if constexpr (b == 2) return q2;
        else return q3;
    };
    double *Vs = VS[grp], *Is = IS[grp];
    if (LAM) T[1] = stamp();
    // image of column pair (0, 1)
    static_for<4>([&](auto NB) {
        constexpr int b = decltype(NB)::value;
        auto &q = qref(NB);
        d2 v;
        v.x = q[0];
        v.y = q[1];
        *reinterpret_cast<d2 *>(LS[0][grp][l + 8 * b]) = v;
        BS[0][grp][l + 8 * b] = bv[b];
    });
    __builtin_amdgcn_wave_barrier();
    static_for<KP / 2>([&](auto JC) {
        constexpr int k = 2 * decltype(JC)::value, cur = decltype(JC)::value & 1, nxt = cur ^ 1;
        constexpr int cb = k / 8, kk = k % 8;
        double(*Ls)[2] = LS[cur][grp];
        const d2 pk = *reinterpret_cast<const d2 *>(Ls[k]);
        const d2 pk1 = *reinterpret_cast<const d2 *>(Ls[k + 1]);
        const d2 bb = *reinterpret_cast<const d2 *>(&BS[cur][grp][k]);
        const double a = pk.x, bq = pk1.x, c2 = pk1.y;
        const double i00 = rsqrt_f64(a);
        const double l00 = a * i00, l10 = bq * i00;
        const double d11 = c2 - l10 * l10;
        const double i11 = rsqrt_f64(d11);
        const double l11 = d11 * i11;
        const double v0 = bb.x * i00, v1 = (bb.y - l10 * v0) * i11;
        const double t10 = l10 * i11;
        if (l == 0) {
            d2 v, iv;
            v.x = v0; v.y = v1; iv.x = i00; iv.y = i11;
            *reinterpret_cast<d2 *>(Vs + k) = v;
            *reinterpret_cast<d2 *>(Is + k) = iv;
        }
        double al[4] = {0.0, 0.0, 0.0, 0.0}, be[4] = {0.0, 0.0, 0.0, 0.0};
        static_for<4>([&](auto NB) {
            constexpr int b = decltype(NB)::value;
            if constexpr (b >= cb) {
                auto &q = qref(NB);
                const double lr0 = q[k] * i00;
                const double lr1 = (q[k + 1] - lr0 * l10) * i11;
                const double a_ = i00 * fma(-lr1, t10, lr0), b_ = lr1 * i11;
                const double nb = fma(-lr1, v1, fma(-lr0, v0, bv[b]));
                if constexpr (b > cb) {
                    q[k] = lr0;
                    q[k + 1] = lr1;
                    al[b] = a_;
                    be[b] = b_;
                    bv[b] = nb;
                } else {
                    const bool gt = l > kk + 1, e1 = l == kk + 1, e0 = l == kk;
                    q[k] = gt ? lr0 : (e1 ? l10 : (e0 ? l00 : q[k]));
                    q[k + 1] = gt ? lr1 : (e1 ? l11 : (e0 ? 0.0 : q[k + 1]));
                    al[b] = gt ? a_ : 0.0;
                    be[b] = gt ? b_ : 0.0;
                    bv[b] = gt ? nb : bv[b];
                }
            }
        });
        if constexpr (k + 2 < KP) {
            constexpr int c0 = k + 2, cb2 = c0 / 8;
            const d2 i2 = *reinterpret_cast<const d2 *>(Ls[c0]);
            const d2 i3 = *reinterpret_cast<const d2 *>(Ls[c0 + 1]);
            static_for<4>([&](auto NB) {
                constexpr int b = decltype(NB)::value;
                if constexpr (b >= cb2) {
                    auto &q = qref(NB);
                    q[c0] = fma(-be[b], i2.y, fma(-al[b], i2.x, q[c0]));
                    q[c0 + 1] = fma(-be[b], i3.y, fma(-al[b], i3.x, q[c0 + 1]));
                    d2 v;
                    v.x = q[c0];
                    v.y = q[c0 + 1];
                    *reinterpret_cast<d2 *>(LS[nxt][grp][l + 8 * b]) = v;
                    BS[nxt][grp][l + 8 * b] = bv[b];
                }
            });
#pragma unroll
            for (int c = c0 + 2; c < KP; ++c) {
                const d2 ic = *reinterpret_cast<const d2 *>(Ls[c]);
                static_for<4>([&](auto NB) {
                    constexpr int b = decltype(NB)::value;
                    if constexpr (b >= cb) {
                        auto &q = qref(NB);
                        if (c < 8 * b + 8) {
                            constexpr int nq = 8 * b + 8;
                            double &x = q[c < nq ? c : 0];
                            x = fma(-be[b], ic.y, fma(-al[b], ic.x, x));
                        }
                    }
                });
            }
            static_for<4>([&](auto NB) {
                constexpr int b = decltype(NB)::value;
                if constexpr (b >= cb) {
                    auto &q = qref(NB);
#pragma unroll
                    for (int c = c0; c < 8 * b + 8; ++c) asm volatile("" : "+v"(q[c]));
                }
            });
            __builtin_amdgcn_wave_barrier();
        }
    });
    if (LAM) T[2] = stamp();
    // back solve L' x = w, w = v + z, pivots (c, c-1) from the bottom (as k_lambda)
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    double ww = 0.0, wv = 0.0;
    static_for<KP / 2>([&](auto JC) {
        constexpr int c = KP - 1 - 2 * decltype(JC)::value;
        constexpr int cb = c / 8;
        double pa = 0.0, pb = 0.0;
        static_for<4>([&](auto NB) {
            constexpr int b = decltype(NB)::value;
            if constexpr (b >= cb) {
                auto &q = qref(NB);
                pa = fma(q[c], x[b], pa);
                pb = fma(q[c - 1], x[b], pb);
            }
        });
        pa = rsum8(pa);
        pb = rsum8(pb);
        auto &qc = qref(IC<cb>{});
        const d2 vv = *reinterpret_cast<const d2 *>(Vs + c - 1);
        const d2 iv = *reinterpret_cast<const d2 *>(Is + c - 1);
        double t = 0.0;
        if (l + 8 * cb == c) {
            const double wc = vv.y + z[cb];
            x[cb] = (wc - pa) * iv.y;
            t = qc[c - 1] * x[cb];
            ww = fma(wc, wc, ww);
            wv = fma(wc, vv.y, wv);
        }
        const double tb = dpp8<0x101>(t);
        if (l + 8 * cb == c - 1) {
            const double wc = vv.x + z[cb];
            x[cb] = (wc - pb - tb) * iv.x;
            ww = fma(wc, wc, ww);
            wv = fma(wc, vv.x, wv);
        }
    });
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (!rv[b]) x[b] = 0.0;
    if (LAM) T[3] = stamp();
    double px = 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int r = l + 8 * b;
        const double p = pin[rowoff + r], tr = tau_cur[toff + r];
        const double pl = rv[b] ? (plam_src ? p : p * tr) : 0.0;
        px = fma(pl * x[b], x[b], px);
    }
    double contrib = (ww - px - 2.0 * wv) / psj;
    contrib = valid ? contrib : 0.0;
    contrib = rsum8(contrib);
    if (valid) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int r = l + 8 * b;
            const double tr = rv[b] ? tau_cur[toff + r] : 0.0;
            const double ps_b = rv[b] ? (1.0 / (d.df * 0.5 + 0.5 * (x[b] * x[b] * tr))) * G[b] : 0.0;
            Lam[rowoff + r] = x[b];
            cpart[rowoff + r] = ps_b * (x[b] * x[b]);
            if (rv[b]) psi[rowoff + r] = ps_b;
        }
        if (l == 0) {
            const double SS = yyj + contrib;
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps;
            ps[(uint32_t)(m * d.PP + j)] = psn;
            omega[(uint32_t)(m * d.PP + j)] = 1.0 / psn;
        }
    }
    if (LAM) {
        T[4] = stamp();
        if (lane == 0) {
            unsigned long long *o = g_stamps + 8 * (blockIdx.y * gridDim.x + blockIdx.x);
            for (int i = 0; i < 5; ++i) o[i] = T[i];
        }
    }
}

// N2: as N1, plus: E_m staged once per wave in LDS (8 dwordx4 global loads per lane instead of
// 40, the 8 row groups then read it as LDS broadcasts); the next pivot pair's image read and
// factor issued right after the look-ahead put, so its latency chain overlaps the rest of the
// trailing update; branch-free selects (only the pivot block masks al / be); the variates and
// the Plam / tau reloads issued late (step 12).  OPT & 1: Plam-free pivot formula with the two
// rsqrt in parallel (i11 = l00 / sqrt(a c - b^2)).
struct Piv { double i00, i11, l00, l10, l11, v0, v1, t10; };
template <int OPT>
__device__ __forceinline__ Piv pivots(d2 pk, d2 pk1, d2 bb) {
    Piv p;
    const double a = pk.x, bq = pk1.x, c2 = pk1.y;
    if (OPT & 1) {
        const double D = fma(a, c2, -(bq * bq));
        p.i00 = rsqrt_f64(a);
        const double iD = rsqrt_f64(D);
        p.l00 = a * p.i00;
        p.l10 = bq * p.i00;
        p.i11 = p.l00 * iD;
        p.l11 = (D * iD) * p.i00;
    } else {
        p.i00 = rsqrt_f64(a);
        p.l00 = a * p.i00;
        p.l10 = bq * p.i00;
        const double d11 = c2 - p.l10 * p.l10;
        p.i11 = rsqrt_f64(d11);
        p.l11 = d11 * p.i11;
    }
    p.v0 = bb.x * p.i00;
    p.v1 = (bb.y - p.l10 * p.v0) * p.i11;
    p.t10 = p.l10 * p.i11;
    return p;
}

template <int LAM = 0, int OPT = 0>
__global__ __launch_bounds__(64) void k_lam_n2(Dims d, const double *__restrict__ C, const double *__restrict__ E,
                                               const double *__restrict__ yy, const double *__restrict__ tau_cur,
                                               double *__restrict__ Lam, double *__restrict__ psi,
                                               const double *__restrict__ plam_src, double *__restrict__ ps,
                                               double *__restrict__ omega, double *__restrict__ cpart, DrawsDev dr,
                                               int64_t iter) {
    unsigned long long T[6];
    if (LAM) T[0] = stamp();
    constexpr int LSN = 2 * 8 * (KP + 1) * 2, BSN = 2 * 8 * (KP + 2), VSN = 8 * (KP + 2);
    constexpr int EP = KP + 2;                       // E row pitch in LDS (conflict-free row reads)
    static_assert(KP * EP <= LSN + BSN, "E staging fits the image area");
    __shared__ __attribute__((aligned(16))) double SM[LSN + BSN + 2 * VSN];
    double(*LS)[8][KP + 1][2] = reinterpret_cast<double(*)[8][KP + 1][2]>(SM);
    double(*BS)[8][KP + 2] = reinterpret_cast<double(*)[8][KP + 2]>(SM + LSN);
    double(*VS)[KP + 2] = reinterpret_cast<double(*)[KP + 2]>(SM + LSN + BSN);
    double(*IS)[KP + 2] = reinterpret_cast<double(*)[KP + 2]>(SM + LSN + BSN + VSN);
    double *Es = SM;
    const int m = blockIdx.y, mg = d.shard0 + m;
    const int lane = threadIdx.x, grp = lane >> 3, l = lane & 7;
    const int j = blockIdx.x * 8 + grp;
    const bool valid = j < d.P;
    const int jj = valid ? j : 0;
    const uint32_t rowoff = (uint32_t)(m * d.PP + jj) * KP, toff = (uint32_t)mg * KP;
    bool rv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) rv[b] = valid && l + 8 * b < d.K;
    // E_m: 1024 doubles, lane t loads pairs 2t + 128 i
    {
        const double *Em = E + (uint32_t)m * KP * KP;
        d2 e[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = *reinterpret_cast<const d2 *>(Em + 2 * lane + 128 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = 2 * lane + 128 * i, r = f >> 5, c = f & 31;
            *reinterpret_cast<d2 *>(Es + r * EP + c) = e[i];
        }
    }
    const double psj = valid ? ps[(uint32_t)(m * d.PP + jj)] : 1.0;
    const double *pin = plam_src ? plam_src : psi;
    double plam[4], bv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const double pv = pin[rowoff + l + 8 * b], tv = tau_cur[toff + l + 8 * b], cv = C[rowoff + l + 8 * b];
        plam[b] = rv[b] ? (plam_src ? pv : pv * tv) : 0.0;
        bv[b] = valid ? psj * cv : 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    double q0[8], q1[16], q2[24], q3[32];
    auto qref = [&](auto NB) -> auto & {
        constexpr int b = decltype(NB)::value;
        if constexpr (b == 0) return q0;
        else if constexpr (b == 1) return q1;
        else if constexpr (b == 2) return q2;
        else return q3;
    };
    static_for<4>([&](auto NB) {
        constexpr int b = decltype(NB)::value, nc = 8 * b + 8;
        auto &q = qref(NB);
        const double *Er = Es + (l + 8 * b) * EP;
#pragma unroll
        for (int c = 0; c < nc; c += 2) {
            const d2 e = *reinterpret_cast<const d2 *>(Er + c);
            q[c] = e.x;
            q[c + 1] = e.y;
        }
    });
    static_for<4>([&](auto NB) {
        constexpr int b = decltype(NB)::value, nc = 8 * b + 8;
        auto &q = qref(NB);
        const int r = l + 8 * b;
#pragma unroll
        for (int c = 0; c < nc; ++c) q[c] *= psj;
#pragma unroll
        for (int c = 8 * b; c < nc; ++c)
            if (c == r) q[c] = rv[b] ? plam[b] + q[c] : 1.0;
    });
    double *Vs = VS[grp], *Is = IS[grp];
    if (LAM) T[1] = stamp();
    __builtin_amdgcn_wave_barrier();
    // image of column pair (0, 1) (overwrites E's staging: every read of it is above)
    static_for<4>([&](auto NB) {
        constexpr int b = decltype(NB)::value;
        auto &q = qref(NB);
        d2 v;
        v.x = q[0];
        v.y = q[1];
        *reinterpret_cast<d2 *>(LS[0][grp][l + 8 * b]) = v;
        BS[0][grp][l + 8 * b] = bv[b];
    });
    __builtin_amdgcn_wave_barrier();
    Piv pv = pivots<OPT>(*reinterpret_cast<const d2 *>(LS[0][grp][0]), *reinterpret_cast<const d2 *>(LS[0][grp][1]),
                         *reinterpret_cast<const d2 *>(&BS[0][grp][0]));
    double z[4], G[4], tv[4], pl2[4], Gps = 0.0, yyj = 0.0;
    static_for<KP / 2>([&](auto JC) {
        constexpr int k = 2 * decltype(JC)::value, cur = decltype(JC)::value & 1, nxt = cur ^ 1;
        constexpr int cb = k / 8, kk = k % 8;
        double(*Ls)[2] = LS[cur][grp];
        const Piv p = pv;
        {   // every lane of the group stores the same values: no exec-mask branch
            d2 v, iv;
            v.x = p.v0; v.y = p.v1; iv.x = p.i00; iv.y = p.i11;
            *reinterpret_cast<d2 *>(Vs + k) = v;
            *reinterpret_cast<d2 *>(Is + k) = iv;
        }
        double al[4] = {0.0, 0.0, 0.0, 0.0}, be[4] = {0.0, 0.0, 0.0, 0.0};
        static_for<4>([&](auto NB) {
            constexpr int b = decltype(NB)::value;
            if constexpr (b >= cb) {
                auto &q = qref(NB);
                const double lr0 = q[k] * p.i00;
                const double lr1 = (q[k + 1] - lr0 * p.l10) * p.i11;
                const double a_ = p.i00 * fma(-lr1, p.t10, lr0), b_ = lr1 * p.i11;
                bv[b] = fma(-lr1, p.v1, fma(-lr0, p.v0, bv[b]));
                if constexpr (b > cb) {
                    q[k] = lr0;
                    q[k + 1] = lr1;
                    al[b] = a_;
                    be[b] = b_;
                } else {
                    const bool gt = l > kk + 1;
                    q[k] = lr0;
                    q[k + 1] = (l == kk) ? 0.0 : lr1;
                    al[b] = gt ? a_ : 0.0;
                    be[b] = gt ? b_ : 0.0;
                }
            }
        });
        if constexpr (k + 2 < KP) {
            constexpr int c0 = k + 2, cb2 = c0 / 8;
            const d2 i2 = *reinterpret_cast<const d2 *>(Ls[c0]);
            const d2 i3 = *reinterpret_cast<const d2 *>(Ls[c0 + 1]);
            static_for<4>([&](auto NB) {
                constexpr int b = decltype(NB)::value;
                if constexpr (b >= cb2) {
                    auto &q = qref(NB);
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
            // next pivot pair: its LDS round trip and rsqrt chain overlap the update below
            pv = pivots<OPT>(*reinterpret_cast<const d2 *>(LS[nxt][grp][c0]),
                             *reinterpret_cast<const d2 *>(LS[nxt][grp][c0 + 1]),
                             *reinterpret_cast<const d2 *>(&BS[nxt][grp][c0]));
#pragma unroll
            for (int c = c0 + 2; c < KP; ++c) {
                const d2 ic = *reinterpret_cast<const d2 *>(Ls[c]);
                static_for<4>([&](auto NB) {
                    constexpr int b = decltype(NB)::value;
                    if constexpr (b >= cb) {
                        auto &q = qref(NB);
                        if (c < 8 * b + 8) {
                            constexpr int nq = 8 * b + 8;
                            double &x = q[c < nq ? c : 0];
                            x = fma(-be[b], ic.y, fma(-al[b], ic.x, x));
                        }
                    }
                });
            }
            static_for<4>([&](auto NB) {
                constexpr int b = decltype(NB)::value;
                if constexpr (b >= cb) {
                    auto &q = qref(NB);
#pragma unroll
                    for (int c = c0; c < 8 * b + 8; ++c) asm volatile("" : "+v"(q[c]));
                }
            });
        }
        if constexpr (k == 24) {   // the back solve's and epilogue's inputs, in flight for 2 steps
            asm volatile("" ::: "memory");
            const uint32_t ti = (uint32_t)(iter - dr.first_iter);
            const uint32_t drow = (ti * (uint32_t)d.g + (uint32_t)mg) * (uint32_t)d.P + (uint32_t)jj;
            const uint32_t dk = drow * (uint32_t)d.K;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t di = rv[b] ? dk + l + 8 * b : dk;
                z[b] = dr.NL[di];
                G[b] = dr.Gpsi[di];
                const double p2 = pin[rowoff + l + 8 * b];
                tv[b] = tau_cur[toff + l + 8 * b];
                pl2[b] = plam_src ? p2 : p2 * tv[b];
            }
            Gps = dr.Gps[drow];
            yyj = yy[(uint32_t)(m * d.PP + jj)];
        }
    });
    if (LAM) T[2] = stamp();
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        z[b] = rv[b] ? z[b] : 0.0;
        G[b] = rv[b] ? G[b] : 0.0;
        pl2[b] = rv[b] ? pl2[b] : 0.0;
        tv[b] = rv[b] ? tv[b] : 0.0;
    }
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    double ww = 0.0, wv = 0.0;
    static_for<KP / 2>([&](auto JC) {
        constexpr int c = KP - 1 - 2 * decltype(JC)::value;
        constexpr int cb = c / 8;
        double pa = 0.0, pb = 0.0;
        static_for<4>([&](auto NB) {
            constexpr int b = decltype(NB)::value;
            if constexpr (b >= cb) {
                auto &q = qref(NB);
                pa = fma(q[c], x[b], pa);
                pb = fma(q[c - 1], x[b], pb);
            }
        });
        pa = rsum8(pa);
        pb = rsum8(pb);
        auto &qc = qref(IC<cb>{});
        const d2 vv = *reinterpret_cast<const d2 *>(Vs + c - 1);
        const d2 iv = *reinterpret_cast<const d2 *>(Is + c - 1);
        const bool isc = l + 8 * cb == c, isc1 = l + 8 * cb == c - 1;
        const double wa = vv.y + z[cb];
        const double xa = (wa - pa) * iv.y;
        x[cb] = isc ? xa : x[cb];
        const double t = isc ? qc[c - 1] * xa : 0.0;
        ww = isc ? fma(wa, wa, ww) : ww;
        wv = isc ? fma(wa, vv.y, wv) : wv;
        const double tb = dpp8<0x101>(t);
        const double wb = vv.x + z[cb];
        const double xb = (wb - pb - tb) * iv.x;
        x[cb] = isc1 ? xb : x[cb];
        ww = isc1 ? fma(wb, wb, ww) : ww;
        wv = isc1 ? fma(wb, vv.x, wv) : wv;
    });
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (!rv[b]) x[b] = 0.0;
    if (LAM) T[3] = stamp();
    double px = 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) px = fma(pl2[b] * x[b], x[b], px);
    double contrib = (ww - px - 2.0 * wv) / psj;
    contrib = valid ? contrib : 0.0;
    contrib = rsum8(contrib);
    if (valid) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int r = l + 8 * b;
            const double ps_b = rv[b] ? (1.0 / (d.df * 0.5 + 0.5 * (x[b] * x[b] * tv[b]))) * G[b] : 0.0;
            Lam[rowoff + r] = x[b];
            cpart[rowoff + r] = ps_b * (x[b] * x[b]);
            if (rv[b]) psi[rowoff + r] = ps_b;
        }
        if (l == 0) {
            const double SS = yyj + contrib;
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps;
            ps[(uint32_t)(m * d.PP + j)] = psn;
            omega[(uint32_t)(m * d.PP + j)] = 1.0 / psn;
        }
    }
    if (LAM) {
        T[4] = stamp();
        if (lane == 0) {
            unsigned long long *o = g_stamps + 8 * (blockIdx.y * gridDim.x + blockIdx.x);
            for (int i = 0; i < 5; ++i) o[i] = T[i];
        }
    }
}

// DPP move without an "old" operand (every source lane of these patterns is valid)
template <int CTRL>
__device__ __forceinline__ double dppx(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsum8x(double v) {
    v += dppx<0xB1>(v);
    v += dppx<0x4E>(v);
    v += dppx<0x141>(v);
    return v;
}
__host__ __device__ constexpr int ncol_of(int KE, int b) { return 8 * b + 8 < KE ? 8 * b + 8 : KE; }

// N3: N2 + the factor width KE (even, <= 32) a compile-time parameter (rows >= KE and their
// columns vanish; KE / 2 pivot steps), Q_j factored unscaled as E_m + diag(Plam_j / ps_j)
// (L_Q = sqrt(ps_j) L, so no per-element scaling; the rhs enters as sqrt(ps_j) C_j and x leaves
// divided by sqrt(ps_j)), |w|^2 and w.v formed after the back solve, DPP without old operands.
template <int KE, int LAM = 0, int LATE = 0, int PIPE = 0>
__global__ __launch_bounds__(64) void k_lam_n3(Dims d, const double *__restrict__ C, const double *__restrict__ E,
                                               const double *__restrict__ yy, const double *__restrict__ tau_cur,
                                               double *__restrict__ Lam, double *__restrict__ psi,
                                               const double *__restrict__ plam_src, double *__restrict__ ps,
                                               double *__restrict__ omega, double *__restrict__ cpart, DrawsDev dr,
                                               int64_t iter) {
    static_assert(KE % 2 == 0 && KE >= 2 && KE <= KP, "even factor width");
    constexpr int NB = (KE + 7) / 8;
    unsigned long long T[6];
    if (LAM) T[0] = stamp();
    constexpr int LSN = 2 * 8 * (KP + 1) * 2, BSN = 2 * 8 * (KP + 2), VSN = 8 * (KP + 2);
    constexpr int EP = KP + 2;
    __shared__ __attribute__((aligned(16))) double SM[LSN + BSN + 2 * VSN];
    double(*LS)[8][KP + 1][2] = reinterpret_cast<double(*)[8][KP + 1][2]>(SM);
    double(*BS)[8][KP + 2] = reinterpret_cast<double(*)[8][KP + 2]>(SM + LSN);
    double(*VS)[KP + 2] = reinterpret_cast<double(*)[KP + 2]>(SM + LSN + BSN);
    double(*IS)[KP + 2] = reinterpret_cast<double(*)[KP + 2]>(SM + LSN + BSN + VSN);
    double *Es = SM;
    const int m = blockIdx.y, mg = d.shard0 + m;
    const int lane = threadIdx.x, grp = lane >> 3, l = lane & 7;
    const int j = blockIdx.x * 8 + grp;
    const bool valid = j < d.P;
    const int jj = valid ? j : 0;
    const uint32_t rowoff = (uint32_t)(m * d.PP + jj) * KP, toff = (uint32_t)mg * KP;
    bool rv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) rv[b] = valid && l + 8 * b < d.K;
    {
        const double *Em = E + (uint32_t)m * KP * KP;
        constexpr int NI = (KE * KP + 127) / 128;    // rows < KE only
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
    const double isj = rsqrt_f64(psj), sj = psj * isj;      // 1 / sqrt(ps_j), sqrt(ps_j)
    const double ipsj = isj * isj;
    const double *pin = plam_src ? plam_src : psi;
    double dg[4], bv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const double pv = pin[rowoff + l + 8 * b], tv = tau_cur[toff + l + 8 * b], cv = C[rowoff + l + 8 * b];
        const double pl = plam_src ? pv : pv * tv;
        dg[b] = rv[b] ? pl * ipsj : 1.0;                   // diag(Plam_j / ps_j); identity padding
        bv[b] = valid ? sj * cv : 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    double q0[ncol_of(KE, 0)], q1[NB > 1 ? ncol_of(KE, 1) : 1], q2[NB > 2 ? ncol_of(KE, 2) : 1],
        q3[NB > 3 ? ncol_of(KE, 3) : 1];
    auto qref = [&](auto NBc) -> auto & {
        constexpr int b = decltype(NBc)::value;
        if constexpr (b == 0) return q0;
        else if constexpr (b == 1) return q1;
        else if constexpr (b == 2) return q2;
        else return q3;
    };
    static_for<NB>([&](auto NBc) {
        constexpr int b = decltype(NBc)::value, nc = ncol_of(KE, b);
        auto &q = qref(NBc);
        const double *Er = Es + (l + 8 * b) * EP;
#pragma unroll
        for (int c = 0; c < nc; c += 2) {
            const d2 e = *reinterpret_cast<const d2 *>(Er + c);
            q[c] = e.x;
            q[c + 1] = e.y;
        }
#pragma unroll
        for (int c = 8 * b; c < nc; ++c)
            if (c == l + 8 * b) q[c] += dg[b];
    });
    double *Vs = VS[grp], *Is = IS[grp];
    if (LAM) T[1] = stamp();
    __builtin_amdgcn_wave_barrier();
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
    Piv pv = pivots<0>(*reinterpret_cast<const d2 *>(LS[0][grp][0]), *reinterpret_cast<const d2 *>(LS[0][grp][1]),
                       *reinterpret_cast<const d2 *>(&BS[0][grp][0]));
    double z[4], G[4], tv[4], pl2[4], Gps = 0.0, yyj = 0.0;
    static_for<KE / 2>([&](auto JC) {
        constexpr int k = 2 * decltype(JC)::value, cur = decltype(JC)::value & 1, nxt = cur ^ 1;
        constexpr int cb = k / 8, kk = k % 8;
        double(*Ls)[2] = LS[cur][grp];
        const Piv p = pv;
        {
            d2 v, iv;
            v.x = p.v0; v.y = p.v1; iv.x = p.i00; iv.y = p.i11;
            *reinterpret_cast<d2 *>(Vs + k) = v;
            *reinterpret_cast<d2 *>(Is + k) = iv;
        }
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
                    const bool gt = l > kk + 1;
                    q[k + 1] = (l == kk) ? 0.0 : lr1;
                    al[b] = gt ? a_ : 0.0;
                    be[b] = gt ? b_ : 0.0;
                }
            }
        });
        if constexpr (k + 2 < KE) {
            constexpr int c0 = k + 2, cb2 = c0 / 8;
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
            pv = pivots<0>(*reinterpret_cast<const d2 *>(LS[nxt][grp][c0]),
                           *reinterpret_cast<const d2 *>(LS[nxt][grp][c0 + 1]),
                           *reinterpret_cast<const d2 *>(&BS[nxt][grp][c0]));
            auto upd = [&](int c, d2 ic) {
                static_for<NB>([&](auto NBc) {
                    constexpr int b = decltype(NBc)::value;
                    if constexpr (b >= cb) {
                        auto &q = qref(NBc);
                        constexpr int nq = ncol_of(KE, b);
                        if (c < nq) {
                            double &x = q[c < nq ? c : 0];
                            x = fma(-be[b], ic.y, fma(-al[b], ic.x, x));
                        }
                    }
                });
            };
            if constexpr (PIPE == 0) {
#pragma unroll
                for (int c = c0 + 2; c < KE; ++c) upd(c, *reinterpret_cast<const d2 *>(Ls[c]));
            } else {
                // batches of PIPE columns, the next batch's reads issued before this batch's FMAs
                constexpr int cs = c0 + 2, nbt = (KE - cs + PIPE - 1) / PIPE;
                d2 buf[2][PIPE];
                static_for<PIPE>([&](auto T) {
                    constexpr int c = cs + decltype(T)::value;
                    if constexpr (c < KE) buf[0][decltype(T)::value] = *reinterpret_cast<const d2 *>(Ls[c]);
                });
                static_for<nbt>([&](auto Bt) {
                    constexpr int bt = decltype(Bt)::value, cur_b = bt & 1;
                    if constexpr (bt + 1 < nbt) {
                        static_for<PIPE>([&](auto T) {
                            constexpr int c = cs + (bt + 1) * PIPE + decltype(T)::value;
                            if constexpr (c < KE)
                                buf[cur_b ^ 1][decltype(T)::value] = *reinterpret_cast<const d2 *>(Ls[c]);
                        });
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<PIPE>([&](auto T) {
                        constexpr int c = cs + bt * PIPE + decltype(T)::value;
                        if constexpr (c < KE) upd(c, buf[cur_b][decltype(T)::value]);
                    });
                    __builtin_amdgcn_sched_barrier(0);
                });
            }
            static_for<NB>([&](auto NBc) {
                constexpr int b = decltype(NBc)::value;
                if constexpr (b >= cb) {
                    auto &q = qref(NBc);
#pragma unroll
                    for (int c = c0; c < ncol_of(KE, b); ++c) asm volatile("" : "+v"(q[c]));
                }
            });
        }
        if constexpr (!LATE && k == (KE >= 8 ? KE - 8 : 0)) {   // the back solve's and epilogue's inputs
            asm volatile("" ::: "memory");
            const uint32_t ti = (uint32_t)(iter - dr.first_iter);
            const uint32_t drow = (ti * (uint32_t)d.g + (uint32_t)mg) * (uint32_t)d.P + (uint32_t)jj;
            const uint32_t dk = drow * (uint32_t)d.K;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t di = rv[b] ? dk + l + 8 * b : dk;
                z[b] = dr.NL[di];
                G[b] = dr.Gpsi[di];
                const double p2 = pin[rowoff + l + 8 * b];
                tv[b] = tau_cur[toff + l + 8 * b];
                pl2[b] = plam_src ? p2 : p2 * tv[b];
            }
            Gps = dr.Gps[drow];
            yyj = yy[(uint32_t)(m * d.PP + jj)];
        }
    });
    if constexpr (LATE) {
        const uint32_t ti = (uint32_t)(iter - dr.first_iter);
        const uint32_t drow = (ti * (uint32_t)d.g + (uint32_t)mg) * (uint32_t)d.P + (uint32_t)jj;
        const uint32_t dk = drow * (uint32_t)d.K;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t di = rv[b] ? dk + l + 8 * b : dk;
            z[b] = dr.NL[di];
            G[b] = dr.Gpsi[di];
            const double p2 = pin[rowoff + l + 8 * b];
            tv[b] = tau_cur[toff + l + 8 * b];
            pl2[b] = plam_src ? p2 : p2 * tv[b];
        }
        Gps = dr.Gps[drow];
        yyj = yy[(uint32_t)(m * d.PP + jj)];
    }
    if (LAM) T[2] = stamp();
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        z[b] = rv[b] ? z[b] : 0.0;
        G[b] = rv[b] ? G[b] : 0.0;
        pl2[b] = rv[b] ? pl2[b] : 0.0;
        tv[b] = rv[b] ? tv[b] : 0.0;
    }
    // back solve L' x = w (w = v + z), pivots (c, c-1) from the bottom
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    static_for<KE / 2>([&](auto JC) {
        constexpr int c = KE - 1 - 2 * decltype(JC)::value;
        constexpr int cb = c / 8;
        double pa = 0.0, pb = 0.0;
        static_for<NB>([&](auto NBc) {
            constexpr int b = decltype(NBc)::value;
            if constexpr (b >= cb) {
                auto &q = qref(NBc);
                pa = fma(q[c], x[b], pa);
                pb = fma(q[c - 1], x[b], pb);
            }
        });
        pa = rsum8x(pa);
        pb = rsum8x(pb);
        auto &qc = qref(IC<cb>{});
        const d2 vv = *reinterpret_cast<const d2 *>(Vs + c - 1);
        const d2 iv = *reinterpret_cast<const d2 *>(Is + c - 1);
        const bool isc = l + 8 * cb == c, isc1 = l + 8 * cb == c - 1;
        const double xa = (vv.y + z[cb] - pa) * iv.y;
        x[cb] = isc ? xa : x[cb];
        const double t = isc ? qc[c - 1] * xa : 0.0;
        const double tb = dppx<0x101>(t);
        const double xb = (vv.x + z[cb] - pb - tb) * iv.x;
        x[cb] = isc1 ? xb : x[cb];
    });
    if (LAM) T[3] = stamp();
    // |w|^2, w.v over the lane's rows (w = v + z), x = x_E / sqrt(ps_j)
    double ww = 0.0, wv = 0.0, px = 0.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const double vr = Vs[l + 8 * b < KE ? l + 8 * b : 0];
        const double w = vr + z[b];
        ww = rv[b] ? fma(w, w, ww) : ww;
        wv = rv[b] ? fma(w, vr, wv) : wv;
        x[b] = rv[b] ? x[b] * isj : 0.0;
        px = fma(pl2[b] * x[b], x[b], px);
    }
    double contrib = (ww - px - 2.0 * wv) * ipsj;
    contrib = valid ? contrib : 0.0;
    contrib = rsum8x(contrib);
    if (valid) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int r = l + 8 * b;
            const double ps_b = rv[b] ? (1.0 / (d.df * 0.5 + 0.5 * (x[b] * x[b] * tv[b]))) * G[b] : 0.0;
            Lam[rowoff + r] = x[b];
            cpart[rowoff + r] = ps_b * (x[b] * x[b]);
            if (rv[b]) psi[rowoff + r] = ps_b;
        }
        if (l == 0) {
            const double SS = yyj + contrib;
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps;
            ps[(uint32_t)(m * d.PP + j)] = psn;
            omega[(uint32_t)(m * d.PP + j)] = 1.0 / psn;
        }
    }
    if (LAM) {
        T[4] = stamp();
        if (lane == 0) {
            unsigned long long *o = g_stamps + 8 * (blockIdx.y * gridDim.x + blockIdx.x);
            for (int i = 0; i < 5; ++i) o[i] = T[i];
        }
    }
}

template <int KE>
__global__ __launch_bounds__(64) void k_lam_n5(Dims d, const double *__restrict__ C, const double *__restrict__ E,
                                               const double *__restrict__ yy, const double *__restrict__ tau_cur,
                                               double *__restrict__ Lam, double *__restrict__ psi,
                                               const double *__restrict__ plam_src, double *__restrict__ ps,
                                               double *__restrict__ omega, double *__restrict__ cpart,
                                               LamDraws ld) {
    static_assert(KE % 2 == 0 && KE >= 2 && KE <= KP, "even factor width");
    constexpr int NB = (KE + 7) / 8;
    // LDS: double-buffered image [2][8 systems][KP + 1 (bank spread)][2] | rhs image [2][8][KP+2] |
    // per system v and 1 / L_kk [8][KP+2] each; E_m is staged (row pitch EP) in the image area first
    constexpr int LSN = 2 * LAM_ROWS * (KP + 1) * 2, BSN = 2 * LAM_ROWS * (KP + 2), VSN = LAM_ROWS * (KP + 2);
    constexpr int EP = KP + 2;
    static_assert(KP * EP <= LSN + BSN, "E staging fits the image area");
    __shared__ __attribute__((aligned(16))) double SM[LSN + BSN + 2 * VSN];
    double(*LS)[LAM_ROWS][KP + 1][2] = reinterpret_cast<double(*)[LAM_ROWS][KP + 1][2]>(SM);
    double(*BS)[LAM_ROWS][KP + 2] = reinterpret_cast<double(*)[LAM_ROWS][KP + 2]>(SM + LSN);
    double *Vs = SM + LSN + BSN, *Is = Vs + VSN;
    double *Es = SM;
    const int m = blockIdx.y, mg = d.shard0 + m;
    const int lane = threadIdx.x, grp = lane >> 3, l = lane & 7;
    Vs += grp * (KP + 2);
    Is += grp * (KP + 2);
    const int j = blockIdx.x * LAM_ROWS + grp;
    const bool valid = j < d.P;
    const int jj = valid ? j : 0;
    const uint32_t rowoff = (uint32_t)(m * d.PP + jj) * KP, toff = (uint32_t)mg * KP;
    bool rv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) rv[b] = valid && l + 8 * b < d.K;
    {   // E_m rows < KE: lane t moves pairs 2t + 128 i
        const double *Em = E + (uint32_t)m * KP * KP;
        constexpr int NI = (KE * KP + 127) / 128;
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
#pragma unroll
        for (int c = 8 * b; c < nc; ++c)
            if (c == l + 8 * b) q[c] += dg[b];
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
            // next pivot pair: reads issued now, its chain computed in stages inside the batches below
            const d2 npk = *reinterpret_cast<const d2 *>(LS[nxt][grp][c0]);
            const d2 npk1 = *reinterpret_cast<const d2 *>(LS[nxt][grp][c0 + 1]);
            const d2 nbb = *reinterpret_cast<const d2 *>(&BS[nxt][grp][c0]);
            LamPiv np;
            auto stage = [&](int st) {
                if (st == 0) np.i00 = rsqrt_f64(npk.x);
                if (st == 1) {
                    np.l10 = npk1.x * np.i00;
                    np.i11 = rsqrt_f64(npk1.y - np.l10 * np.l10);
                }
                if (st == 2) {
                    np.v0 = nbb.x * np.i00;
                    np.v1 = (nbb.y - np.l10 * np.v0) * np.i11;
                    np.t10 = np.l10 * np.i11;
                }
            };
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
                if constexpr (bt < 3) stage(bt);
                static_for<LAM_PIPE>([&](auto T) {
                    constexpr int c = cs + bt * LAM_PIPE + decltype(T)::value;
                    if constexpr (c < KE) upd(c, buf[cur_b][decltype(T)::value]);
                });
                __builtin_amdgcn_sched_barrier(0);
            });
            static_for<3>([&](auto St) {
                if constexpr (decltype(St)::value >= nbt) stage(decltype(St)::value);
            });
            pv = np;
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
        const double xa = (vv.y + z[cb] - pa) * iv.y;
        x[cb] = isc ? xa : x[cb];
        const double t = isc ? qc[c - 1] * xa : 0.0;               // L[c][c-1] x_c
        const double tb = dpp8_d<0x101>(t);                        // row_shl:1: lane c%8 -> c%8 - 1
        const double xb = (vv.x + z[cb] - pb - tb) * iv.x;
        x[cb] = isc1 ? xb : x[cb];
    });
    // ---- SS_j = yy_j - 2 x.C_j + x'E x (dc:169 by identity, no Y pass).  x = L_Q'^{-1} w, so
    //      x'Q_j x = |w|^2 and x'E x = (|w|^2 - sum_r Plam_jr x_r^2) / ps_j: no E re-read;
    //      ps_j x.C_j = x.blam = x.(L_Q v) = (L_Q'x).v = w.v: no C re-read.
    double ww = 0.0, wv = 0.0, px = 0.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const double vr = Vs[l + 8 * b < KE ? l + 8 * b : 0];
        const double w = vr + z[b];
        ww = rv[b] ? fma(w, w, ww) : ww;
        wv = rv[b] ? fma(w, vr, wv) : wv;
        x[b] = rv[b] ? x[b] * isj : 0.0;                           // Lambda_j = L^{-T} w / sqrt(ps_j)
        px = fma(pl2[b] * x[b], x[b], px);
    }
    double contrib = (ww - px - 2.0 * wv) * ipsj;
    contrib = valid ? contrib : 0.0;
    contrib = rowsum8(contrib);
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
        if (l == 0) {
            const double SS = yyj + contrib;
            const double psn = (1.0 / (d.bs + 0.5 * SS)) * Gps;     // dc:170
            ps[(uint32_t)(m * d.PP + j)] = psn;
            omega[(uint32_t)(m * d.PP + j)] = 1.0 / psn;            // dc:171 (Q1)
        }
    }
}

}  // namespace lv

template <class Run>
void run_variants(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, const double *tau, Run &&run) {
    const dim3 grid((d.P + 7) / 8, d.G);
    {
        const size_t row0 = ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
        LamDraws ld{dr.NL + row0 * d.K, dr.Gpsi + row0 * d.K, dr.Gps + row0};
        if (d.K <= 30)
            run("n5 staged pivots KE=30", [&] {
                hipLaunchKernelGGL((lv::k_lam_n5<30>), grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam,
                                   b.psi, nullptr, b.ps, b.omega, b.cpart, ld);
            });
    }
    if (getenv("LAM_ONLY_NEW")) return;
    run("n1 (draws from buffers)", [&] {
        hipLaunchKernelGGL(lv::k_lam_n1<0>, grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam, b.psi,
                           nullptr, b.ps, b.omega, b.cpart, dr, iter);
    });
    // phase stamps (s_memtime at waitcnt-drained points): per-wave cycles of each phase
    const size_t nw = (size_t)grid.x * grid.y;
    unsigned long long *st = nullptr;
    (void)hipMalloc(&st, nw * 8 * 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(lv::g_stamps), &st, sizeof(st));
    run("n2", [&] {
        hipLaunchKernelGGL((lv::k_lam_n2<0, 0>), grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam, b.psi,
                           nullptr, b.ps, b.omega, b.cpart, dr, iter);
    });
    run("n2 parallel rsqrt pivots", [&] {
        hipLaunchKernelGGL((lv::k_lam_n2<0, 1>), grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam, b.psi,
                           nullptr, b.ps, b.omega, b.cpart, dr, iter);
    });
    run("n2 + phase stamps", [&] {
        hipLaunchKernelGGL((lv::k_lam_n2<1, 0>), grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam, b.psi,
                           nullptr, b.ps, b.omega, b.cpart, dr, iter);
    });
    {
        std::vector<unsigned long long> h2(nw * 8);
        (void)hipMemcpy(h2.data(), st, nw * 64, hipMemcpyDeviceToHost);
        double q[4] = {0, 0, 0, 0};
        for (size_t w = 0; w < nw; ++w)
            for (int i = 0; i < 4; ++i) q[i] += (double)(h2[8 * w + i + 1] - h2[8 * w + i]);
        printf("   n2 phases (mean cycles per wave): loads+build %.0f  factor %.0f  back %.0f  epilogue %.0f\n",
               q[0] / nw, q[1] / nw, q[2] / nw, q[3] / nw);
    }
    auto n3 = [&](auto KEc, auto LAMc, auto LATEc, auto PIPEc) {
        constexpr int KE = decltype(KEc)::value, LAM = decltype(LAMc)::value, LATE = decltype(LATEc)::value;
        constexpr int PIPE = decltype(PIPEc)::value;
        hipLaunchKernelGGL((lv::k_lam_n3<KE, LAM, LATE, PIPE>), grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam, b.psi,
                           nullptr, b.ps, b.omega, b.cpart, dr, iter);
    };
    if (d.K <= 30) {
        run("n3 KE=30", [&] { n3(lv::IC<30>{}, lv::IC<0>{}, lv::IC<0>{}, lv::IC<0>{}); });
        run("n3 KE=30 late loads", [&] { n3(lv::IC<30>{}, lv::IC<0>{}, lv::IC<1>{}, lv::IC<0>{}); });
        run("n3 KE=30 late pipe2", [&] { n3(lv::IC<30>{}, lv::IC<0>{}, lv::IC<1>{}, lv::IC<2>{}); });
        run("n3 KE=30 late pipe3", [&] { n3(lv::IC<30>{}, lv::IC<0>{}, lv::IC<1>{}, lv::IC<3>{}); });
        run("n3 KE=30 late pipe4", [&] { n3(lv::IC<30>{}, lv::IC<0>{}, lv::IC<1>{}, lv::IC<4>{}); });
        run("n3 KE=30 late pipe4 + stamps", [&] { n3(lv::IC<30>{}, lv::IC<1>{}, lv::IC<1>{}, lv::IC<4>{}); });
        std::vector<unsigned long long> h3(nw * 8);
        (void)hipMemcpy(h3.data(), st, nw * 64, hipMemcpyDeviceToHost);
        double q[4] = {0, 0, 0, 0};
        for (size_t w = 0; w < nw; ++w)
            for (int i = 0; i < 4; ++i) q[i] += (double)(h3[8 * w + i + 1] - h3[8 * w + i]);
        printf("   n3 phases (mean cycles per wave): loads+build %.0f  factor %.0f  back %.0f  epilogue %.0f\n",
               q[0] / nw, q[1] / nw, q[2] / nw, q[3] / nw);
    }
    run("n3 KE=32", [&] { n3(lv::IC<32>{}, lv::IC<0>{}, lv::IC<0>{}, lv::IC<0>{}); });
    run("n1 + phase stamps", [&] {
        hipLaunchKernelGGL(lv::k_lam_n1<1>, grid, dim3(64), 0, nullptr, d, b.C, b.E, b.yy, tau, b.Lam, b.psi,
                           nullptr, b.ps, b.omega, b.cpart, dr, iter);
    });
    std::vector<unsigned long long> h(nw * 8);
    (void)hipMemcpy(h.data(), st, nw * 64, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, t1 = 0;
    double ph[4] = {0, 0, 0, 0};
    for (size_t w = 0; w < nw; ++w) {
        t0 = std::min(t0, h[8 * w]);
        t1 = std::max(t1, h[8 * w + 4]);
        for (int i = 0; i < 4; ++i) ph[i] += (double)(h[8 * w + i + 1] - h[8 * w + i]);
    }
    printf("   phases (mean cycles per wave): loads+build %.0f  factor %.0f  back %.0f  epilogue %.0f ; "
           "kernel span %llu cycles\n", ph[0] / nw, ph[1] / nw, ph[2] / nw, ph[3] / nw, t1 - t0);
    (void)hipFree(st);
}

}  // namespace dcfm
