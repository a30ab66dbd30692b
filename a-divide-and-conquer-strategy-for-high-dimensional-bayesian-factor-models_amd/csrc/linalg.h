// Device helpers shared by the sweep kernels (and tools/ microbenchmarks):
// fp64 MFMA wrapper, half-wave lane broadcast, fp64 rsqrt, and the per-half-wave
// register Cholesky factorisations used for the K x K systems of dc:100,118,142.
#pragma once
#include <hip/hip_runtime.h>
#include "dcfm_internal.h"
#include "philox.h"

#include <type_traits>
#include <utility>

namespace dcfm {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d4 mfma16x16x4(double a, double b, d4 c) {
    // v_mfma_f64_16x16x4_f64: A[i=lane&15][k=lane>>4], B[k=lane>>4][j=lane&15],
    // C/D: col = lane&15, row = (lane>>4) + 4*reg
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// the same product with A negated by the instruction's neg modifier (blgp bit 0 of an f64 MFMA on
// gfx950: neg:[1,0,0]) -- bit for bit (-a) b + c, without a VALU sign flip of the operand
__device__ __forceinline__ d4 mfma16x16x4_na(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
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

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1 (DPP lane
// selectors and per-step register choices must be constants)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// value of lane LANE of this lane's 16-lane DPP row (v_mov_b32_dpp row_newbcast)
template <int LANE>
__device__ __forceinline__ double bcast16(double v) {
    static_assert(LANE >= 0 && LANE < 16, "row_newbcast lane");
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + LANE, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + LANE, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Canonical shard sum, independent of the rank count: sum_{m < n} x_m evaluated as the
// left-complete binary tree T(0, n) = T(0, h) + T(h, n - h), h = the largest power of two
// below n.  A rank's G consecutive shards (G a power of two, offset a multiple of G) are
// one subtree, and the tree over the ranks' subtotals has the same shape, so the per-rank
// sums combined over ranks reproduce T(0, g) bit for bit: the sweep gives the same numbers
// on 1, 2, 4 or 8 GPUs (the X message sum dc:120-124 and the A sum dc:117).  Evaluated as
// a binary counter: after i pushes, level l holds a finished 2^l-subtree iff bit l of i is
// set.  Levels stay in registers (unrolled, constant indices); n < 2^TREE_LEVELS.
constexpr int TREE_LEVELS = 16;
template <class T, int L = TREE_LEVELS>
struct TreeSum {
    T s[L];
    int i = 0;
    // static_for: the level indices are constants from the start, so s[] is promoted to registers
    __device__ __forceinline__ void push(T v) {
        bool open = true;   // still carrying
        static_for<L>([&](auto Q) {
            if (open) {
                if ((i >> Q) & 1) {
                    v = s[Q] + v;
                } else {
                    s[Q] = v;
                    open = false;
                }
            }
        });
        ++i;
    }
    // right to left: the smallest finished subtree is the rightmost
    __device__ __forceinline__ T total() const {
        T acc{};
        bool have = false;
        static_for<L>([&](auto Q) {
            if ((i >> Q) & 1) {
                acc = have ? s[Q] + acc : s[Q];
                have = true;
            }
        });
        return acc;
    }
};
// sum_{k < n} load(k) in the canonical tree order; the loads go out in batches of B
// (predicated, all in flight together) before the batch is pushed
template <class T, int B = 8, int L = TREE_LEVELS, class F>
__device__ __forceinline__ T tree_sum_f(int n, F &&load) {
    TreeSum<T, L> ts;
    for (int k = 0; k < n; k += B) {
        T v[B];
        static_for<B>([&](auto U) { if (k + U < n) v[U] = load(k + U); });
        static_for<B>([&](auto U) { if (k + U < n) ts.push(v[U]); });
    }
    return ts.total();
}
// sum_{k < n} src[k * stride] in the canonical tree order
__device__ __forceinline__ double tree_sum(const double *__restrict__ src, int n, size_t stride) {
    return tree_sum_f<double>(n, [&](int k) { return src[(size_t)k * stride]; });
}

// Agent-scope (all XCDs) coherent access for data handed between blocks of one launch:
// relaxed atomics bypass the non-coherent per-XCD L2 copies (sc1), no L2 flush needed.
__device__ __forceinline__ void st_agent(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// 1/sqrt(x): hardware estimate + one third-order (Halley-type) step y (1 + e/2 + 3e^2/8), e = 1 - x y^2
// (6 operations instead of rsqrt_f64's 9).  Measured on gfx950 (tools/dev/rsq_acc.hip, 4M arguments over
// 2^-100 .. 2^100): max relative error 0.624 x 2^-52, as rsqrt_f64 (0.622); the estimate alone 2^-24.2
__device__ __forceinline__ double rsqrt_f64_h(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double e = fma(-x * y, y, 1.0);
    return fma(y * e, fma(e, 0.375, 0.5), y);
}

// XCD-aware block remap (bijective): hardware deals consecutive block ids
// round-robin over the 8 XCDs; give each XCD a contiguous range of work items
// so that blocks sharing operands (one shard's tiles) share one L2.
__device__ __forceinline__ int xcd_remap(int b, int total) {
    const int xcd = b & 7, slot = b >> 3;
    const int q = total >> 3, rem = total & 7;
    return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + slot;
}

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

// standard gamma of the delta site, h = 0-based factor index (dc:158,163): the injected
// buffer, or — generated draws — the counter-addressed Philox variate itself (the value
// k_draws writes), so the delta chain never depends on which draw-batch slot holds its
// iteration (k_wcol runs iteration t's chain during iteration t+1)
__device__ inline double delta_G(const Dims &d, const DrawsDev &dr, int64_t iter, int mg, int h) {
    if (d.inject) return dr.Gdelta[((size_t)(iter - dr.first_iter) * d.g + mg) * d.K + h];
    const double shape = (h == 0) ? d.ad1 + 0.5 * d.P * d.K : d.ad2 + 0.5 * d.P * (d.K - h);
    return Rng(d.seed).gamma(shape, SITE_DELTA, (uint32_t)mg, 0, (uint32_t)h, (uint32_t)iter);
}

// eta = sqrt(rho) X + sqrt(1-rho) Z    (dc:81,133) — one definition for every use, with the
// contraction spelled out: left to fp-contract, hipcc fused either product depending on the
// surrounding code, so two instantiations of one kernel (k_cpass with and without the parity
// split) gave different last bits
__device__ __forceinline__ double eta_of(double sr, double s1r, double x, double z) {
    return fma(sr, x, s1r * z);
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

// ----------------------------------------------------------------------------
// 2-column-blocked register Cholesky (16 serial steps instead of 32).
// Layout of the LDS image P (pair-packed lower L): column pair j = (2j, 2j+1),
// rows c >= 2j, entry (c, e) at pb2(j) + 2 (c - 2j) + e, so L[c][2j] and
// L[c][2j+1] are one 16-byte read; then KP slots of 1/L[k][k] and KP scratch.
// Lane r = lane & 31 of each half-wave holds row r in q[] (entries c <= r read).
// Optional fused forward solve: bv holds b_r; vr returns (L^{-1} b)_r.
// ----------------------------------------------------------------------------
__host__ __device__ constexpr int pb2(int j) { return 64 * j - 2 * j * (j - 1); }
constexpr int PACK2 = pb2(KP / 2);
constexpr int P2STRIDE = PACK2 + 2 * KP;
__device__ __forceinline__ int p2idx(int c, int k) { return pb2(k >> 1) + 2 * (c - (k & ~1)) + (k & 1); }

template <bool FWD>
__device__ __forceinline__ void chol2_rows(double (&q)[KP], double *P, int r, bool upper, double bv,
                                           double &vr) {
#pragma unroll
    for (int j = 0; j < KP / 2; ++j) {
        const int k = 2 * j;
        // 2x2 diagonal block, factored redundantly in every lane
        const double a = readsel(q[k], k, upper);
        const double b = readsel(q[k], k + 1, upper);
        const double c2 = readsel(q[k + 1], k + 1, upper);
        const double i00 = rsqrt_f64(a);
        const double l00 = a * i00;
        const double l10 = b * i00;
        const double d11 = c2 - l10 * l10;
        const double i11 = rsqrt_f64(d11);
        const double l11 = d11 * i11;
        double lr0, lr1;
        if (r > k + 1) {
            lr0 = q[k] * i00;
            lr1 = (q[k + 1] - lr0 * l10) * i11;
        } else if (r == k + 1) {
            lr0 = l10;
            lr1 = l11;
        } else if (r == k) {
            lr0 = l00;
            lr1 = 0.0;
        } else {
            lr0 = 0.0;
            lr1 = 0.0;
        }
        q[k] = lr0;
        q[k + 1] = lr1;
        if (r >= k) {
            d2 v;
            v.x = lr0;
            v.y = lr1;
            *reinterpret_cast<d2 *>(P + pb2(j) + 2 * (r - k)) = v;
        }
        if (r == k) {
            d2 v;
            v.x = i00;
            v.y = i11;
            *reinterpret_cast<d2 *>(P + PACK2 + k) = v;
        }
        if (FWD) {   // v_k = b_k / L_kk ; v_{k+1} = (b_{k+1} - L_{k+1,k} v_k) / L_{k+1,k+1}
            const double v0 = readsel(bv, k, upper) * i00;
            const double v1 = (readsel(bv, k + 1, upper) - l10 * v0) * i11;
            if (r == k) vr = v0;
            if (r == k + 1) vr = v1;
            if (r > k + 1) bv -= lr0 * v0 + lr1 * v1;
        }
#pragma unroll
        for (int c = k + 2; c < KP; ++c) {
            const d2 lc = *reinterpret_cast<const d2 *>(P + pb2(j) + 2 * (c - k));
            q[c] -= lr0 * lc.x + lr1 * lc.y;
        }
#pragma unroll
        for (int c = k + 2; c < KP; ++c) asm volatile("" : "+v"(q[c]));
    }
}

constexpr int TS16 = 16;

// value of x held by lane 4*(lane/4) + J (DPP quad_perm [J,J,J,J])
template <int J>
__device__ __forceinline__ double quad_bcast(double x) {
    constexpr int ctrl = J | (J << 2) | (J << 4) | (J << 6);
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// 1/x to full fp64 precision from the hardware estimate: e = 1 - x y, y (1 + e + e^2 + e^3)
// (error e^4; four dependent operations after v_rcp_f64)
__device__ __forceinline__ double rcp_f64(double x) {
    const double y = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, y, 1.0);
    return fma(y, fma(fma(e, e, e), e, e), y);
}

// one step k = 4 kk + J of chol_inv16 (below); explicit scalars keep it in registers.
// Elimination in LDL' form: the update a_rc -= a_rk a_ck / a_kk (= l_r l_c) and the unit
// inverse W_r -= (a_rk / a_kk) W_k need only 1/a_kk, so the per-pivot chain is readlane ->
// rcp -> multiplier -> update, with no square root; the LDS hand-off (column k below the
// pivot, row k of W, both unscaled) is issued first and overlaps it.  The pivot a_kk = d_k
// is kept by row k's lanes for the final scaling L^{-1} = D^{-1/2} W.
template <int J>
__device__ __forceinline__ void chol16_step(double &a0, double &a1, double &a2, double &a3, double &R0, double &R1,
                                            double &R2, double &R3, double &dr, int kk, int r, int cg,
                                            double *lds_l, double *lds_u) {
    const int k = 4 * kk + J;
    const double v = quad_bcast<J>(a0);                         // a[r][k]
    lds_l[r] = (r > k) ? v : 0.0;       // the quad's 4 lanes store the same value: no exec-mask branch
    if (r == k) {
        lds_u[cg] = R0; lds_u[4 + cg] = R1; lds_u[8 + cg] = R2; lds_u[12 + cg] = R3;
    }
    __builtin_amdgcn_wave_barrier();
    const double *pl = lds_l + 4 * kk + cg;
    const double l0 = pl[0], l1 = pl[4], l2 = pl[8], l3 = pl[12];
    const double u0 = lds_u[cg], u1 = lds_u[4 + cg], u2 = lds_u[8 + cg], u3 = lds_u[12 + cg];
    __builtin_amdgcn_sched_barrier(0);                          // the reads are in flight during the chain
    const double piv = readlane_d(a0, 4 * k + J);
    const double f = (r > k) ? v * rcp_f64(piv) : 0.0;
    a0 = fma(-f, l0, a0); a1 = fma(-f, l1, a1); a2 = fma(-f, l2, a2); a3 = fma(-f, l3, a3);
    R0 = fma(-f, u0, R0); R1 = fma(-f, u1, R1); R2 = fma(-f, u2, R2); R3 = fma(-f, u3, R3);
    dr = (r == k) ? piv : dr;
    __builtin_amdgcn_wave_barrier();
}

// Cholesky factor and inverse of the 16x16 diagonal block at (o, o) of Sm (lower
// triangle read) on one wave: writes Ub(o.., o..) = L^{-1} (zeros above the diagonal).
// The one-block kernels run this cold every iteration, so the code is a rolled loop and
// the per-step latency chain is short: lane = 4 r + cg holds row r, columns 4 i + cg
// (i = 0..3) of the working matrix in a0..a3 (shifted one column group per outer step,
// so the pivot column is always a0) and of the unit inverse W (L = L1 D^{1/2}, W = L1^{-1})
// in R0..R3.  Step k: pivot by readlane, a_rk by a DPP quad broadcast, one LDS round trip
// hands out column k (lds_l, 32 slots, the upper 16 zero) and row k of W (lds_u, 16 slots);
// at the end each row r scales W_r by 1/sqrt(d_r).
// COLMAJ: Ub is written column-major (element (r, c) at c LDP + r; tile_linalg.h layout)
template <int LDP, bool COLMAJ = false>
__device__ __forceinline__ void chol_inv16_p(const double *Sm, int o, double *Ub, double *lds_l, double *lds_u,
                                             int lane) {
    const int r = lane >> 2, cg = lane & 3;
    const double *srow = Sm + (o + r) * LDP + o + cg;   // entries above the diagonal are never consumed
    double a0 = srow[0], a1 = srow[4], a2 = srow[8], a3 = srow[12];
    double R0 = (cg == r) ? 1.0 : 0.0, R1 = (4 + cg == r) ? 1.0 : 0.0;
    double R2 = (8 + cg == r) ? 1.0 : 0.0, R3 = (12 + cg == r) ? 1.0 : 0.0;
    double dr = 1.0;
    if (lane < 16) lds_l[16 + lane] = 0.0;
#pragma unroll 1
    for (int kk = 0; kk < 4; ++kk) {
        chol16_step<0>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        chol16_step<1>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        chol16_step<2>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        chol16_step<3>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u);
        a0 = a1; a1 = a2; a2 = a3; a3 = 0.0;
    }
    const double ik = rsqrt_f64(dr);                     // 1 / L_rr
    if (COLMAJ) {
        double *ucol = Ub + (o + cg) * LDP + o + r;
        ucol[0] = R0 * ik; ucol[4 * LDP] = R1 * ik; ucol[8 * LDP] = R2 * ik; ucol[12 * LDP] = R3 * ik;
    } else {
        double *urow = Ub + (o + r) * LDP + o + cg;
        urow[0] = R0 * ik; urow[4] = R1 * ik; urow[8] = R2 * ik; urow[12] = R3 * ik;
    }
}
// chol_inv16_p with its 16 pivot steps unrolled, calling hook(std::integral_constant<int, k>) once step
// k's LDS hand-off is in flight: independent work (k_lambda_w's look-ahead: the rest of the previous
// block column's trailing MFMAs) issued into the pivot chain's latency.  Same operations on the block as
// chol_inv16_p, so the same bits.
template <int J, class Hook>
__device__ __forceinline__ void chol16_step_h(double &a0, double &a1, double &a2, double &a3, double &R0, double &R1,
                                              double &R2, double &R3, double &dr, int kk, int r, int cg,
                                              double *lds_l, double *lds_u, Hook &&hook) {
    const int k = 4 * kk + J;
    const double v = quad_bcast<J>(a0);                         // a[r][k]
    lds_l[r] = (r > k) ? v : 0.0;
    if (r == k) {
        lds_u[cg] = R0; lds_u[4 + cg] = R1; lds_u[8 + cg] = R2; lds_u[12 + cg] = R3;
    }
    __builtin_amdgcn_wave_barrier();
    const double *pl = lds_l + 4 * kk + cg;
    const double l0 = pl[0], l1 = pl[4], l2 = pl[8], l3 = pl[12];
    const double u0 = lds_u[cg], u1 = lds_u[4 + cg], u2 = lds_u[8 + cg], u3 = lds_u[12 + cg];
    __builtin_amdgcn_sched_barrier(0);                          // the reads are in flight during the chain
    hook();
    const double piv = readlane_d(a0, 4 * k + J);
    const double f = (r > k) ? v * rcp_f64(piv) : 0.0;
    a0 = fma(-f, l0, a0); a1 = fma(-f, l1, a1); a2 = fma(-f, l2, a2); a3 = fma(-f, l3, a3);
    R0 = fma(-f, u0, R0); R1 = fma(-f, u1, R1); R2 = fma(-f, u2, R2); R3 = fma(-f, u3, R3);
    dr = (r == k) ? piv : dr;
    __builtin_amdgcn_wave_barrier();
}
template <int LDP, class Hook>
__device__ __forceinline__ void chol_inv16_hook(const double *Sm, int o, double *Ub, double *lds_l, double *lds_u,
                                                int lane, Hook &&hook) {
    const int r = lane >> 2, cg = lane & 3;
    const double *srow = Sm + (o + r) * LDP + o + cg;
    double a0 = srow[0], a1 = srow[4], a2 = srow[8], a3 = srow[12];
    double R0 = (cg == r) ? 1.0 : 0.0, R1 = (4 + cg == r) ? 1.0 : 0.0;
    double R2 = (8 + cg == r) ? 1.0 : 0.0, R3 = (12 + cg == r) ? 1.0 : 0.0;
    double dr = 1.0;
    if (lane < 16) lds_l[16 + lane] = 0.0;
    static_for<4>([&](auto KK) {
        constexpr int kk = decltype(KK)::value;
        chol16_step_h<0>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u,
                         [&] { hook(std::integral_constant<int, 4 * kk>{}); });
        chol16_step_h<1>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u,
                         [&] { hook(std::integral_constant<int, 4 * kk + 1>{}); });
        chol16_step_h<2>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u,
                         [&] { hook(std::integral_constant<int, 4 * kk + 2>{}); });
        chol16_step_h<3>(a0, a1, a2, a3, R0, R1, R2, R3, dr, kk, r, cg, lds_l, lds_u,
                         [&] { hook(std::integral_constant<int, 4 * kk + 3>{}); });
        a0 = a1; a1 = a2; a2 = a3; a3 = 0.0;
    });
    const double ik = rsqrt_f64(dr);                     // 1 / L_rr
    double *urow = Ub + (o + r) * LDP + o + cg;
    urow[0] = R0 * ik; urow[4] = R1 * ik; urow[8] = R2 * ik; urow[12] = R3 * ik;
}
// U = L^{-1} (L L' = S) of a 16x16 SPD tile held in registers in the fp64 MFMA C/D layout (lane
// (c16, q) holds S[q + 4g][c16] in element g; its upper triangle is read), returned in the same
// layout, by 4 x 4 blocks with no LDS: block step b reads S_bb (10 readlanes), factors it and
// forms M_b = L_bb^{-1} uniformly in every lane, then four fp64 MFMAs:
//   P   = S_{.b} M_b'      panel L_{.b}       (A = M_b, B = block row b of S: element b, as held)
//   V   = M_b W_{b.}       block row b of U   (W: the running I - sum L_{.j} U_{j.}, W_0 = I)
//   S  -= P_m P_m'          Schur complement   (P_m: P on the rows below block b, else 0)
//   W  -= P_m V
// P's and V's element 0 is the A / B operand of the next product as it lands (lane (r, k) holds
// P[r][k], lane (c, k) V[k][c]), so the per-block chain is readlanes -> 4 x 4 factor -> two
// dependent MFMAs, four times, instead of 16 pivot round trips through LDS.  hook(b) runs once
// block b's readlanes are issued (independent MFMAs into the chain's latency).  A non-positive
// pivot gives NaN (rsqrt of a negative or zero number), which the caller's finite check reports
// as the reference's chol failure (dc:142).
template <class Hook>
__device__ __forceinline__ d4 chol_inv16_blk(d4 S, int lane, Hook &&hook) {
    const int c16 = lane & 15, q = lane >> 4;
    d4 W, U;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        W[g] = (q + 4 * g == c16) ? 1.0 : 0.0;
        U[g] = 0.0;
    }
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    static_for<4>([&](auto BC) {
        constexpr int b = decltype(BC)::value, o = 4 * b;
        // S_bb[m][n] (m <= n) = S[o + m][o + n]: lane 16 m + o + n, element b
        const double s00 = readlane_d(S[b], o), s01 = readlane_d(S[b], o + 1);
        const double s02 = readlane_d(S[b], o + 2), s03 = readlane_d(S[b], o + 3);
        const double s11 = readlane_d(S[b], 16 + o + 1), s12 = readlane_d(S[b], 16 + o + 2);
        const double s13 = readlane_d(S[b], 16 + o + 3), s22 = readlane_d(S[b], 32 + o + 2);
        const double s23 = readlane_d(S[b], 32 + o + 3), s33 = readlane_d(S[b], 48 + o + 3);
        hook(std::integral_constant<int, b>{});
        const double i0 = rsqrt_f64_h(s00);
        const double l10 = s01 * i0, l20 = s02 * i0, l30 = s03 * i0;
        const double i1 = rsqrt_f64_h(fma(-l10, l10, s11));
        const double l21 = fma(-l20, l10, s12) * i1, l31 = fma(-l30, l10, s13) * i1;
        const double i2 = rsqrt_f64_h(fma(-l21, l21, fma(-l20, l20, s22)));
        const double l32 = fma(-l31, l21, fma(-l30, l20, s23)) * i2;
        const double i3 = rsqrt_f64_h(fma(-l32, l32, fma(-l31, l31, fma(-l30, l30, s33))));
        const double m10 = -(l10 * i0) * i1;
        const double m21 = -(l21 * i1) * i2;
        const double m20 = -fma(l21, m10, l20 * i0) * i2;
        const double m32 = -(l32 * i2) * i3;
        const double m31 = -fma(l32, m21, l31 * i1) * i3;
        const double m30 = -fma(l32, m20, fma(l31, m10, l30 * i0)) * i3;
        // A operand: lane (k = c16, m = q) = lane 16 m + k holds M_b[k][m] (rows k >= 4 zero); one
        // select per entry on a constant lane (a nested choice by c16 and q compiled to branches)
        double a = lane == 0 ? i0 : 0.0;
        a = lane == 1 ? m10 : a;
        a = lane == 17 ? i1 : a;
        a = lane == 2 ? m20 : a;
        a = lane == 18 ? m21 : a;
        a = lane == 34 ? i2 : a;
        a = lane == 3 ? m30 : a;
        a = lane == 19 ? m31 : a;
        a = lane == 35 ? m32 : a;
        a = lane == 51 ? i3 : a;
        const d4 P = mfma16x16x4(a, S[b], zero);
        const d4 V = mfma16x16x4(a, W[b], zero);
        U[b] = V[0];
        if constexpr (b < 3) {
            const double pm = (c16 >= o + 4) ? P[0] : 0.0;
            S = mfma16x16x4_na(pm, pm, S);
            W = mfma16x16x4_na(pm, V[0], W);
        }
    });
    return U;
}

__device__ __forceinline__ void chol_inv16(const double (*Sm)[KP + 1], int o, double (*Ub)[KP + 1],
                                           double *lds_l, double *lds_u, int lane) {
    chol_inv16_p<KP + 1>(&Sm[0][0], o, &Ub[0][0], lds_l, lds_u, lane);
}

// DPP helpers: a double from lane CTRL-permuted within its 16-lane row; sum over the row
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// v of lane l ^ 16 / l ^ 32 (the partner row of the wave) by gfx950's v_permlane16_swap /
// v_permlane32_swap: a register exchange between rows, where a lane shuffle (ds_bpermute) costs an LDS
// round trip.  With both operands v the swap leaves the partner's value in the second result for the
// lanes whose partner is above them and in the first for the others.
__device__ __forceinline__ double xor16_d(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const bool up = (__lane_id() & 16) == 0;
    return __hiloint2double(up ? b[1] : b[0], up ? a[1] : a[0]);
}
__device__ __forceinline__ double xor32_d(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const bool up = __lane_id() < 32;
    return __hiloint2double(up ? b[1] : b[0], up ? a[1] : a[0]);
}
__device__ __forceinline__ double rowsum16(double v) {
    v += dpp_d<0xB1>(v);     // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);     // quad_perm [2,3,0,1]
    v += dpp_d<0x124>(v);    // row_ror:4
    v += dpp_d<0x128>(v);    // row_ror:8
    return v;
}

// U = L^{-1}, L = chol of the KP x KP (= 32) SPD matrix whose lower triangle is in
// Sm, on one wave: two chol_inv16 diagonal blocks plus fp64 MFMA for the rest:
//   L21 = A21 U11',  S22 <- S22 - L21 L21'  (in place in Sm),  U21 = -U22 L21 U11.
// Wk: 16 x (KP+1) scratch (L21).  Upper triangle of Us is written 0.
__device__ __forceinline__ void chol_inv32(double (*Sm)[KP + 1], double (*Us)[KP + 1], double (*Wk)[KP + 1],
                                           double *lds_l, double *lds_u, int lane) {
    static_assert(KP == 32, "narrow operator path");
    const int i = lane & 15, q = lane >> 4;
    chol_inv16(Sm, 0, Us, lds_l, lds_u, lane);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    d4 l21 = {0.0, 0.0, 0.0, 0.0};                       // L21[q+4g][i] = sum_k A21[.][k] U11[i][k]
#pragma unroll
    for (int s = 0; s < 4; ++s) l21 = mfma16x16x4(Sm[16 + i][4 * s + q], Us[i][4 * s + q], l21);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        Wk[q + 4 * g][i] = l21[g];
        Us[q + 4 * g][16 + i] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    d4 s22;
#pragma unroll
    for (int g = 0; g < 4; ++g) s22[g] = Sm[16 + q + 4 * g][16 + i];
#pragma unroll
    for (int s = 0; s < 4; ++s) s22 = mfma16x16x4_na(Wk[i][4 * s + q], Wk[i][4 * s + q], s22);
#pragma unroll
    for (int g = 0; g < 4; ++g) Sm[16 + q + 4 * g][16 + i] = s22[g];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    chol_inv16(Sm, 16, Us, lds_l, lds_u, lane);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    d4 x = {0.0, 0.0, 0.0, 0.0};                         // X = L21 U11  (NN)
#pragma unroll
    for (int s = 0; s < 4; ++s) x = mfma16x16x4(Wk[i][4 * s + q], Us[4 * s + q][i], x);
    d4 u21 = {0.0, 0.0, 0.0, 0.0};                       // U21 = -U22 X, X in C/D layout = B operand
#pragma unroll
    for (int g = 0; g < 4; ++g) u21 = mfma16x16x4_na(Us[16 + i][16 + q + 4 * g], x[g], u21);
#pragma unroll
    for (int g = 0; g < 4; ++g) Us[16 + q + 4 * g][i] = u21[g];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// One 16x16 tile of a 32x32 product in LDS, fp64 MFMA (whole wave, 8 k-steps):
//   NT: C = A B'  (C[a][c] = sum_b A[a][b] B[c][b]);   NN: C = A B (B[b][c]).
// Tile (ti, tj); returns the C/D fragment: lane (j = lane&15, q = lane>>4) holds
// C[16 ti + q + 4 g][16 tj + j], g = 0..3.
template <bool NT>
__device__ __forceinline__ d4 mfma_tile32(const double (*A)[KP + 1], const double (*B)[KP + 1], int ti, int tj,
                                          int lane) {
    const int i = lane & 15, k = lane >> 4;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KP / 4; ++s) {
        const double a = A[16 * ti + i][4 * s + k];
        const double b = NT ? B[16 * tj + i][4 * s + k] : B[4 * s + k][16 * tj + i];
        acc = mfma16x16x4(a, b, acc);
    }
    return acc;
}

// U = L^{-1} from the pair-packed image P of chol2_rows: lane j (threads 0..31)
// forward-substitutes column j; result in Us[a][j].
__device__ __forceinline__ void lower_inverse2(const double *P, double (*Us)[KP + 1], int t) {
    if (t >= KP) return;
    const int j = t;
    double u[KP];
#pragma unroll
    for (int a = 0; a < KP; ++a) {
        double acc = (a == j) ? 1.0 : 0.0;
#pragma unroll
        for (int b = 0; b < a; ++b) acc -= P[pb2(b >> 1) + 2 * (a - (b & ~1)) + (b & 1)] * u[b];
        u[a] = acc * P[PACK2 + a];
    }
#pragma unroll
    for (int a = 0; a < KP; ++a) Us[a][j] = u[a];
}

// ----------------------------------------------------------------------------
// U = L^{-1} from the LDS image Lt of a lower Cholesky factor (chol_rows): lane j
// (threads 0..31) forward-substitutes column j; result in Us[a][j].
// ----------------------------------------------------------------------------
__device__ __forceinline__ void lower_inverse(const double (*Lt)[LS], double (*Us)[KP + 1], int t) {
    if (t >= KP) return;
    const int j = t;
    double u[KP];
#pragma unroll
    for (int a = 0; a < KP; ++a) {
        double acc = (a == j) ? 1.0 : 0.0;
#pragma unroll
        for (int b = 0; b < a; ++b) acc -= Lt[b][a] * u[b];    // L[a][b] = Lt[b][a]
        u[a] = acc * Lt[a][KP];
    }
#pragma unroll
    for (int a = 0; a < KP; ++a) Us[a][j] = u[a];
}

}  // namespace dcfm
