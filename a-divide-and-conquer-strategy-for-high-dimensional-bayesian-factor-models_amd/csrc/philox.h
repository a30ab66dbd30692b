// Counter-based on-device RNG for the Gibbs sweep (replaces MATLAB's global
// stream consumed at dc:104,126,142,150,158,163,170 — SURVEY Appendix B).
//
// Philox4x32-10 (Salmon et al., SC'11).  Every variate is addressed by a
// counter built from (iteration, site, global shard, row, index), so a run is
// independent of the number of GPUs, of launch geometry and of scheduling.
//
//   ctr.w = iter            (1-based dc:90 iteration; 0 for diagnostics)
//   ctr.z = site << 24 | global shard
//   ctr.y = row             (i for Z/X sites, j for loading sites)
//   ctr.x = normals: index>>1 (one call -> two Box-Muller normals)
//           gammas : 0x80000000 | index << 8 | attempt << 1 | {0: normal, 1: uniform}
//
// Standard normal: Box-Muller on two 53-bit uniforms in (0,1].
// Standard gamma(a >= 1): Marsaglia-Tsang squeeze/rejection (every gamma shape the
// reference's defaults draw is >= 1: df/2+0.5 = 2, as+n/2, ad+P*K/2 ...); shapes 1 and 2
// (the psi site uses 2) as a sum of exponentials; a < 1 (other hyper-parameters) by the
// boost Ga(a) = Ga(a+1) U^(1/a).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcfm {

enum RngSite : uint32_t {
    SITE_Z = 1,      // dc:104  N(0,1)  K x n x g
    SITE_X = 2,      // dc:126  N(0,1)  K x n
    SITE_LAMBDA = 3, // dc:142  N(0,1)  K x P x g
    SITE_PSI = 4,    // dc:150  Ga(df/2+0.5)
    SITE_DELTA = 5,  // dc:158,163  Ga(ad + ...)
    SITE_PS = 6,     // dc:170  Ga(as+n/2)
    SITE_INIT_PS = 7,     // dc:69  Ga(as)     P x 1 x g   (dcfm_init_state, iter 0)
    SITE_INIT_X = 8,      // dc:71  N(0,1)     n x K
    SITE_INIT_PSI = 9,    // dc:73  Ga(df/2)   P x K x g
    SITE_INIT_Z = 10,     // dc:80  N(0,1)     n x K x g
    SITE_INIT_D1 = 11,    // dc:83  Ga(ad1)    delta(1,:,m)
    SITE_INIT_D2 = 12,    // dc:83  Ga(ad2)    delta(2:K,:,m)
    SITE_DIAG = 15,  // dcfm_rng_fill
};

struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one 32x32 -> 64 product per multiplier (v_mad_u64_u32: lo and hi in one instruction)
        const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// 53-bit uniform in (0, 1]
__device__ __forceinline__ double u01_53(uint32_t hi, uint32_t lo) {
    const uint64_t v = ((static_cast<uint64_t>(hi) << 32) | lo) >> 11;
    return static_cast<double>(v + 1) * 0x1.0p-53;
}

// ---- transcendental kernels for arguments produced by u01_53 (u in [2^-53, 1]) ----
// The library log / sqrt / sincospi handle every IEEE case (~350 instructions per
// Box-Muller pair with Philox); these cover exactly the uniforms' range in ~1/3 of
// that, to within a few ulp (the variates are checked statistically, tests/test_gpu_rng.py).

// log(u), u in [2^-106, 1] (a uniform or the product of two): u = 2^e m, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s),
// s = (m-1)/(m+1), |s| <= 0.1716: series to s^23 (truncation < 1e-18 relative)
__device__ __forceinline__ double log_u01(double u) {
    double m = __builtin_amdgcn_frexp_mant(u);              // [0.5, 1)
    int e = __builtin_amdgcn_frexp_exp(u);
    const bool lo = m < 0.70710678118654752440;
    m = lo ? 2.0 * m : m;
    e = lo ? e - 1 : e;
    const double a = m - 1.0, b = m + 1.0;
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    r = fma(fma(-b, r, 1.0), r, r);
    double sv = a * r;
    sv = fma(fma(-sv, b, a), r, sv);                        // s with a residual correction
    const double z = sv * sv;
    double q = 1.0 / 23;
    q = fma(q, z, 1.0 / 21); q = fma(q, z, 1.0 / 19); q = fma(q, z, 1.0 / 17);
    q = fma(q, z, 1.0 / 15); q = fma(q, z, 1.0 / 13); q = fma(q, z, 1.0 / 11);
    q = fma(q, z, 1.0 / 9);  q = fma(q, z, 1.0 / 7);  q = fma(q, z, 1.0 / 5);
    q = fma(q, z, 1.0 / 3);
    const double s2 = 2.0 * sv;
    const double lm = fma(s2 * z, q, s2);                   // log m
    const double fe = (double)e;
    return fma(fe, 6.93147180369123816490e-01, fma(fe, 1.90821492927058770002e-10, lm));   // e ln2 (hi + lo)
}

// sqrt(x), x >= 0 (0 -> 0): reciprocal-sqrt estimate, two Newton steps, one on the root
__device__ __forceinline__ double sqrt_nonneg(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * fma(-0.5 * x * y, y, 1.5);
    y = y * fma(-0.5 * x * y, y, 1.5);
    double r = x * y;
    r = fma(0.5 * y, fma(-r, r, x), r);
    return x > 0.0 ? r : 0.0;
}

// sin, cos of 2 pi u, u in (0, 1]: t = 4u quarter turns (exact), nearest quadrant q,
// phi = (t - q) pi/2 in [-pi/4, pi/4], Taylor to phi^17 / phi^18
__device__ __forceinline__ void sincos_2pi_u01(double u, double &sn, double &cs) {
    const double t = 4.0 * u;
    const double q = __builtin_rint(t);
    const double f = t - q;
    const double ph = fma(f, 1.57079632679489655800e+00, f * 6.12323399573676603587e-17);
    const double z = ph * ph;
    double ps = 2.81145725434552076319e-15;                // 1/17!
    ps = fma(ps, z, -7.64716373181981647590e-13);          // -1/15!
    ps = fma(ps, z, 1.60590438368216145994e-10);           // 1/13!
    ps = fma(ps, z, -2.50521083854417187751e-08);          // -1/11!
    ps = fma(ps, z, 2.75573192239858906526e-06);           // 1/9!
    ps = fma(ps, z, -1.98412698412698412526e-04);          // -1/7!
    ps = fma(ps, z, 8.33333333333333321769e-03);           // 1/5!
    ps = fma(ps, z, -1.66666666666666657415e-01);          // -1/3!
    const double sp = fma(ph * z, ps, ph);
    double pc = 1.56192069685862264622e-16;                // 1/18!
    pc = fma(pc, z, -4.77947733238738529744e-14);          // -1/16!
    pc = fma(pc, z, 1.14707455977297247139e-11);           // 1/14!
    pc = fma(pc, z, -2.08767569878680989792e-09);          // -1/12!
    pc = fma(pc, z, 2.75573192239858906526e-07);           // 1/10!
    pc = fma(pc, z, -2.48015873015873015873e-05);          // -1/8!
    pc = fma(pc, z, 1.38888888888888894189e-03);           // 1/6!
    pc = fma(pc, z, -4.16666666666666643537e-02);          // -1/4!
    pc = fma(pc, z, 0.5);
    const double cp = fma(-z, pc, 1.0);                    // 1 - z/2 + ...
    const int qi = (int)q & 3;
    const double s0 = (qi & 1) ? cp : sp, c0 = (qi & 1) ? sp : cp;
    sn = (qi & 2) ? -s0 : s0;
    cs = ((qi + 1) & 2) ? -c0 : c0;
}

struct Rng {
    uint32_t k0, k1;
    __device__ __forceinline__ Rng(uint64_t seed)
        : k0(static_cast<uint32_t>(seed)), k1(static_cast<uint32_t>(seed >> 32)) {}

    __device__ __forceinline__ u32x4 raw(uint32_t site, uint32_t shard, uint32_t row,
                                         uint32_t x, uint32_t iter) const {
        return philox4x32_10(u32x4{x, row, (site << 24) | (shard & 0xFFFFFFu), iter}, k0, k1);
    }

    // normals idx = 2q and 2q+1 of (site, shard, row, iter)
    __device__ __forceinline__ void normal2(uint32_t site, uint32_t shard, uint32_t row,
                                            uint32_t q, uint32_t iter, double &n0, double &n1) const {
        const u32x4 r = raw(site, shard, row, q, iter);
        const double u1 = u01_53(r.x, r.y), u2 = u01_53(r.z, r.w);
        const double rad = sqrt_nonneg(-2.0 * log_u01(u1));
        double s, c;
        sincos_2pi_u01(u2, s, c);
        n0 = rad * c;
        n1 = rad * s;
    }

    __device__ __forceinline__ double normal(uint32_t site, uint32_t shard, uint32_t row,
                                             uint32_t idx, uint32_t iter) const {
        double a, b;
        normal2(site, shard, row, idx >> 1, iter, a, b);
        return (idx & 1u) ? b : a;
    }

    // standard gamma(shape > 0): integer shapes 1, 2 inline (the psi site), shapes >= 1
    // Marsaglia & Tsang (2000), shapes below 1 by their boost Ga(a) = Ga(a + 1) U^(1/a)
    // (U from its own counter: attempt bits 1..6 of gamma_mt never reach bit 7)
    __device__ __forceinline__ double gamma(double shape, uint32_t site, uint32_t shard, uint32_t row,
                                            uint32_t idx, uint32_t iter) const {
        if (shape < 1.0) {
            const double g1 = gamma_mt(shape + 1.0, site, shard, row, idx, iter);
            const u32x4 b = raw(site, shard, row, 0x80000000u | ((idx & 0x7FFFFFu) << 8) | 0x80u, iter);
            return g1 * exp(log_u01(u01_53(b.x, b.y)) / shape);
        }
        if (shape == 1.0 || shape == 2.0) {
            // integer shape: sum of shape exponentials, -log(u1 [* u2]) — exact, no rejection; one
            // log of the product (>= 2^-106, a normal double) instead of a sum of two logs
            const u32x4 a = raw(site, shard, row, 0x80000000u | ((idx & 0x7FFFFFu) << 8), iter);
            const double u1 = u01_53(a.x, a.y);
            return -log_u01(shape == 1.0 ? u1 : u1 * u01_53(a.z, a.w));
        }
        return gamma_mt(shape, site, shard, row, idx, iter);
    }
    __device__ __forceinline__ double gamma_mt(double shape, uint32_t site, uint32_t shard, uint32_t row,
                                            uint32_t idx, uint32_t iter) const {
        const double d = shape - 1.0 / 3.0;
        const double c = 1.0 / sqrt(9.0 * d);
        double v = 1.0;
        for (uint32_t att = 0; att < 64; ++att) {
            const uint32_t base = 0x80000000u | ((idx & 0x7FFFFFu) << 8) | (att << 1);
            const u32x4 a = raw(site, shard, row, base, iter);
            const double u1 = u01_53(a.x, a.y), u2 = u01_53(a.z, a.w);
            double s, cs;
            sincos_2pi_u01(u2, s, cs);
            const double x = sqrt_nonneg(-2.0 * log_u01(u1)) * cs;
            v = 1.0 + c * x;
            if (v <= 0.0) continue;
            v = v * v * v;
            const u32x4 b = raw(site, shard, row, base | 1u, iter);
            const double u = u01_53(b.x, b.y);
            const double x2 = x * x;
            if (u < 1.0 - 0.0331 * x2 * x2) return d * v;
            if (log_u01(u) < 0.5 * x2 + d * (1.0 - v + log(v))) return d * v;
        }
        return d * (v > 0.0 ? v : 1.0);   // unreachable in practice (p(reject 64x) < 1e-80)
    }
};

}  // namespace dcfm
