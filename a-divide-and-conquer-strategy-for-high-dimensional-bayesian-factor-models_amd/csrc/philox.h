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
// Standard gamma(a >= 1): Marsaglia-Tsang squeeze/rejection (every gamma shape
// in the reference is >= 1: df/2+0.5 = 2, as+n/2, ad+P*K/2 ...); shapes 1 and 2
// (the psi site uses 2) as a sum of exponentials.
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
    SITE_DIAG = 15,  // dcfm_rng_fill
};

struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = M0 * c.x, hi0 = __umulhi(M0, c.x);
        const uint32_t lo1 = M1 * c.z, hi1 = __umulhi(M1, c.z);
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
        const double rad = sqrt(-2.0 * log(u1));
        double s, c;
        sincospi(2.0 * u2, &s, &c);
        n0 = rad * c;
        n1 = rad * s;
    }

    __device__ __forceinline__ double normal(uint32_t site, uint32_t shard, uint32_t row,
                                             uint32_t idx, uint32_t iter) const {
        double a, b;
        normal2(site, shard, row, idx >> 1, iter, a, b);
        return (idx & 1u) ? b : a;
    }

    // standard gamma(shape >= 1), Marsaglia & Tsang (2000)
    __device__ double gamma(double shape, uint32_t site, uint32_t shard, uint32_t row,
                            uint32_t idx, uint32_t iter) const {
        if (shape == 1.0 || shape == 2.0) {
            // integer shape: sum of shape exponentials, -log(u1 [* u2]) — exact, no rejection
            const u32x4 a = raw(site, shard, row, 0x80000000u | ((idx & 0x7FFFFFu) << 8), iter);
            const double u1 = u01_53(a.x, a.y);
            return shape == 1.0 ? -log(u1) : -log(u1 * u01_53(a.z, a.w));
        }
        const double d = shape - 1.0 / 3.0;
        const double c = 1.0 / sqrt(9.0 * d);
        double v = 1.0;
        for (uint32_t att = 0; att < 64; ++att) {
            const uint32_t base = 0x80000000u | ((idx & 0x7FFFFFu) << 8) | (att << 1);
            const u32x4 a = raw(site, shard, row, base, iter);
            const double u1 = u01_53(a.x, a.y), u2 = u01_53(a.z, a.w);
            double s, cs;
            sincospi(2.0 * u2, &s, &cs);
            const double x = sqrt(-2.0 * log(u1)) * cs;
            v = 1.0 + c * x;
            if (v <= 0.0) continue;
            v = v * v * v;
            const u32x4 b = raw(site, shard, row, base | 1u, iter);
            const double u = u01_53(b.x, b.y);
            const double x2 = x * x;
            if (u < 1.0 - 0.0331 * x2 * x2) return d * v;
            if (log(u) < 0.5 * x2 + d * (1.0 - v + log(v))) return d * v;
        }
        return d * (v > 0.0 ? v : 1.0);   // unreachable in practice (p(reject 64x) < 1e-80)
    }
};

}  // namespace dcfm
