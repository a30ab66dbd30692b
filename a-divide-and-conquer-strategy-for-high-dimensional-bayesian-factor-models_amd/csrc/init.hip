// On-device initial state (dc:68-87): the chain's starting point drawn
// from the same counter-based Philox stream as the sweep, written straight into the HBM
// layout, so start-up needs no host draws and no state upload (c5: 15 M normals and 3 M
// gammas).  Counters: iteration 0 (the sweep's iterations are 1-based) and the
// SITE_INIT_* sites; variate e of (site, global shard) uses row = e / 32, index = e % 32 —
// the dcfm_rng_fill convention, so the host can reproduce every variate, with
// e = MATLAB's linear index inside the shard's array:
//   ps0   e = j            ps = (1/bs) Ga(as)                 dc:69   omega = ps (Q1, dc:84)
//   X0    e = i + n k      X = N(0,1)            (shard 0)    dc:71
//   psi0  e = j + P k      psijh = (2/df) Ga(df/2)            dc:73
//   Z0    e = i + n k      Z = N(0,1)                         dc:80
//   delta e = h            delta(1) = bd1 Ga(ad1), delta(h>1) = bd2 Ga(ad2)   dc:83
//   tauh = cumprod(delta) per shard (dc:85), Plam = psijh .* tauh' (dc:86), Lambda = 0 (dc:70).
// delta / tau are drawn for all g shards on every rank (replicated state), the rest for
// the rank's local shards only; every rank's values are those of a one-rank run.
#include "dcfm_internal.h"
#include "philox.h"

namespace dcfm {

// one thread per global shard: delta, tau (buffer 0), padding 1
__global__ __launch_bounds__(64) void k_init_delta(Dims d, double *__restrict__ delta, double *__restrict__ tau) {
    const int mg = blockIdx.x * 64 + threadIdx.x;
    if (mg >= d.g) return;
    const Rng rng(d.seed);
    double cp = 1.0;
    for (int h = 0; h < d.kp; ++h) {
        double dv = 1.0, tv = 1.0;
        if (h < d.K) {
            dv = h == 0 ? d.bd1 * rng.gamma(d.ad1, SITE_INIT_D1, mg, 0, 0, 0)
                        : d.bd2 * rng.gamma(d.ad2, SITE_INIT_D2, mg, (uint32_t)h / 32, (uint32_t)h % 32, 0);
            cp = cp * dv;
            tv = cp;
        }
        delta[(size_t)mg * d.kp + h] = dv;
        tau[(size_t)mg * d.kp + h] = tv;
    }
}

__device__ __forceinline__ double init_normal(const Rng &rng, uint32_t site, int mg, int64_t e) {
    return rng.normal(site, (uint32_t)mg, (uint32_t)(e / 32), (uint32_t)(e % 32), 0);
}
__device__ __forceinline__ double init_gamma(const Rng &rng, double a, uint32_t site, int mg, int64_t e) {
    return rng.gamma(a, site, (uint32_t)mg, (uint32_t)(e / 32), (uint32_t)(e % 32), 0);
}

// grid-stride over the loading-row arrays [G][PP][KW], the shard factors [G][NP][KW], X
// [NP][KW] and ps / omega [G][PP]; padding written as zeros
__global__ __launch_bounds__(256) void k_init_state(Dims d, Bufs b, const double *__restrict__ tau) {
    const Rng rng(d.seed);
    const int KW = d.kp;
    const int64_t nrow = (int64_t)d.G * d.PP * KW, nz = (int64_t)d.G * d.NP * KW, nx = (int64_t)d.NP * KW;
    const int64_t np = (int64_t)d.G * d.PP;
    const int64_t total = nrow + nz + nx + np;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        if (e < nrow) {                                   // Lambda, psi, Plam
            const int k = (int)(e % KW);
            const int64_t r = e / KW;
            const int j = (int)(r % d.PP), m = (int)(r / d.PP), mg = d.shard0 + m;
            double psi = 0.0, plam = 0.0;
            if (j < d.P && k < d.K) {
                psi = (2.0 / d.df) * init_gamma(rng, d.df / 2.0, SITE_INIT_PSI, mg, (int64_t)j + (int64_t)d.P * k);
                plam = psi * tau[(size_t)mg * KW + k];
            }
            b.Lam[e] = 0.0;
            b.psi[e] = psi;
            b.Plam[e] = plam;
        } else if (e < nrow + nz) {                       // Z
            const int64_t q = e - nrow;
            const int k = (int)(q % KW);
            const int64_t r = q / KW;
            const int i = (int)(r % d.NP), m = (int)(r / d.NP);
            b.Z[q] = (i < d.n && k < d.K)
                         ? init_normal(rng, SITE_INIT_Z, d.shard0 + m, (int64_t)i + (int64_t)d.n * k) : 0.0;
        } else if (e < nrow + nz + nx) {                  // X (global, shard 0 counters)
            const int64_t q = e - nrow - nz;
            const int k = (int)(q % KW), i = (int)(q / KW);
            b.X[q] = (i < d.n && k < d.K) ? init_normal(rng, SITE_INIT_X, 0, (int64_t)i + (int64_t)d.n * k) : 0.0;
        } else {                                          // ps, omega (Q1: omega = ps at init)
            const int64_t q = e - nrow - nz - nx;
            const int j = (int)(q % d.PP), m = (int)(q / d.PP);
            const double v = j < d.P ? (1.0 / d.bs) * init_gamma(rng, d.as_, SITE_INIT_PS, d.shard0 + m, j) : 0.0;
            b.ps[q] = v;
            b.omega[q] = v;
        }
    }
}

void launch_init_state(const Dims &d, const Bufs &b, hipStream_t s) {
    hipLaunchKernelGGL(k_init_delta, dim3((d.g + 63) / 64), dim3(64), 0, s, d, b.delta, b.tau);
    hipLaunchKernelGGL(k_init_state, dim3(4096), dim3(256), 0, s, d, b, b.tau);
}

}  // namespace dcfm
