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

// K > 32 default mode: only the 32-row tiles whose guard k_lambda_w tripped (b.rflag); the flag is
// read by every thread before resid_tile's barrier and cleared by thread 0 after it
template <int KW>
__global__ __launch_bounds__(256) void k_resid_flagged(Dims d, const double *__restrict__ Y, const double *__restrict__ X,
                                                       const double *__restrict__ Z, const double *__restrict__ Lam,
                                                       const double *__restrict__ Gps, double *__restrict__ ps,
                                                       double *__restrict__ omega, int *__restrict__ rflag) {
    __shared__ double red[4][32];
    int *f = rflag + blockIdx.y * (d.PP / 32) + blockIdx.x;
    if (*f == 0) return;
    resid_tile<KW>(d, Y, X, Z, Lam, Gps, ps, omega, blockIdx.y, blockIdx.x * 32, red);
    if (threadIdx.x == 0) *f = 0;
}

void launch_resid_flagged(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s) {
    const double *Gps = dr.Gps + ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
    const dim3 grid(d.PP / 32, d.G);
    switch (d.kp) {
    case 64: hipLaunchKernelGGL(k_resid_flagged<64>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega, b.rflag); break;
    default: hipLaunchKernelGGL(k_resid_flagged<128>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega, b.rflag); break;
    }
}

void launch_resid(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s, bool gen) {
    const double *Gps;
    if (gen) Gps = lam_gen_plan(d, b.ldraw).Gps;   // the generated fused chain: k_wcol's buffer
    else Gps = dr.Gps + ((size_t)(iter - dr.first_iter) * d.g + d.shard0) * d.P;
    const dim3 grid(d.PP / 32, d.G);
    switch (d.kp) {
    case 32: hipLaunchKernelGGL(k_resid<32>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    case 64: hipLaunchKernelGGL(k_resid<64>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    default: hipLaunchKernelGGL(k_resid<128>, grid, dim3(256), 0, s, d, b.Y, b.X, b.Z, b.Lam, Gps, b.ps, b.omega); break;
    }
}

}  // namespace dcfm
