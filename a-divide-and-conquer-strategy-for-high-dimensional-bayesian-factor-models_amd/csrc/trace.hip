// Per-iteration chain trace for convergence diagnostics across chains.
//
// The reference keeps no trace (it only accumulates Sigmaout, dc:180-196); to compare the
// c4 configuration's parallel chains (split-R-hat, effective sample size) each chain needs
// a few scalar summaries of its state per iteration.  After an iteration has finished
// (dc:137-177 done), k_trace_part reduces this rank's local shards:
//   q0 = sum_m sum_{j,h} Lambda_jh^2          ||Lambda||_F^2  (= tr(Lambda Lambda'))
//   q1 = sum_m sum_j omega_j                  tr(Omega)  -> q0 + q1 = tr(Sigma draw, dc:185)
//   q2 = sum_m sum_j log ps_j                 residual precisions (dc:170)
//   q3 = sum_m sum_h log tau_h^m              the shrinkage process (dc:163)
// TRACE_SLICES blocks per local shard, each a fixed slice of the shard's loading rows (fixed
// in-order sums: deterministic), publishing partials [G][TRACE_SLICES][4] into a scratch; the last
// slice block of a shard to finish (a per-shard ticket) adds the shard's partials in slice order into
// the iteration's trace row [G][4], so the stored trace holds 4 doubles per shard and iteration
// (round 6: the [cap][G][TRACE_SLICES][4] partials were 164 MB at c3's 5,000-iteration trace);
// dcfm_get_trace adds the shards in shard order on the host.  (A second, one-block summing launch
// cost 7.6 us per iteration on the chain; one block per shard, 159 us at c4: a latency-bound walk
// over the shard's 1.3 MB of Lambda.)  Ranks that split one chain's shards add their rows (the
// host all-reduces).  Cost when enabled: one read of Lambda (G x PP x KW doubles; 5 MB at c3), off
// by default.
#include "dcfm_internal.h"
#include "linalg.h"

namespace dcfm {

__global__ __launch_bounds__(256) void k_trace_part(const double *__restrict__ Lam, const double *__restrict__ omega,
                                                    const double *__restrict__ ps, const double *__restrict__ tau,
                                                    int P, int PP, int KW, int K, int shard0,
                                                    double *__restrict__ part, unsigned *__restrict__ ticket,
                                                    double *__restrict__ row) {
    __shared__ double red[4][256];
    const int sl = blockIdx.x, m = blockIdx.y, t = threadIdx.x;
    const int j0 = (int)((long long)P * sl / TRACE_SLICES), j1 = (int)((long long)P * (sl + 1) / TRACE_SLICES);
    const double *L = Lam + (size_t)m * PP * KW;
    double q0 = 0.0, q1 = 0.0, q2 = 0.0, q3 = 0.0;
    // rows [j0, j1) (padding columns k >= K hold zeros)
    for (int e = j0 * KW + t; e < j1 * KW; e += 256) { const double v = L[e]; q0 += v * v; }
    for (int j = j0 + t; j < j1; j += 256) {
        q1 += omega[(size_t)m * PP + j];
        q2 += log(ps[(size_t)m * PP + j]);
    }
    if (sl == 0)
        for (int hh = t; hh < K; hh += 256) q3 += log(tau[(size_t)(shard0 + m) * KW + hh]);
    red[0][t] = q0; red[1][t] = q1; red[2][t] = q2; red[3][t] = q3;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (t < s) {
#pragma unroll
            for (int q = 0; q < 4; ++q) red[q][t] += red[q][t + s];
        }
        __syncthreads();
    }
    if (t < 4) st_agent(part + ((size_t)m * TRACE_SLICES + sl) * 4 + t, red[t][0]);
    // the shard's last slice block folds the slices (agent-scope hand-off, kernels.hip signal_count)
    __shared__ unsigned last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        last = __hip_atomic_fetch_add(ticket + m, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == TRACE_SLICES - 1;
        if (last) __hip_atomic_store(ticket + m, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next iteration
    }
    __syncthreads();
    if (!last || t >= 4) return;
    double acc = 0.0;
    for (int k = 0; k < TRACE_SLICES; ++k) acc += ld_agent(part + ((size_t)m * TRACE_SLICES + k) * 4 + t);
    row[(size_t)m * 4 + t] = acc;
}

void launch_trace(const Dims &d, const Bufs &b, const double *tau_cur, double *scratch, double *row, hipStream_t s) {
    unsigned *ticket = reinterpret_cast<unsigned *>(scratch + trace_scratch_doubles(d.G) - (d.G + 1) / 2);
    hipLaunchKernelGGL(k_trace_part, dim3(TRACE_SLICES, d.G), dim3(256), 0, s, b.Lam, b.omega, b.ps, tau_cur, d.P, d.PP, d.kp,
                       d.K, d.shard0, scratch, ticket, row);
}

}  // namespace dcfm
