/*
 * dcfm.h — C ABI of the MI355X-native Gibbs sweep + covariance assembly for the
 * divide-and-conquer sparse latent-factor model (Sabnis & Pati, arXiv 1612.02875).
 *
 * Drop-in boundary.  The reference has no plugin or operator
 * API: its only interface is the MATLAB function
 *     Sigmaout = divideconquer(Y,g,k,BURNIN,MCMC,thin,rho)      (divideconquer.m:1)
 * and the boundary sits INSIDE it, between the driver (dc:29-87: zero-column
 * removal, partition, standardisation, hyper-parameters, initial draws) and the
 * iteration loop (dc:90-197).  These entry points take over exactly the loop's
 * read/write set; a MEX gateway or the Python host twin
 * (package ``dcfm_amd``, ctypes) calls them.
 *
 * Conventions
 *  - Plain C, no exceptions cross the ABI.  Every int-returning call returns
 *    DCFM_OK (0) or a DCFM_ERR_* code; dcfm_last_error() gives the message.
 *  - Host arrays are MATLAB column-major with the reference's shapes (so a MEX
 *    gateway passes mxGetPr/mxGetDoubles pointers straight through).  The
 *    caller owns every host buffer; the library copies and never keeps a
 *    caller pointer.
 *  - "local" arrays cover the shards this rank owns: global shards
 *    [shard0, shard0 + g_local) with g_local = g / nranks, shard0 = rank*g_local.
 *  - A handle is not thread-safe.  One process (one host thread) per GPU.
 *  - dcfm_run is asynchronous w.r.t. the host (work is queued on the handle's
 *    HIP stream); dcfm_get_*, dcfm_synchronize block.
 */
#ifndef DCFM_H
#define DCFM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCFM_ABI_VERSION 2

/* status codes */
#define DCFM_OK              0
#define DCFM_ERR_INVALID     1   /* bad argument / shape / call order            */
#define DCFM_ERR_UNSUPPORTED 2   /* valid for the reference, not yet built here  */
#define DCFM_ERR_HIP         3   /* HIP runtime error (incl. no device)          */
#define DCFM_ERR_RCCL        4   /* RCCL error                                   */
#define DCFM_ERR_NUMERIC     5   /* non-finite state detected                    */
#define DCFM_ERR_ALLOC       6   /* device or host allocation failed             */

/* dcfm_config.flags */
#define DCFM_FLAG_INJECT_DRAWS 0x1u  /* read standard variates from dcfm_set_draws
                                        buffers instead of on-device Philox        */
#define DCFM_FLAG_UNFUSED      0x2u  /* K <= 32 through the per-kernel side-stream layout
                                        (k_prep / k_xchol on a second stream, k_draws
                                        batches) instead of the fused launch chain;
                                        same results (tests, diagnostics)           */
#define DCFM_FLAG_ONE_STREAM   0x4u  /* every launch on one stream (isolated timings) */
#define DCFM_FLAG_FLAT_PRIORITY 0x8u /* default priority for every stream          */
#define DCFM_FLAG_COMM_SELF    0x20u  /* one rank through the collective data path with a
                                        real one-rank RCCL communicator (dcfm_comm_init):
                                        exercises the RCCL calls on a one-GPU box; same
                                        results as the plain one-rank chain (tests)        */
#define DCFM_FLAG_EXACT_RESIDUAL 0x10u /* ps / omega (dc:169-171) from the direct residual
                                        sum((Yd - eta*Lambda').^2), one extra pass over Y
                                        (k_resid), instead of the SS identity inside the
                                        loading-row kernel (parity runs)   */
#define DCFM_FLAG_GUARD_ALL    0x40u  /* the SS-identity guard rejects every row: the default
                                        path's own residual fallback (K <= 32: resid_rows8 in
                                        the loading-row kernel; K > 32: every tile through
                                        k_resid_flagged) for every row (tests)            */

typedef struct dcfm_handle dcfm_handle;

/* Replaces the scalars the loop reads: dc:41 (P, K), dc:45 (N, effsamp),
 * dc:62-65 (hyper-parameters), plus build-side placement and RNG settings. */
typedef struct {
    int32_t n;          /* observations (rows of Y), dc:30                       */
    int32_t P;          /* variables per shard, P = p/g, dc:41                   */
    int32_t g;          /* total number of shards (groups), dc:1                 */
    int32_t K;          /* factors per shard, K = k/g, dc:41                     */
    double  rho;        /* correlation of the shared factor, dc:1                */
    int64_t burnin;     /* BURNIN, dc:1                                          */
    int64_t mcmc;       /* MCMC, dc:1;  effsamp = mcmc/thin (dc:45, quirk Q8)    */
    int64_t thin;       /* thin, dc:1                                            */
    double  as_, bs, df, ad1, bd1, ad2, bd2;  /* dc:62-65 (1,0.3,3,2,1,2,1)      */
    uint64_t seed;      /* Philox key (counter-based RNG; ignored with INJECT)   */
    int32_t nranks;     /* ranks sharing the chain (1 = single GPU)              */
    int32_t rank;       /* this rank                                             */
    int32_t device;     /* HIP device ordinal this handle runs on                */
    uint32_t flags;     /* DCFM_FLAG_*                                           */
    int32_t asm_batch;  /* saved samples per covariance-assembly flush (0 = 32)  */
    int32_t reserved[7];
} dcfm_config;

/* Sampler state (dc:69-87, updated by dc:90-177).  All column-major.
 * NULL members are skipped by get, and are an error for set unless noted. */
typedef struct {
    double *Lambda;  /* P x K x g_local   loadings                  (dc:70,144) */
    double *ps;      /* P x 1 x g_local   residual precisions       (dc:69,170) */
    double *omega;   /* P x g_local       diag(Omega) (Q1: = ps at init,
                                          = 1./ps after dc:171)                 */
    double *psi;     /* P x K x g_local   psijh                     (dc:73,150) */
    double *Plam;    /* P x K x g_local   loading precisions        (dc:77,176) */
    double *X;       /* n x K             shared factor, replicated (dc:71,128) */
    double *Z;       /* n x K x g_local   shard factors             (dc:71,106) */
    double *eta;     /* n x K x g_local   get only; set ignores it (Q12)        */
    double *delta;   /* K x 1 x g         ALL shards (replicated)   (dc:74,163) */
    double *tauh;    /* K x 1 x g         ALL shards (replicated)   (dc:76,163) */
} dcfm_state_view;

/* Injected standard variates, ALL shards, column-major,
 * one trailing iteration dimension of length n_iter:
 *   NZ K x n x g x T (dc:104)   NX K x n x T (dc:126)   NL K x P x g x T (dc:142)
 *   Gpsi P x K x g x T  standard gamma, shape df/2+0.5       (dc:150)
 *   Gdelta K x g x T    shape ad1+P*K/2 (h=1), ad2+P*(K-h+1)/2 (dc:158,163)
 *   Gps P x g x T       shape as+n/2                           (dc:170)     */
typedef struct {
    const double *NZ, *NX, *NL, *Gpsi, *Gdelta, *Gps;
} dcfm_draws_view;

/* ---- lifecycle ---------------------------------------------------------- */
int  dcfm_create(const dcfm_config *cfg, dcfm_handle **out);
void dcfm_destroy(dcfm_handle *h);
const char *dcfm_last_error(const dcfm_handle *h);   /* h may be NULL */
int  dcfm_abi_version(void);

/* ---- multi-rank: RCCL communicator over xGMI ----------------------------
 * Rank 0 calls dcfm_comm_unique_id, the host broadcasts the 128 bytes
 * (torch.distributed / MPI / files — any side channel), every rank calls
 * dcfm_comm_init.  Not needed when nranks == 1. */
int  dcfm_comm_unique_id(uint8_t out[128]);
int  dcfm_comm_init(dcfm_handle *h, const uint8_t id[128]);
/* Test communicator: the n handles (nranks = n, ranks 0..n-1, one device) exchange
 * through device copies inside this process instead of RCCL, each handle driven by
 * its own host thread — the multi-rank sweep on a single GPU.  Same collective
 * semantics and call order as dcfm_comm_init. */
int  dcfm_comm_init_loopback(dcfm_handle *const *handles, int32_t n);

/* ---- inputs -------------------------------------------------------------- */
/* Yd(:,:,shard0+1 : shard0+g_local) after dc:48-59, n x P x g_local.        */
int  dcfm_set_data(dcfm_handle *h, const double *Yd_local);
/* On-device ingest (replaces the host's dc:48-59): Y is the raw
 * n x p_in matrix (column-major, after the caller's zero-column removal, dc:31-39, or
 * before it — cols index Y's own columns); cols[m*P + j] (0-based) is the input column
 * of local shard m, position j, i.e. keep(varind((shard0+m)*P + j)) - 1 in MATLAB terms.
 * Y goes to HBM once; the kernel gathers, centres, scales by 1./sqrt(var) (n - 1) and
 * lays Yd out for the sweep.  sd_out (nullable): P x g_local sample standard deviations
 * (for unpermute_sigma); dev_ms (nullable): the kernel's device time.  A constant
 * column (zero variance, Q13) is DCFM_ERR_INVALID; needs n >= 2. */
int  dcfm_set_data_raw(dcfm_handle *h, const double *Y, int64_t p_in, const int64_t *cols,
                       double *sd_out, double *dev_ms);
/* Yd as the sweep holds it, n x P x g_local column-major (the layout of dcfm_set_data). */
int  dcfm_get_data(dcfm_handle *h, double *Yd_local);
/* dc:31-34 on the device: nnz_out[j] = nnz(Y(:,j)) for the n x p column-major Y (NaN
 * counts as non-zero).  No handle: the kept width p (hence P = p/g) is not known yet. */
int  dcfm_count_nonzero_columns(int device, const double *Y, int32_t n, int64_t p, int32_t *nnz_out,
                                double *dev_ms);
int  dcfm_set_state(dcfm_handle *h, const dcfm_state_view *s);
/* Initial state on the device (dc:68-87), instead of dcfm_set_state:
 * ps = Ga(as)/bs, omega = ps (Q1), X, Z ~ N(0,1), psijh = (2/df) Ga(df/2), delta(1) =
 * bd1 Ga(ad1), delta(2:K) = bd2 Ga(ad2), tauh = cumprod, Plam = psijh .* tauh', Lambda = 0,
 * from the handle's Philox key at iteration-0 counters (sites 7-12; variate e of a shard
 * = MATLAB linear index e inside that shard's array, counter row e/32, index e%32 — as
 * dcfm_rng_fill, which reproduces them).  Identical on any number of ranks. */
int  dcfm_init_state(dcfm_handle *h);
/* Draws for iterations first_iter .. first_iter+n_iter-1 (1-based, as iter). */
int  dcfm_set_draws(dcfm_handle *h, const dcfm_draws_view *d, int64_t first_iter, int64_t n_iter);

/* ---- the hot loop (dc:90-197) ------------------------------------------- */
/* Runs iterations first_iter .. first_iter+n_iter-1 (1-based).  Saved
 * iterations (mod(iter,thin)==0 && iter>burnin, dc:180) feed the covariance
 * assembly (dc:182-195); pending saved samples are flushed before return.   */
int  dcfm_run(dcfm_handle *h, int64_t first_iter, int64_t n_iter);
int  dcfm_synchronize(dcfm_handle *h);

/* ---- outputs ------------------------------------------------------------ */
int  dcfm_get_state(dcfm_handle *h, dcfm_state_view *out);
/* dcfm_get_state without the non-finite check: after a dcfm_run that ended in
 * DCFM_ERR_NUMERIC, the state as the device holds it (NaN / Inf included), so a
 * caller can see which stage of the failing iteration went non-finite.  The
 * handle stays in its error state until set_state / init_state. */
int  dcfm_get_state_raw(dcfm_handle *h, dcfm_state_view *out);
/* Sigmaout, p x p (p = P*g), symmetric, in the reference's permuted and
 * standardised coordinates (dc:186-195, quirk Q7).  Collective when
 * nranks > 1: every rank must call it; rank 0 receives the matrix (out may be
 * NULL on the other ranks and is not written there).  Sigmaout is block-sharded
 * over the ranks (dcfm_sigma_block): the read-out moves each element once, from
 * its owner to rank 0 (RCCL send/recv), in column stripes of <= 2 GiB. */
int  dcfm_get_sigma(dcfm_handle *h, double *out);
/* Columns col0 .. col0+ncols-1 of Sigmaout: p x ncols column-major, i.e. exactly
 * out = Sigmaout(:, col0+1 : col0+ncols) — a contiguous chunk of the MATLAB array,
 * so a caller can fill a p x p result stripe by stripe (config c5: 80 GB) with
 * device scratch of only p x ncols.  Collective when nranks > 1; the stripe goes
 * to rank 0 only (as dcfm_get_sigma). */
int  dcfm_get_sigma_cols(dcfm_handle *h, int64_t col0, int64_t ncols, double *out);
/* This rank's block of Sigmaout (the build's output sharding; the reference holds
 * the whole p x p, dc:42): out[0], out[1] = the rows [row0, row1) whose lower
 * triangle it accumulates (contiguous 128-row tiles, balanced by tile count over
 * the ranks), out[2] = its device bytes for Sigmaout (~p^2 / (2 nranks) * 8). */
int  dcfm_sigma_block(const dcfm_handle *h, int64_t out[3]);
int64_t dcfm_saved_samples(const dcfm_handle *h);
/* Error of Sigmaout against a truth Sigma0 = U U' + diag(s) given in the same permuted,
 * standardised coordinates (U: p x r column-major, r <= 32; s: p), computed on the
 * device (Sigmaout never leaves HBM; c5: 80 GB).  out[0] = ||Sigmaout - Sigma0||_F,
 * out[1] = ||Sigma0||_F, out[2] = ||Sigmaout - Sigma0||_2 from `iters` Lanczos steps
 * (seeded start, full reorthogonalisation; exact when iters >= p; 0 skips it).  The
 * reference leaves this to the caller (Frobenius and
 * operator-norm error against the synthetic truth).  Collective when nranks > 1. */
int  dcfm_sigma_error(dcfm_handle *h, const double *U, int32_t r, const double *s, int32_t iters,
                      uint64_t seed, double out[3]);

/* ---- chain trace (convergence diagnostics across chains) ----
 * dcfm_set_trace(h, cap): record one row per iteration of later dcfm_run calls, up to cap
 * rows (0 = off, the default; resets the count).  Row = this rank's local-shard sums
 *   [ ||Lambda||_F^2,  sum omega (= tr Omega),  sum log ps,  sum_m sum_h log tau_h^m ]
 * after the iteration (tr of the iteration's Sigma draw = row[0] + row[1], dc:185); ranks
 * that split one chain add their rows.  dcfm_get_trace: out (nullable) gets count x 4
 * doubles, row-major. */
int  dcfm_set_trace(dcfm_handle *h, int64_t capacity);
int  dcfm_get_trace(dcfm_handle *h, double *out, int64_t *count);

/* ---- measurement --------------------------------------------------------- */
/* Per-kernel HIP-event timing on the handle's stream (off by default).
 * Kernel ids: DCFM_K_* below.  Times are accumulated device milliseconds. */
#define DCFM_K_PREP     0
#define DCFM_K_WPASS    1
#define DCFM_K_ZDRAW    2
#define DCFM_K_XRED     3
#define DCFM_K_XDRAW    4
#define DCFM_K_CPASS    5
#define DCFM_K_LAMBDA   6
#define DCFM_K_COLSUM   7
#define DCFM_K_DELTA    8
#define DCFM_K_SAVE     9
#define DCFM_K_ASSEMBLE 10
#define DCFM_K_COMM     11
#define DCFM_K_XCHOL    12
#define DCFM_K_DRAWS    13   /* on-device Philox variates of the next iteration (side stream) */
#define DCFM_K_RESID    14   /* direct-residual ps / omega (DCFM_FLAG_EXACT_RESIDUAL) */
#define DCFM_K_COUNT    15
int  dcfm_set_profiling(dcfm_handle *h, int enable);
/* Time only the kernels whose bit (1u << DCFM_K_*) is set: two events per timed
 * launch cost host time, so a throughput run times just the kernel it reports. */
int  dcfm_set_profiling_mask(dcfm_handle *h, uint32_t mask);
/* Time one in `stride` launches of each timed kernel (the first of every `stride`; default 1),
 * e.g. to keep event records off most launches of a long run.  Reset to 1 by
 * dcfm_set_profiling[_mask]. */
int  dcfm_set_profiling_stride(dcfm_handle *h, int32_t stride);
int  dcfm_get_kernel_stats(dcfm_handle *h, double ms[DCFM_K_COUNT], int64_t launches[DCFM_K_COUNT]);
const char *dcfm_kernel_name(int id);

/* ---- diagnostics (RNG statistical tests) --------------------------------
 * Fills out[0..count) with on-device Philox variates exactly as the sweep
 * draws them: kind 0 = standard normal, kind 1 = standard gamma(shape).
 * Variate i uses counter (site, shard, row = i / 32, k = i % 32, iter). */
int  dcfm_rng_fill(int device, uint64_t seed, int kind, double shape, int32_t site,
                   int32_t shard, int64_t iter, int64_t count, double *out);
/* As dcfm_rng_fill with rows of `width` variates: out[e], e < count <= rows * width, uses
 * counter (site, shard, row = e / width, k = e % width, iter) — e.g. width = K for the
 * per-row variates of the K > 32 kernels (row j's normals / gammas at indices 0..K-1). */
int  dcfm_rng_fill_rows(int device, uint64_t seed, int kind, double shape, int32_t site,
                        int32_t shard, int64_t iter, int64_t rows, int32_t width, int64_t count,
                        double *out);

#ifdef __cplusplus
}
#endif
#endif /* DCFM_H */
