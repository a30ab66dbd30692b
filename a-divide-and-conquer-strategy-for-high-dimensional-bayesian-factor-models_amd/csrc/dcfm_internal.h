// Internal layout + kernel launch declarations for libdcfm (MI355X / gfx950).
//
// HBM layout (C order, last index fastest), G = local shards, mg = global shard,
// KW = d.kp = the padded factor width (32 for K <= 32, 64 for K <= 64, 128 for K <= 128):
//   Y      [G][NP][PP]   standardised data, rows i padded to NP (x16), cols j to PP (x16), zeros
//   yy     [G][PP]       sum_i Y_ij^2 (set_data)                -> residual SS identity
//   Lam    [G][PP][KW]   loadings, k padded to KW with zeros
//   omega  [G][PP]       diag(Omega);   ps [G][PP]
//   psi    [G][PP][KW];  Plam [G][PP][KW] (the caller's Plam; valid until the first
//                        iteration, after which Plam = psi o tau is formed on the fly)
//   X      [NP][KW]      replicated;    Z [G][NP][KW]
//   delta, tau [2][g][KW] replicated on every rank, double-buffered per iteration
//   W      [G][NP][KW]   W_m = Y_m (omega o Lambda_m)  (k_wpass; the fused K <= 32 chain keeps it in
//                        registers: k_wcol draws Z from the W-pass accumulators)
//   A      [G][KW][KW]   A_m = Lambda_m' diag(omega) Lambda_m             (k_prep)
//   ZM     [G][4][KW][KW] Z-draw operators {M1, M2, U, NA} of shard m         (k_prep)
//   Sp     [G][NP][KW]   per-shard X message W_m - sqrt(1-rho) A_m Z_m'   (k_zdraw / k_wcol)
//   xin    [NP][KW]      local sum over shards of Sp;  xall [nranks][NP][KW] all-gathered (== xin if 1 rank;
//                        inside the packed message with the fused several-rank chain, Dims::xstride apart)
//   xa, xa_all [nranks][KW][KW]  per-rank sum of A_m (gathered);  XM [2][KW][KW] X-draw operators {Tx, Ux} (k_xchol)
//   C      [G][PP][KW]   C_m = Y_m' eta_m  (k_cpass);  E [G][KW][KW] = eta_m' eta_m
//   cpart  [G][PP][KW]   psi o Lambda^2 per loading row (k_lambda), summed over rows by k_colsum
//   sloc   [G][KW], sall [g][KW]  column sums (all-gathered)
//   Lb     [2][p][LDB]   saved Lambda rows of an assembly batch (double-buffered), sample s at cols s*K..
//   wsum   [2][p]        sum of saved omega of the batch
//   Sigma  [ntiles][128][128]  this rank's block of the lower triangle of Sigmaout, tile-packed:
//                        rank r owns the contiguous tile rows [T0, T1) (balanced by tile count,
//                        sigma_split), tile (ti, tj), tj <= ti, at index tri(ti) - tri(T0) + tj,
//                        inside in k_assemble's accumulator order (sig_tile_off: each lane's two
//                        values of a 16x16 MFMA tile adjacent, so a wave moves the tile with 16-byte
//                        accesses); ~p^2 / (2 nranks) doubles per rank
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcfm {

constexpr int KP = 32;         // padded factor width of the narrow (K <= 32) kernels
constexpr int KP_MAX = 128;    // widest supported padding (K <= 128, config c4 has K = 100)
constexpr int ASM_TILE = 128;  // covariance-assembly output tile
// Wide paths (KW >= 64) keep E_m = eta_m' eta_m in the loading-row kernel's layout: the
// upper 16x16 tiles (Kc <= I) of the KW/16 x KW/16 tile grid, tile t = etile(KW/16, Kc, I) in
// the fp64 MFMA C/D layout, pair g2 = g / 2 of lane l = c + 16 q at (2t + g2) 128 + 2l + (g & 1)
// for element (16 Kc + q + 4g, 16 I + c) -- one contiguous 16-byte read per lane and pair.
__host__ __device__ constexpr int etile(int nbw, int Kc, int I) { return Kc * nbw - Kc * (Kc - 1) / 2 + (I - Kc); }
__host__ __device__ constexpr int etile_index(int nbw, int R, int Cc) {
    return (2 * etile(nbw, R >> 4, Cc >> 4) + ((R & 15) >> 3)) * 128 + 2 * ((Cc & 15) + 16 * (R & 3)) +
           (((R & 15) >> 2) & 1);
}
constexpr int ASM_KC = 16;            // k_assemble's k chunk (kext, LDB are multiples)

struct Dims {
    int n, P, g, K, G;          // G = local shards
    int NP, PP;                 // padded rows / cols
    int shard0;                 // first global shard of this rank
    int nranks, rank;
    int coll;                   // the collective (multi-rank) data path: nranks > 1, or one rank with
                                // a real RCCL communicator (DCFM_FLAG_COMM_SELF)
    int p;                      // P * g
    int kp;                     // padded factor width KW of every [..][KW] array: 32, 64 or 128
    double rho, sr, s1r;        // rho, sqrt(rho), sqrt(1-rho)
    double as_, bs, df, ad1, bd1, ad2, bd2;
    uint64_t seed;
    int inject;
    // gathered-message layout of the fused several-rank chain: the per-rank message is
    // [sloc G x KP | sum_m A_m KP x KP | X message NP x KP] (ONE all-gather per iteration), so
    // rank r's column sums sit at r * xstride, its A sum at that + G*KP and its X message at
    // that + G*KP + KP*KP.  sgap = KP*KP + NP*KP and xstride = G*KP + KP*KP + NP*KP there;
    // sgap = 0, xstride = KW*KW for separate gathers.
    int sgap, xstride;
};

// injected draws on device, [T][...] with T = n_iter of dcfm_set_draws
struct DrawsDev {
    const double *NZ, *NX, *NL, *Gpsi, *Gdelta, *Gps;  // full-g arrays
    int64_t first_iter, n_iter;
};

// loading-row variates of one iteration in k_lambda's layout (local shard m, loading row j):
// NL [G][P][K] (dc:142 zlam), Gpsi [G][P][K] (dc:150), Gps [G][P] (dc:170)
struct LamDraws { const double *NL, *Gpsi, *Gps; };
// k_wcol's extra blocks generate them for the generated fused chain (K <= 32): one index
// space — [0, n_ps) ps gammas, [n_ps, n_psi) psi gammas, [n_psi, n_all) normal pairs — walked
// grid-stride by b_total blocks of LAM_GEN_THREADS behind the W tiles (VALU work in the slots
// and issue cycles the streaming W pass leaves free)
#ifndef DCFM_LAM_GEN_BLOCKS
#define DCFM_LAM_GEN_BLOCKS 160
#endif
constexpr int LAM_GEN_THREADS = 256, LAM_GEN_BLOCKS = DCFM_LAM_GEN_BLOCKS;
struct LamGen { double *NL, *Gpsi, *Gps; int n_ps, n_psi, n_all, b_total; };
inline int lam_gen_doubles(const Dims &d) { return 2 * d.G * d.P * d.K + d.G * d.P; }
inline LamGen lam_gen_plan(const Dims &d, double *base) {
    const int T = LAM_GEN_THREADS, GP = d.G * d.P;
    LamGen g;
    g.NL = base;
    g.Gpsi = base + (size_t)GP * d.K;
    g.Gps = base + 2 * (size_t)GP * d.K;
    g.n_ps = GP;
    g.n_psi = GP + GP * d.K;
    g.n_all = g.n_psi + GP * ((d.K + 1) / 2);
    const int full = (g.n_all + T - 1) / T;
    g.b_total = full < LAM_GEN_BLOCKS ? full : LAM_GEN_BLOCKS;
    return g;
}

struct Bufs {
    double *Y, *yy, *Lam, *omega, *ps, *psi, *Plam, *X, *Z, *delta, *tau;
    double *ldraw;                     // LamDraws of the generated fused chain (lam_gen_plan), else null
    double *W, *A, *ZM, *Sp, *xin, *xall, *C, *E, *cpart, *sloc, *sall;
    double *Lb[2], *wsum[2], *Sigma;
    double *xa, *xa_all, *XM;          // per-rank sum of A, gathered sums, X-draw operators
    double *xpart;                     // k_wcol chunk sums of A (xsum_blocks(G) x KP x KP)
    unsigned *ticket;                  // k_wcol last-arrival ticket (0 between launches)
    unsigned long long *sync;          // hand-off counters (monotonic): [0] = k_xdraw XM out (several ranks),
                                       // [2 + chunk] = k_wcol A_m of the chunk out,
                                       // [SYNC_ZM + m] = k_wcol Z operators of shard m out
    double *msg_all;                   // packed gather target (fused, nranks > 1), else null
    double *agree;                     // 3 doubles: the failure counts of a collective call (dcfm.hip agree)
    int *rflag;                        // K > 32: [G][PP / 32] 32-row tiles whose SS identity the guard of
                                       // k_lambda_w rejected (k_resid_flagged redoes them and clears the flag)
    int2 *tiles;
    int ntiles, LDB;
    int T0, T1;                        // owned tile rows of Sigma (block-sharded, see above)
};

// k_wcol shard sum of A
constexpr int XSUM_BLOCKS = 8;
constexpr int TRACE_SLICES = 16;       // k_trace_part blocks per local shard (slices of its loading rows)
// Bufs::sync: [0] the X operators (k_xdraw, several ranks), [1] spare, [2, 2 + 256) chunk counters of the A sum, [SYNC_ZM, SYNC_ZM + G) the
// per-shard Z-operator counters (the fused W pass draws Z once its shard's operators are out)
constexpr int SYNC_ZM = 2 + 256;
// blocks of the A sum: G / chunk, chunk = a power of two dividing G, grown while more than
// XSUM_BLOCKS chunks remain — so each chunk is a subtree of the canonical tree (TreeSum) and
// the tree over the chunk sums is T(0, G).  G <= XSUM_BLOCKS: one block sums every shard
// (tree8 with zero padding is T(0, G)), without the chunk-sum hand-off round
__host__ __device__ inline int xsum_blocks(int G) {
    if (G <= XSUM_BLOCKS) return 1;
    int chunk = 1;
    while (G / chunk > XSUM_BLOCKS && (G / chunk) % 2 == 0) chunk *= 2;
    return G / chunk;
}

// Sigma block-sharding helpers (host + device)
__host__ __device__ inline long long tri(long long t) { return t * (t + 1) / 2; }
// offset of the stored element (a, b), a >= b, in a rank's tile-packed Sigma (owner of tile row a/128)
// Inside a tile, element (ra, cb) sits where k_assemble's wave w = 2 (ra / 64) + cb / 64 holds it
// in the f64 MFMA C/D layout: 16x16 tile (u, v) = ((ra / 16) % 4, (cb / 16) % 4), row ra % 16 =
// q + 4 g, lane q * 16 + cb % 16; the lane's values g = 2 h, 2 h + 1 are adjacent, so a wave moves
// one (u, v, h) slice as one 16-byte access per lane, 1 KiB contiguous
__host__ __device__ inline int sig_tile_off(int u, int v, int g, int w, int lane) {
    return ((((w * 4 + u) * 4 + v) * 2 + (g >> 1)) * 64 + lane) * 2 + (g & 1);
}
__host__ __device__ inline size_t sig_off(int a, int b, int T0) {
    const int ta = a / ASM_TILE, tb = b / ASM_TILE, ra = a % ASM_TILE, cb = b % ASM_TILE, rr = ra & 15;
    return (size_t)(tri(ta) - tri(T0) + tb) * ASM_TILE * ASM_TILE +
           sig_tile_off((ra >> 4) & 3, (cb >> 4) & 3, rr >> 2, 2 * (ra >> 6) + (cb >> 6), (rr & 3) * 16 + (cb & 15));
}
// Packed window of a rank owning rows [R0, R1) in a column stripe: column c holds the rows
// [lo(c), R1) of Sigmaout(:, c) it owns (lo = 0 for c in [R0, R1): the upper part mirrored from
// its own rows; lo = R0 for c < R0; nothing for c >= R1).  off(c) = start of column c in the
// rank's packed stripe [c0, ...).
__host__ __device__ inline long long win_lo(long long c, long long R0, long long R1) {
    return (c >= R0 && c < R1) ? 0 : (c < R0 ? R0 : R1);
}
__host__ __device__ inline long long win_off(long long c, long long c0, long long R0, long long R1) {
    const long long na = (c < R0 ? c : R0) - c0;                 // columns of [c0, c) below R0
    const long long b0 = c0 > R0 ? c0 : R0, b1 = c < R1 ? c : R1;  // columns of [c0, c) in [R0, R1)
    return (na > 0 ? na : 0) * (R1 - R0) + (b1 > b0 ? b1 - b0 : 0) * R1;
}

// launchers (kernels.hip)
void launch_prep(const Dims &d, const Bufs &b, hipStream_t s);
void launch_wpass(const Dims &d, const Bufs &b, hipStream_t s);
void launch_zdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s);
void launch_xred(const Dims &d, const Bufs &b, hipStream_t s);
// fused K <= 32 launches (kernels.hip: k_wcol, k_xdraw roles)
// K <= 32: the Z operators + shard sum of A (ops), the previous iteration's column sums
// (colsum) and the Y pass W with the Z draw of its rows (wpass: Z, Sp; needs ops) in one launch
// (k_wcol); one rank also factors Xprec
void launch_wcol(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, bool ops, bool colsum, bool wpass,
                 unsigned long long ops_epoch, hipStream_t s, bool lamgen = false);
// several ranks, K <= 32: k_xdraw with the X operators (block 0, from the ranks' A sums of the
// packed gather, published through the counter b.sync[0] at xm_epoch) and the row blocks
// summing the ranks' X messages
void launch_xdraw_mr(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, unsigned long long xm_epoch,
                     hipStream_t s);
void launch_asum(const Dims &d, const Bufs &b, hipStream_t s);
void launch_xchol(const Dims &d, const Bufs &b, hipStream_t s);
void launch_xdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s,
                  bool from_shards = false);
// k_cpass; with delta_in (fused K <= 32 chain) also the delta / tau chain of delta_iter in
// extra blocks (column sums from b.sall)
void launch_cpass(const Dims &d, const Bufs &b, hipStream_t s, const DrawsDev &dr = DrawsDev{},
                  const double *delta_in = nullptr, const double *tau_in = nullptr, double *delta_out = nullptr,
                  double *tau_out = nullptr, int64_t delta_iter = 0);
// gen: K <= 32 reads the variates k_wcol generated into b.ldraw (the generated fused chain)
// instead of the draw buffers dr (injected draws, k_draws batches).
// K <= 32: a wave whose SS identity may be off by more than ~kappa_max eps for one of its rows (lambda.h
// guard) takes its rows' ps, omega from dc:169's direct residual instead (resid_rows8, same launch)
#ifndef DCFM_KAPPA_MAX
#define DCFM_KAPPA_MAX 1e3
#endif
constexpr double KAPPA_IDENTITY_MAX = DCFM_KAPPA_MAX;
void launch_lambda(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter,
                   const double *tau_cur, const double *plam_src, hipStream_t s, bool gen = false,
                   double kappa_max = KAPPA_IDENTITY_MAX);
void launch_colsum(const Dims &d, const Bufs &b, hipStream_t s);
// resid.hip (DCFM_FLAG_EXACT_RESIDUAL): ps, omega from the direct residual Yd - eta Lambda' (dc:169-171)
// for every loading row, after the loading-row kernel, with its ps variates (gen: b.ldraw, else dr)
void launch_resid(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s, bool gen);
// K > 32, default mode: the same for the 32-row tiles k_lambda_w's guard flagged (b.rflag); the other
// blocks exit at once
void launch_resid_flagged(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s);
void launch_delta(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter,
                  const double *delta_in, const double *tau_in, double *delta_out,
                  double *tau_out, hipStream_t s);
void launch_save(const Dims &d, const Bufs &b, double *Lb, double *wsum, int slot, hipStream_t s);
void launch_assemble(const Dims &d, const Bufs &b, const double *Lb, const double *wsum, int kext,
                     double inv_eff, hipStream_t s);
// column stripe [c0, c0 + nc) of Sigmaout from a rank's tile-packed block (tile rows [T0, T1)):
// the rank's packed windows (win_lo / win_off; with one rank = the dense p x nc stripe)
void launch_sigma_pack(const double *S, int p, int T0, int T1, int c0, int nc, double *out, hipStream_t s);
// root of the gather: the dense p x nc stripe from every rank's packed windows, rank k's at
// recv + base[k]; Tb[0..nranks] are the ranks' tile-row boundaries (device arrays)
void launch_sigma_unpack(const double *recv, int p, int c0, int nc, const int *Tb, const long long *base,
                         int nranks, double *out, hipStream_t s);
void launch_eta(const Dims &d, const Bufs &b, double *eta_out, hipStream_t s);
// sigma_err.hip: rows' sums of (Sigmaout - U U' - diag s) v, squares and truth squares
// (partials [splits][p] in y / fro / tru; summed into out[0..p), out[p..2p), out[2p..3p))
int sigma_err_splits(int p);
void launch_sigma_err(const double *S, int p, const double *U, int R, const double *sdiag, const double *v,
                      int T0, int T1, bool first, double *y, double *fro, double *tru, double *out,
                      hipStream_t s);
// ingest.hip: dc:31-34 column nnz counts; dc:50-59 partition + standardise into Y / yy
void launch_nnz_cols(const double *Y, int n, long long p, int *nnz, hipStream_t s);
void launch_stdize(const Dims &d, const double *Yraw, const long long *cols, double *Y, double *yy, double *sd,
                   int *bad, double *mean_inv, hipStream_t s);
// trace.hip: per-iteration chain summaries (||Lambda||_F^2, tr Omega, sum log ps, sum log tau) into
// row [G][4]; scratch = trace_scratch_doubles(G) zeroed doubles (slice partials + per-shard tickets)
inline size_t trace_scratch_doubles(int G) { return (size_t)G * TRACE_SLICES * 4 + (G + 1) / 2; }
void launch_trace(const Dims &d, const Bufs &b, const double *tau_cur, double *scratch, double *row, hipStream_t s);
// init.hip: dc:68-87 initial state from Philox (iteration-0 counters), delta/tau buffer 0
void launch_init_state(const Dims &d, const Bufs &b, hipStream_t s);
void launch_draws(const Dims &d, const DrawsDev &dr, int64_t iter, hipStream_t s);
// NaN / Inf sentinel over the state (sets *flag = 1 if any value is non-finite)
void launch_finite(const Dims &d, const Bufs &b, const double *tau_cur, int *flag, hipStream_t s);
// dst[i] = sum_k src[k * count + i] in slice order (loopback all-reduce)
void launch_sum_slices(const double *src, int ns, size_t count, double *dst, hipStream_t s);
void launch_rng_fill(uint64_t seed, int kind, double shape, int site, int shard, int64_t iter,
                     int64_t count, int width, double *out, hipStream_t s);

// wide-factor kernels (kp = 64 / 128; kernels_wide.hip), dispatched from the launchers above
namespace wide {
void launch_prep(const Dims &d, const Bufs &b, hipStream_t s);
void launch_xchol(const Dims &d, const Bufs &b, hipStream_t s);
void launch_zdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s);
void launch_xdraw(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, hipStream_t s);
void launch_lambda(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, const double *tau_cur,
                   const double *plam_src, hipStream_t s, double kappa_max);
void launch_delta(const Dims &d, const Bufs &b, const DrawsDev &dr, int64_t iter, const double *delta_in,
                  const double *tau_in, double *delta_out, double *tau_out, hipStream_t s);
}  // namespace wide

}  // namespace dcfm
