// C-ABI implementation (include/dcfm.h): handle, HBM allocation, layout
// conversion between the reference's MATLAB column-major arrays and the
// device layout (dcfm_internal.h), the per-iteration launch sequence of the hot
// loop (divideconquer.m:90-197) and the RCCL exchanges over xGMI.
#include "../../include/dcfm.h"
#include "dcfm_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace dcfm;

namespace {

struct ProfRec { int kid; hipEvent_t a, b; };

// In-process loopback collectives (dcfm_comm_init_loopback): n handles on one device,
// one host thread per rank, the same all-gather / all-reduce semantics as the RCCL
// communicators — so the multi-rank sweep runs and is parity-tested on a single GPU.
// Per collective: every rank posts its send pointer and a "ready" event (barrier), copies
// every other rank's slice in on its own stream after that rank's event, posts a "done"
// event (barrier), waits for every rank's "done" (no send buffer is reused before all
// ranks read it), and a last barrier frees the posting slots for the next collective.
struct LoopGroup {
    int n;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<const double *> send;
    std::vector<hipEvent_t> ready, done;
    explicit LoopGroup(int n_) : n(n_), send(n_, nullptr), ready(n_, nullptr), done(n_, nullptr) {}
    bool barrier(std::unique_lock<std::mutex> &lk) {
        const uint64_t my = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        return cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != my; });
    }
};

}  // namespace

struct dcfm_handle {
    dcfm_config cfg{};
    Dims d{};
    Bufs b{};
    DrawsDev dr{};
    hipStream_t stream = nullptr;     // main: the sweep chain
    hipStream_t side = nullptr;       // k_prep + k_xchol, overlapping k_wpass (unfused paths)
    hipStream_t sdraw = nullptr;      // on-device Philox variates, a batch ahead of the sweep
    hipStream_t sasm = nullptr;       // covariance assembly, overlapping later iterations
    ncclComm_t comm = nullptr, comm_side = nullptr, comm_asm = nullptr;
    bool comm_ok = false;
    std::shared_ptr<LoopGroup> loop;  // loopback collectives instead of RCCL (testing)
    std::vector<int> Tb;              // Sigma tile-row boundaries of all ranks (block-sharded)
    hipEvent_t lp_ready = nullptr, lp_done = nullptr;
    hipEvent_t e_lam = nullptr, e_prep = nullptr, e_xchol = nullptr, e_batch = nullptr,
               e_free[2] = {nullptr, nullptr}, e_drawn[2] = {nullptr, nullptr}, e_used[2] = {nullptr, nullptr};
    bool fused = false;           // K <= 32 fused launch chain (else the side-stream layout), fixed at create
    bool plam_valid = false;      // b.Plam holds the caller's Plam (no iteration run since set_state)
    unsigned long long wc_ops = 0;   // k_wcol launches with the operator roles (hand-off counter epoch)
    unsigned long long xm_ops = 0;   // k_xdraw launches with the X-operator role (several ranks; its counter's epoch)
    bool asm_pending[2] = {false, false};
    int cur = 0;                  // delta/tau buffer in use
    int lb = 0;                   // Lb buffer being filled
    int B = 16;                   // saved samples per flush
    int batch = 0;                // saved samples pending in Lb[lb]
    int64_t saved = 0;
    bool have_data = false, have_state = false;
    int *nan_dev = nullptr;       // k_finite flag (device) and its pinned host mirror
    int *nan_host = nullptr;
    std::string err;
    std::vector<void *> allocs;
    double *draws_mem = nullptr;
    // on-device Philox draws (no INJECT): two slots of DB iterations, the next batch
    // generated on sdraw while the sweep consumes the current one, so the main stream
    // waits on an event once per batch.  A slot is valid for the iterations it was
    // generated for whatever the state (the stream is counter-based).
    DrawsDev gen[2] = {};
    int64_t gen_first[2] = {-1, -1}, gen_n[2] = {0, 0};
    bool used_pending[2] = {false, false};   // e_used[slot] recorded after the slot's last consumer
    int DB = 1;                              // iterations per draws batch
    size_t draw_iter_sz[6] = {};             // per-iteration doubles of NZ, NX, NL, Gpsi, Gdelta, Gps
    // per-iteration chain trace (dcfm_set_trace): [scratch | rows [trace_cap][G][4]] (trace.hip)
    double *trace = nullptr;
    int64_t trace_cap = 0, trace_n = 0;
    bool prof = false;
    uint32_t prof_mask = 0;       // kernel ids (bit DCFM_K_*) timed with events
    int prof_stride = 1;          // time one in prof_stride launches of each (dcfm_set_profiling_stride)
    int64_t prof_seq[DCFM_K_COUNT] = {};   // launches seen per kernel id since the mask was set
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> evpool;
    double kms[DCFM_K_COUNT] = {};
    int64_t kcnt[DCFM_K_COUNT] = {};
};

static std::string g_err;  // errors without a handle

static int fail(dcfm_handle *h, int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf; else g_err = buf;
    return code;
}

#define HIPC(h, x)                                                                        \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess)                                                             \
            return fail(h, DCFM_ERR_HIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                              \
    } while (0)

#define NCCLC(h, x)                                                                       \
    do {                                                                                  \
        ncclResult_t r_ = (x);                                                            \
        if (r_ != ncclSuccess)                                                            \
            return fail(h, DCFM_ERR_RCCL, "%s failed: %s", #x, ncclGetErrorString(r_));   \
    } while (0)

static int dalloc(dcfm_handle *h, double **p, size_t n) {
    void *q = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&q, n * sizeof(double));
    if (e != hipSuccess)
        return fail(h, DCFM_ERR_ALLOC, "hipMalloc(%zu doubles) failed: %s", n, hipGetErrorString(e));
    e = hipMemset(q, 0, n * sizeof(double));
    if (e != hipSuccess) return fail(h, DCFM_ERR_HIP, "hipMemset failed: %s", hipGetErrorString(e));
    h->allocs.push_back(q);
    *p = static_cast<double *>(q);
    return DCFM_OK;
}

static int round_up(int a, int b) { return (a + b - 1) / b * b; }

// ---------------------------------------------------------------------------
// collectives: RCCL communicator per stream (CH_*), or the in-process loopback group
// ---------------------------------------------------------------------------
enum { CH_MAIN = 0, CH_SIDE = 1, CH_ASM = 2 };

static int loop_allgather(dcfm_handle *h, const double *send, double *recv, size_t count, hipStream_t s) {
    LoopGroup &G = *h->loop;
    const int r = h->d.rank;
    HIPC(h, hipEventRecord(h->lp_ready, s));
    {
        std::unique_lock<std::mutex> lk(G.mu);
        G.send[r] = send;
        G.ready[r] = h->lp_ready;
        if (!G.barrier(lk)) return fail(h, DCFM_ERR_RCCL, "loopback all-gather: ranks did not meet");
    }
    for (int k = 0; k < G.n; ++k) {
        double *dst = recv + (size_t)k * count;
        if (G.send[k] == dst) continue;                      // in place
        if (k != r) HIPC(h, hipStreamWaitEvent(s, G.ready[k], 0));
        HIPC(h, hipMemcpyAsync(dst, G.send[k], count * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    HIPC(h, hipEventRecord(h->lp_done, s));
    {
        std::unique_lock<std::mutex> lk(G.mu);
        G.done[r] = h->lp_done;
        if (!G.barrier(lk)) return fail(h, DCFM_ERR_RCCL, "loopback all-gather: ranks did not meet");
    }
    for (int k = 0; k < G.n; ++k)
        if (k != r) HIPC(h, hipStreamWaitEvent(s, G.done[k], 0));
    {
        std::unique_lock<std::mutex> lk(G.mu);
        if (!G.barrier(lk)) return fail(h, DCFM_ERR_RCCL, "loopback all-gather: ranks did not meet");
    }
    return DCFM_OK;
}

// Gather to one rank: rank k's cnt[k] doubles land at recv + base[k] on root (recv is
// only read on root; root's own part is already in place when send == recv + base[root]).
static int loop_gather(dcfm_handle *h, const double *send, double *recv, const std::vector<long long> &base,
                       const std::vector<long long> &cnt, int root, hipStream_t s) {
    LoopGroup &G = *h->loop;
    const int r = h->d.rank;
    HIPC(h, hipEventRecord(h->lp_ready, s));
    {
        std::unique_lock<std::mutex> lk(G.mu);
        G.send[r] = send;
        G.ready[r] = h->lp_ready;
        if (!G.barrier(lk)) return fail(h, DCFM_ERR_RCCL, "loopback gather: ranks did not meet");
    }
    if (r == root)
        for (int k = 0; k < G.n; ++k) {
            if (cnt[k] == 0 || G.send[k] == recv + base[k]) continue;
            if (k != r) HIPC(h, hipStreamWaitEvent(s, G.ready[k], 0));
            HIPC(h, hipMemcpyAsync(recv + base[k], G.send[k], cnt[k] * sizeof(double), hipMemcpyDeviceToDevice, s));
        }
    HIPC(h, hipEventRecord(h->lp_done, s));
    {
        std::unique_lock<std::mutex> lk(G.mu);
        G.done[r] = h->lp_done;
        if (!G.barrier(lk)) return fail(h, DCFM_ERR_RCCL, "loopback gather: ranks did not meet");
    }
    if (r != root) HIPC(h, hipStreamWaitEvent(s, G.done[root], 0));   // root has read my buffer
    {
        std::unique_lock<std::mutex> lk(G.mu);
        if (!G.barrier(lk)) return fail(h, DCFM_ERR_RCCL, "loopback gather: ranks did not meet");
    }
    return DCFM_OK;
}

// recv = concatenation over ranks of count doubles (send may be recv + rank * count)
static int coll_allgather(dcfm_handle *h, int ch, const double *send, double *recv, size_t count, hipStream_t s) {
    if (h->loop) return loop_allgather(h, send, recv, count, s);
    ncclComm_t c = ch == CH_MAIN ? h->comm : (ch == CH_SIDE ? h->comm_side : h->comm_asm);
    NCCLC(h, ncclAllGather(send, recv, count, ncclDouble, c, s));
    return DCFM_OK;
}

// Point-to-point gather of variable-size parts to `root` (no all-reduce of the data): RCCL
// send / recv in one group on the assembly communicator, or the loopback group.
static int coll_gather(dcfm_handle *h, const double *send, double *recv, const std::vector<long long> &base,
                       const std::vector<long long> &cnt, int root, hipStream_t s) {
    if (h->loop) return loop_gather(h, send, recv, base, cnt, root, s);
    const int r = h->d.rank;
    NCCLC(h, ncclGroupStart());
    if (r == root) {
        for (int k = 0; k < h->d.nranks; ++k)
            if (k != root && cnt[k] > 0)
                NCCLC(h, ncclRecv(recv + base[k], (size_t)cnt[k], ncclDouble, k, h->comm_asm, s));
    } else if (cnt[r] > 0) {
        NCCLC(h, ncclSend(send, (size_t)cnt[r], ncclDouble, root, h->comm_asm, s));
    }
    NCCLC(h, ncclGroupEnd());
    return DCFM_OK;
}

// buf = sum over ranks of buf (in rank order for the loopback group)
static int coll_allreduce_sum(dcfm_handle *h, int ch, double *buf, size_t count, hipStream_t s) {
    if (!h->loop) {
        ncclComm_t c = ch == CH_MAIN ? h->comm : (ch == CH_SIDE ? h->comm_side : h->comm_asm);
        NCCLC(h, ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c, s));
        return DCFM_OK;
    }
    void *q = nullptr;
    HIPC(h, hipMalloc(&q, (size_t)h->loop->n * count * sizeof(double)));
    double *all = static_cast<double *>(q);
    int rc = loop_allgather(h, buf, all, count, s);
    if (rc == DCFM_OK) {
        launch_sum_slices(all, h->loop->n, count, buf, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = fail(h, DCFM_ERR_HIP, "loopback all-reduce: %s", hipGetErrorString(e));
    }
    (void)hipFree(all);
    return rc;
}

// ---------------------------------------------------------------------------
// profiling helpers
// ---------------------------------------------------------------------------
static hipEvent_t get_event(dcfm_handle *h) {
    if (!h->evpool.empty()) {
        hipEvent_t e = h->evpool.back();
        h->evpool.pop_back();
        return e;
    }
    // timing only (read after sync_all): no system-scope fence, whose L2 write-back and
    // invalidate per record cost microseconds and slowed the kernel that followed
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

struct KTimer {
    dcfm_handle *h;
    int kid;
    hipStream_t s;
    hipEvent_t a = nullptr;
    KTimer(dcfm_handle *h_, int k, hipStream_t s_) : h(h_), kid(k), s(s_) {
        if (h->prof && (h->prof_mask >> k & 1u) && h->prof_seq[k]++ % h->prof_stride == 0) {
            a = get_event(h);
            if (a) (void)hipEventRecord(a, s);
        }
    }
    ~KTimer() {
        if (h->prof && a) {
            hipEvent_t b = get_event(h);
            if (b) {
                (void)hipEventRecord(b, s);
                h->recs.push_back({kid, a, b});
            }
        }
    }
};

static void sync_all(dcfm_handle *h) {
    (void)hipStreamSynchronize(h->stream);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->sdraw) (void)hipStreamSynchronize(h->sdraw);
    if (h->sasm) (void)hipStreamSynchronize(h->sasm);
}

// row t of the chain trace ([G][4] shard sums after the scratch, trace.hip)
static double *trace_row(dcfm_handle *h, int64_t t) {
    return h->trace + trace_scratch_doubles(h->d.G) + (size_t)t * h->d.G * 4;
}

// DCFM_ERR_NUMERIC once the sentinel of a finished dcfm_run has seen a non-finite state
// (call after the streams are synchronised)
static int numeric_status(dcfm_handle *h) {
    if (h->nan_host && *h->nan_host)
        return fail(h, DCFM_ERR_NUMERIC, "non-finite sampler state (NaN / Inf in Lambda, ps, omega, X or tau) "
                                         "after dcfm_run; set_state / init_state to restart");
    return DCFM_OK;
}
// Collective entry points (get_sigma_cols, sigma_error) must take the same path on every rank:
// a failure only some ranks see (an argument only the root checks, a non-finite local shard)
// would otherwise leave the others blocked in the collective.  Every rank contributes
// [invalid, numeric, other] failure counts to an all-reduce first; any failure anywhere
// fails the call on all ranks (a rank that saw none reports which failure another rank had).
static int agree(dcfm_handle *h, int code) {
    if (!h->d.coll) return code;
    const double f[3] = {code == DCFM_ERR_INVALID ? 1.0 : 0.0, code == DCFM_ERR_NUMERIC ? 1.0 : 0.0,
                         (code != DCFM_OK && code != DCFM_ERR_INVALID && code != DCFM_ERR_NUMERIC) ? 1.0 : 0.0};
    double g[3] = {0.0, 0.0, 0.0};
    const std::string mine = h->err;
    hipError_t e = hipMemcpyAsync(h->b.agree, f, sizeof f, hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) return fail(h, DCFM_ERR_HIP, "agree: %s", hipGetErrorString(e));
    if (int rc = coll_allreduce_sum(h, CH_ASM, h->b.agree, 3, h->stream)) return rc;
    HIPC(h, hipMemcpyAsync(g, h->b.agree, sizeof g, hipMemcpyDeviceToHost, h->stream));
    HIPC(h, hipStreamSynchronize(h->stream));
    if (code != DCFM_OK) {
        h->err = mine;
        return code;
    }
    if (g[0] > 0.0) return fail(h, DCFM_ERR_INVALID, "another rank rejected the collective call's arguments");
    if (g[1] > 0.0) return fail(h, DCFM_ERR_NUMERIC, "another rank's sampler state is non-finite");
    if (g[2] > 0.0) return fail(h, DCFM_ERR_HIP, "the collective call failed on another rank");
    return DCFM_OK;
}
static int reset_numeric(dcfm_handle *h) {
    HIPC(h, hipMemset(h->nan_dev, 0, sizeof(int)));
    *h->nan_host = 0;
    return DCFM_OK;
}

static void collect_prof(dcfm_handle *h) {
    if (h->recs.empty()) return;
    sync_all(h);
    for (auto &r : h->recs) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            h->kms[r.kid] += ms;
            h->kcnt[r.kid] += 1;
        }
        h->evpool.push_back(r.a);
        h->evpool.push_back(r.b);
    }
    h->recs.clear();
}

// Sigma block-sharding: tile rows [Tb[k], Tb[k+1]) to rank k, contiguous, each rank's
// share of the nt(nt+1)/2 lower tiles as near total/nranks as row granularity allows
// (rank k's tiles: tri(Tb[k+1]) - tri(Tb[k])).  Ranks may own no rows when nt < nranks.
static std::vector<int> sigma_split(int nt, int nranks) {
    std::vector<int> Tb(nranks + 1, nt);
    Tb[0] = 0;
    const double total = (double)tri(nt);
    for (int k = 1; k < nranks; ++k) {
        const double target = total * k / nranks;
        int t = Tb[k - 1];
        while (t < nt && (double)tri(t) < target) ++t;                 // first t with tri(t) >= target
        if (t > Tb[k - 1] && target - (double)tri(t - 1) < (double)tri(t) - target) --t;   // the nearer
        Tb[k] = t;
    }
    return Tb;
}

// ---------------------------------------------------------------------------
extern "C" {

int dcfm_abi_version(void) { return DCFM_ABI_VERSION; }

const char *dcfm_last_error(const dcfm_handle *h) { return h ? h->err.c_str() : g_err.c_str(); }

const char *dcfm_kernel_name(int id) {
    static const char *names[DCFM_K_COUNT] = {"k_prep",  "k_wpass", "k_zdraw",  "k_xred",
                                              "k_xdraw", "k_cpass", "k_lambda", "k_colsum",
                                              "k_delta", "k_save",  "k_assemble", "rccl", "k_xchol",
                                              "k_draws", "k_resid"};
    return (id >= 0 && id < DCFM_K_COUNT) ? names[id] : "?";
}

int dcfm_create(const dcfm_config *cfg, dcfm_handle **out) {
    if (!cfg || !out) return fail(nullptr, DCFM_ERR_INVALID, "null argument");
    *out = nullptr;
    const dcfm_config &c = *cfg;
    if (c.n < 1 || c.P < 1 || c.g < 1 || c.K < 1)
        return fail(nullptr, DCFM_ERR_INVALID, "n, P, g, K must be >= 1");
    if (c.K > KP_MAX)
        return fail(nullptr, DCFM_ERR_UNSUPPORTED, "K = %d > %d not supported by this build", c.K, KP_MAX);
    if (!(c.rho >= 0.0 && c.rho <= 1.0)) return fail(nullptr, DCFM_ERR_INVALID, "rho must be in [0,1]");
    if (c.thin < 1 || c.mcmc < 0 || c.burnin < 0)
        return fail(nullptr, DCFM_ERR_INVALID, "thin >= 1, mcmc >= 0, burnin >= 0 required");
    if (!(c.bs > 0 && c.bd1 > 0 && c.bd2 > 0 && c.df > 0))
        return fail(nullptr, DCFM_ERR_INVALID, "bs, bd1, bd2, df must be > 0 (dc:62-65)");
    // on-device gammas (philox.h): Marsaglia-Tsang for shape >= 1, boosted below 1, so every
    // positive hyper-parameter the reference accepts (dc:62-65) is drawn on the device
    if (!(c.as_ > 0.0 && c.ad1 > 0.0 && c.ad2 > 0.0))
        return fail(nullptr, DCFM_ERR_INVALID, "as, ad1, ad2 must be > 0 (dc:62-65; got %g, %g, %g)", c.as_, c.ad1,
                    c.ad2);
    const int nranks = c.nranks < 1 ? 1 : c.nranks;
    if (c.rank < 0 || c.rank >= nranks) return fail(nullptr, DCFM_ERR_INVALID, "bad rank");
    {   // the fused K <= 32 chain keeps the canonical shard-sum trees' levels in registers
        // (k_wcol TreeSum<.., 8>, k_xdraw <.., 10>); the other layouts sum with TREE_LEVELS = 16
        const bool fused = c.K <= KP && !(c.flags & DCFM_FLAG_UNFUSED);
        const int Gl = c.g / nranks, nxs = xsum_blocks(Gl);
        if (fused && (c.g > 1023 || nxs > 255 || Gl / nxs > 255))
            return fail(nullptr, DCFM_ERR_UNSUPPORTED, "g = %d shards (%d per rank): the fused K <= 32 chain takes at "
                        "most 1023, and a per-rank count whose odd part is below 256 (DCFM_FLAG_UNFUSED lifts "
                        "this)", c.g, Gl);
        if (!fused && c.g >= (1 << 16))    // TreeSum's default depth (linalg.h TREE_LEVELS)
            return fail(nullptr, DCFM_ERR_UNSUPPORTED, "g = %d shards: at most %d", c.g, (1 << 16) - 1);
    }
    if (c.g % nranks)
        return fail(nullptr, DCFM_ERR_UNSUPPORTED, "g = %d not divisible by nranks = %d", c.g, nranks);
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev < 1)
        return fail(nullptr, DCFM_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    if (c.device < 0 || c.device >= ndev) return fail(nullptr, DCFM_ERR_INVALID, "bad device %d", c.device);

    dcfm_handle *h = new dcfm_handle();
    h->cfg = c;
    h->cfg.nranks = nranks;
    HIPC(h, hipSetDevice(c.device));
    // Stream priorities: the sweep chain (main, side) at the greatest priority, the draws
    // a batch ahead and the covariance assembly at the least, so the dispatcher hands
    // freed CUs to the latency-critical chain first (DCFM_FLAG_FLAT_PRIORITY: all default).
    int prio_lo = 0, prio_hi = 0;
    if (!(c.flags & DCFM_FLAG_FLAT_PRIORITY)) HIPC(h, hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIPC(h, hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, prio_hi));
    {   // DCFM_FLAG_ONE_STREAM: one stream for everything (isolated per-kernel timings)
        if (c.flags & DCFM_FLAG_ONE_STREAM) {
            h->side = h->sasm = h->sdraw = h->stream;
        } else {
            HIPC(h, hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, prio_hi));
            HIPC(h, hipStreamCreateWithPriority(&h->sdraw, hipStreamNonBlocking, prio_lo));
            HIPC(h, hipStreamCreateWithPriority(&h->sasm, hipStreamNonBlocking, prio_lo));
        }
    }
    HIPC(h, hipEventCreateWithFlags(&h->e_lam, hipEventDisableTiming));
    HIPC(h, hipEventCreateWithFlags(&h->e_prep, hipEventDisableTiming));
    HIPC(h, hipEventCreateWithFlags(&h->e_xchol, hipEventDisableTiming));
    HIPC(h, hipEventCreateWithFlags(&h->e_batch, hipEventDisableTiming));
    HIPC(h, hipEventCreateWithFlags(&h->e_free[0], hipEventDisableTiming));
    HIPC(h, hipEventCreateWithFlags(&h->e_free[1], hipEventDisableTiming));
    for (int sl = 0; sl < 2; ++sl) {
        HIPC(h, hipEventCreateWithFlags(&h->e_drawn[sl], hipEventDisableTiming));
        HIPC(h, hipEventCreateWithFlags(&h->e_used[sl], hipEventDisableTiming));
    }

    {
        void *q = nullptr;
        HIPC(h, hipMalloc(&q, sizeof(int)));
        h->allocs.push_back(q);
        h->nan_dev = static_cast<int *>(q);
        HIPC(h, hipMemset(h->nan_dev, 0, sizeof(int)));
        HIPC(h, hipHostMalloc(&q, sizeof(int), hipHostMallocDefault));
        h->nan_host = static_cast<int *>(q);
        *h->nan_host = 0;
    }
    Dims &d = h->d;
    d.n = c.n; d.P = c.P; d.g = c.g; d.K = c.K;
    d.nranks = nranks; d.rank = c.rank;
    d.coll = (nranks > 1 || (c.flags & DCFM_FLAG_COMM_SELF)) ? 1 : 0;
    d.G = c.g / nranks;
    d.shard0 = c.rank * d.G;
    d.NP = round_up(c.n, 128);
    d.PP = round_up(c.P, 32);
    d.p = c.P * c.g;
    d.kp = c.K <= 32 ? 32 : (c.K <= 64 ? 64 : 128);
    d.rho = c.rho; d.sr = std::sqrt(c.rho); d.s1r = std::sqrt(1.0 - c.rho);
    d.as_ = c.as_; d.bs = c.bs; d.df = c.df; d.ad1 = c.ad1; d.bd1 = c.bd1; d.ad2 = c.ad2; d.bd2 = c.bd2;
    d.seed = c.seed;
    d.inject = (c.flags & DCFM_FLAG_INJECT_DRAWS) ? 1 : 0;
    // K <= 32 runs the fused launch chain unless DCFM_FLAG_UNFUSED asks for the side-stream layout
    h->fused = d.kp == KP && !(c.flags & DCFM_FLAG_UNFUSED);
    // fused narrow chain on several ranks: column sums, the A sum and the X message travel in
    // ONE message per iteration (Dims::sgap / xstride)
    const bool packed = d.coll && h->fused;
    d.sgap = packed ? KP * KP + d.NP * KP : 0;
    d.xstride = packed ? d.G * KP + KP * KP + d.NP * KP : d.kp * d.kp;
    h->B = c.asm_batch > 0 ? c.asm_batch : 32;

    Bufs &b = h->b;
    const size_t G = d.G, NP = d.NP, PP = d.PP, g = d.g, p = d.p, KP = d.kp;
    b.LDB = round_up(h->B * d.K, ASM_KC);
    int rc = DCFM_OK;
#define ALLOC(ptr, n) if ((rc = dalloc(h, &(ptr), (n))) != DCFM_OK) { int r2 = rc; std::string m = h->err; dcfm_destroy(h); g_err = m; return r2; }
    ALLOC(b.Y, G * NP * PP);
    ALLOC(b.yy, G * PP);
    ALLOC(b.Lam, G * PP * KP);
    ALLOC(b.omega, G * PP);
    ALLOC(b.ps, G * PP);
    ALLOC(b.psi, G * PP * KP);
    ALLOC(b.Plam, G * PP * KP);
    ALLOC(b.X, NP * KP);
    ALLOC(b.Z, G * NP * KP);
    ALLOC(b.delta, 2 * g * KP);
    ALLOC(b.tau, 2 * g * KP);
    ALLOC(b.W, G * NP * KP);
    ALLOC(b.A, G * KP * KP);
    ALLOC(b.ZM, G * 4 * KP * KP);
    ALLOC(b.Sp, G * NP * KP);
    if (d.sgap) {   // packed message [sloc | xa | xin] and its gather (dcfm_internal.h, Dims::sgap)
        const size_t msg = (size_t)d.xstride;
        ALLOC(b.sloc, msg);
        b.xa = b.sloc + (size_t)G * KP;
        b.xin = b.xa + KP * KP;
        ALLOC(b.msg_all, (size_t)nranks * msg);
        b.sall = b.msg_all;
        b.xa_all = b.msg_all + (size_t)G * KP;
        b.xall = b.xa_all + KP * KP;
    } else {
        ALLOC(b.xin, NP * KP);
        if (d.coll) { ALLOC(b.xall, (size_t)nranks * NP * KP); } else b.xall = b.xin;
        ALLOC(b.xa, KP * KP);
        ALLOC(b.xa_all, (size_t)nranks * KP * KP);
    }
    ALLOC(b.XM, 2 * KP * KP);
    ALLOC(b.agree, 3);
    {
        double *rf = nullptr;
        ALLOC(rf, (G * (PP / 32) + 1) / 2);   // zeroed: no tile flagged
        b.rflag = reinterpret_cast<int *>(rf);
    }
    ALLOC(b.xpart, (size_t)G * KP * KP);  // k_wcol: xsum_blocks(G) <= G chunk sums
    {
        double *tk = nullptr;
        ALLOC(tk, 1);
        b.ticket = reinterpret_cast<unsigned *>(tk);
        double *sy = nullptr;
        ALLOC(sy, SYNC_ZM + G);           // zeroed: the hand-off counters start at 0 (<= 255 chunks, G shards)
        b.sync = reinterpret_cast<unsigned long long *>(sy);
    }
    ALLOC(b.C, G * PP * KP);
    ALLOC(b.E, G * KP * KP);
    ALLOC(b.cpart, G * PP * KP);
    if (!d.sgap) {
        ALLOC(b.sloc, G * KP);
        if (d.coll) { ALLOC(b.sall, g * KP); } else b.sall = b.sloc;
    }
    ALLOC(b.Lb[0], p * (size_t)b.LDB);
    ALLOC(b.Lb[1], p * (size_t)b.LDB);
    ALLOC(b.wsum[0], p);
    ALLOC(b.wsum[1], p);
    // Sigmaout block-sharded over ranks: contiguous tile rows balanced by tile count
    {
        const int nt = (d.p + ASM_TILE - 1) / ASM_TILE;
        h->Tb = sigma_split(nt, nranks);
        b.T0 = h->Tb[c.rank];
        b.T1 = h->Tb[c.rank + 1];
    }
    ALLOC(b.Sigma, (size_t)(tri(b.T1) - tri(b.T0)) * ASM_TILE * ASM_TILE);
    // the generated fused chain: k_wcol's LAMGEN blocks draw the loading-row variates into b.ldraw
    // each iteration (lam_draws)
    if (h->fused && !d.inject) ALLOC(b.ldraw, (size_t)lam_gen_doubles(d));
    if (!d.inject && !h->fused) {   // k_draws batches of the side-stream layouts
        const size_t K = c.K, n = c.n, P = c.P;
        const size_t nz = K * n * g, nx = K * n, nl = K * P * g, gpsi = P * K * g, gdel = K * g, gps = P * g;
        const size_t per_it = nz + nx + nl + gpsi + gdel + gps;
        // batches of up to 8 iterations, two slots within ~2 GiB
        h->DB = (int)std::max<size_t>(1, std::min<size_t>(8, (size_t(2) << 30) / (2 * per_it * sizeof(double))));
        const size_t sz[6] = {nz, nx, nl, gpsi, gdel, gps};
        for (int i = 0; i < 6; ++i) h->draw_iter_sz[i] = sz[i];
        double *gm = nullptr;
        ALLOC(gm, 2 * (size_t)h->DB * per_it);
        for (int sl = 0; sl < 2; ++sl) {
            DrawsDev &G = h->gen[sl];
            G.NZ = gm; gm += nz * h->DB;
            G.NX = gm; gm += nx * h->DB;
            G.NL = gm; gm += nl * h->DB;
            G.Gpsi = gm; gm += gpsi * h->DB;
            G.Gdelta = gm; gm += gdel * h->DB;
            G.Gps = gm; gm += gps * h->DB;
            G.first_iter = -1;
            G.n_iter = h->DB;
        }
    }
#undef ALLOC
    // this rank's lower-triangle assembly tiles in k_assemble's processing order: 8 x 8-tile
    // supertiles (row bands of the rank's block, then column bands), row-major inside — the
    // tiles an XCD runs together share their Lb panels in L2.  (Storage is by (ti, tj).)
    {
        constexpr int SB = 8;
        std::vector<int2> tl;
        for (int rb0 = b.T0; rb0 < b.T1; rb0 += SB) {
            const int rb1 = std::min(b.T1, rb0 + SB);
            for (int cb0 = 0; cb0 < rb1; cb0 += SB)
                for (int ti = rb0; ti < rb1; ++ti)
                    for (int tj = cb0; tj < std::min(cb0 + SB, ti + 1); ++tj) tl.push_back(make_int2(ti, tj));
        }
        if ((int64_t)tl.size() != tri(b.T1) - tri(b.T0))
            return fail(h, DCFM_ERR_INVALID, "assembly tile list: %zu tiles for %lld", tl.size(),
                        (long long)(tri(b.T1) - tri(b.T0)));
        b.ntiles = (int)tl.size();
        void *q = nullptr;
        HIPC(h, hipMalloc(&q, std::max<size_t>(1, tl.size()) * sizeof(int2)));
        h->allocs.push_back(q);
        b.tiles = static_cast<int2 *>(q);
        if (!tl.empty()) HIPC(h, hipMemcpy(b.tiles, tl.data(), tl.size() * sizeof(int2), hipMemcpyHostToDevice));
    }
    // pad delta/tau with ones
    {
        std::vector<double> ones(2 * g * KP, 1.0);
        HIPC(h, hipMemcpy(b.delta, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice));
        HIPC(h, hipMemcpy(b.tau, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    *out = h;
    return DCFM_OK;
}

void dcfm_destroy(dcfm_handle *h) {
    if (!h) return;
    (void)hipSetDevice(h->cfg.device);
    if (h->stream) sync_all(h);
    for (auto &r : h->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : h->evpool) (void)hipEventDestroy(e);
    for (hipEvent_t e : {h->e_lam, h->e_prep, h->e_xchol, h->e_batch, h->e_free[0], h->e_free[1], h->e_drawn[0],
                         h->e_drawn[1], h->e_used[0], h->e_used[1]})
        if (e) (void)hipEventDestroy(e);
    if (h->lp_ready) (void)hipEventDestroy(h->lp_ready);
    if (h->lp_done) (void)hipEventDestroy(h->lp_done);
    if (h->comm_asm) ncclCommDestroy(h->comm_asm);
    if (h->comm_side) ncclCommDestroy(h->comm_side);
    if (h->comm) ncclCommDestroy(h->comm);
    for (void *q : h->allocs) (void)hipFree(q);
    if (h->nan_host) (void)hipHostFree(h->nan_host);
    if (h->draws_mem) (void)hipFree(h->draws_mem);
    if (h->trace) (void)hipFree(h->trace);
    if (h->sasm && h->sasm != h->stream) (void)hipStreamDestroy(h->sasm);
    if (h->side && h->side != h->stream) (void)hipStreamDestroy(h->side);
    if (h->sdraw && h->sdraw != h->stream) (void)hipStreamDestroy(h->sdraw);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int dcfm_comm_unique_id(uint8_t out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(nullptr, DCFM_ERR_RCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    std::memcpy(out, &id, 128);
    return DCFM_OK;
}

int dcfm_comm_init(dcfm_handle *h, const uint8_t id[128]) {
    if (!h || !id) return fail(h, DCFM_ERR_INVALID, "null argument");
    if (!h->d.coll) return DCFM_OK;
    HIPC(h, hipSetDevice(h->cfg.device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    NCCLC(h, ncclCommInitRank(&h->comm, h->d.nranks, uid, h->d.rank));
    // one communicator per stream so collectives on different streams never interleave
    NCCLC(h, ncclCommSplit(h->comm, 0, h->d.rank, &h->comm_side, nullptr));
    NCCLC(h, ncclCommSplit(h->comm, 0, h->d.rank, &h->comm_asm, nullptr));
    h->comm_ok = true;
    return DCFM_OK;
}

int dcfm_comm_init_loopback(dcfm_handle *const *hs, int32_t n) {
    if (!hs || n < 1) return fail(nullptr, DCFM_ERR_INVALID, "null handles or n < 1");
    for (int r = 0; r < n; ++r) {
        if (!hs[r]) return fail(nullptr, DCFM_ERR_INVALID, "null handle %d", r);
        if (hs[r]->d.nranks != n || hs[r]->d.rank != r)
            return fail(hs[r], DCFM_ERR_INVALID, "handle %d: nranks %d rank %d, expected %d / %d", r,
                        hs[r]->d.nranks, hs[r]->d.rank, n, r);
        if (hs[r]->cfg.device != hs[0]->cfg.device)
            return fail(hs[r], DCFM_ERR_INVALID, "loopback ranks must share one device");
    }
    auto G = std::make_shared<LoopGroup>(n);
    for (int r = 0; r < n; ++r) {
        dcfm_handle *h = hs[r];
        HIPC(h, hipSetDevice(h->cfg.device));
        if (!h->lp_ready) HIPC(h, hipEventCreateWithFlags(&h->lp_ready, hipEventDisableTiming));
        if (!h->lp_done) HIPC(h, hipEventCreateWithFlags(&h->lp_done, hipEventDisableTiming));
        h->loop = G;
        h->comm_ok = true;
    }
    return DCFM_OK;
}

// Yd local: n x P x G column-major: (i, j, m) at i + n*j + n*P*m  ->  Y[m][i][j]
int dcfm_set_data(dcfm_handle *h, const double *Yd) {
    if (!h || !Yd) return fail(h, DCFM_ERR_INVALID, "null argument");
    const Dims &d = h->d;
    HIPC(h, hipSetDevice(h->cfg.device));
    std::vector<double> buf((size_t)d.NP * d.PP, 0.0);
    std::vector<double> yy((size_t)d.G * d.PP, 0.0);
    for (int m = 0; m < d.G; ++m) {
        std::fill(buf.begin(), buf.end(), 0.0);
        const double *src = Yd + (size_t)m * d.n * d.P;
        for (int j = 0; j < d.P; ++j) {
            double s = 0.0;
            for (int i = 0; i < d.n; ++i) {
                const double v = src[(size_t)j * d.n + i];
                buf[(size_t)i * d.PP + j] = v;
                s += v * v;
            }
            yy[(size_t)m * d.PP + j] = s;
        }
        HIPC(h, hipMemcpy(h->b.Y + (size_t)m * d.NP * d.PP, buf.data(), buf.size() * sizeof(double),
                          hipMemcpyHostToDevice));
    }
    HIPC(h, hipMemcpy(h->b.yy, yy.data(), yy.size() * sizeof(double), hipMemcpyHostToDevice));
    h->have_data = true;
    return DCFM_OK;
}

// device scratch freed on every return path of the ingest entry points
struct DevScratch {
    std::vector<void *> p;
    ~DevScratch() { for (void *q : p) (void)hipFree(q); }
    hipError_t alloc(void **q, size_t bytes) {
        hipError_t e = hipMalloc(q, std::max<size_t>(bytes, 1));
        if (e == hipSuccess) p.push_back(*q);
        return e;
    }
};

int dcfm_set_data_raw(dcfm_handle *h, const double *Y, int64_t p_in, const int64_t *cols, double *sd_out,
                      double *dev_ms) {
    if (!h || !Y || !cols) return fail(h, DCFM_ERR_INVALID, "null argument");
    const Dims &d = h->d;
    if (d.n < 2) return fail(h, DCFM_ERR_INVALID, "set_data_raw: var (dc:57) needs n >= 2");
    const int64_t ncols = (int64_t)d.P * d.G;
    for (int64_t c = 0; c < ncols; ++c)
        if (cols[c] < 0 || cols[c] >= p_in)
            return fail(h, DCFM_ERR_INVALID, "set_data_raw: cols[%lld] = %lld outside [0, %lld)", (long long)c,
                        (long long)cols[c], (long long)p_in);
    HIPC(h, hipSetDevice(h->cfg.device));
    DevScratch sc;
    void *qY = nullptr, *qc = nullptr, *qsd = nullptr, *qbad = nullptr, *qmi = nullptr;
    const size_t ybytes = (size_t)d.n * (size_t)p_in * sizeof(double);
    if (sc.alloc(&qY, ybytes) != hipSuccess || sc.alloc(&qc, ncols * sizeof(int64_t)) != hipSuccess ||
        sc.alloc(&qsd, ncols * sizeof(double)) != hipSuccess || sc.alloc(&qbad, sizeof(int)) != hipSuccess ||
        sc.alloc(&qmi, 2 * ncols * sizeof(double)) != hipSuccess)
        return fail(h, DCFM_ERR_ALLOC, "set_data_raw: device scratch (%zu bytes of Y) failed", ybytes);
    hipStream_t s = h->stream;
    HIPC(h, hipMemcpyAsync(qY, Y, ybytes, hipMemcpyHostToDevice, s));
    HIPC(h, hipMemcpyAsync(qc, cols, ncols * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPC(h, hipMemsetAsync(qbad, 0, sizeof(int), s));
    hipEvent_t ea = get_event(h), eb = get_event(h);
    if (!ea || !eb) return fail(h, DCFM_ERR_HIP, "set_data_raw: hipEventCreate failed");
    HIPC(h, hipEventRecord(ea, s));
    launch_stdize(d, static_cast<const double *>(qY), static_cast<const long long *>(qc), h->b.Y, h->b.yy,
                  static_cast<double *>(qsd), static_cast<int *>(qbad), static_cast<double *>(qmi), s);
    HIPC(h, hipGetLastError());
    HIPC(h, hipEventRecord(eb, s));
    int bad = 0;
    HIPC(h, hipMemcpyAsync(&bad, qbad, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPC(h, hipStreamSynchronize(s));
    if (dev_ms) {
        float ms = 0.f;
        HIPC(h, hipEventElapsedTime(&ms, ea, eb));
        *dev_ms = ms;
    }
    h->evpool.push_back(ea);
    h->evpool.push_back(eb);
    if (bad) {
        h->have_data = false;
        return fail(h, DCFM_ERR_INVALID, "a constant non-zero column has zero variance (dc:59 divides by zero, Q13)");
    }
    if (sd_out) HIPC(h, hipMemcpy(sd_out, qsd, ncols * sizeof(double), hipMemcpyDeviceToHost));
    h->have_data = true;
    return DCFM_OK;
}

int dcfm_init_state(dcfm_handle *h) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    HIPC(h, hipSetDevice(h->cfg.device));
    sync_all(h);
    launch_init_state(h->d, h->b, h->stream);
    HIPC(h, hipGetLastError());
    HIPC(h, hipStreamSynchronize(h->stream));
    h->cur = 0;
    h->plam_valid = true;      // Plam = psi o tau' was formed (dc:86), as set_state's caller Plam
    h->have_state = true;
    return reset_numeric(h);
}

int dcfm_get_data(dcfm_handle *h, double *Yd_local) {
    if (!h || !Yd_local) return fail(h, DCFM_ERR_INVALID, "null argument");
    if (!h->have_data) return fail(h, DCFM_ERR_INVALID, "get_data: no data set");
    const Dims &d = h->d;
    HIPC(h, hipSetDevice(h->cfg.device));
    HIPC(h, hipStreamSynchronize(h->stream));
    std::vector<double> buf((size_t)d.NP * d.PP);
    for (int m = 0; m < d.G; ++m) {
        HIPC(h, hipMemcpy(buf.data(), h->b.Y + (size_t)m * d.NP * d.PP, buf.size() * sizeof(double),
                          hipMemcpyDeviceToHost));
        double *dst = Yd_local + (size_t)m * d.n * d.P;
        for (int j = 0; j < d.P; ++j)
            for (int i = 0; i < d.n; ++i) dst[(size_t)j * d.n + i] = buf[(size_t)i * d.PP + j];
    }
    return DCFM_OK;
}

int dcfm_count_nonzero_columns(int device, const double *Y, int32_t n, int64_t p, int32_t *nnz_out,
                               double *dev_ms) {
    if (!Y || !nnz_out || n < 0 || p < 0) return fail(nullptr, DCFM_ERR_INVALID, "count_nonzero_columns: bad argument");
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail(nullptr, DCFM_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e));
    DevScratch sc;
    void *qY = nullptr, *qn = nullptr;
    const size_t ybytes = (size_t)n * (size_t)p * sizeof(double);
    if (sc.alloc(&qY, ybytes) != hipSuccess || sc.alloc(&qn, (size_t)p * sizeof(int32_t)) != hipSuccess)
        return fail(nullptr, DCFM_ERR_ALLOC, "count_nonzero_columns: device scratch (%zu bytes) failed", ybytes);
    hipEvent_t ea = nullptr, eb = nullptr;
    float ms = 0.f;
    e = hipMemcpy(qY, Y, ybytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipEventCreate(&ea);
    if (e == hipSuccess) e = hipEventCreate(&eb);
    if (e == hipSuccess) e = hipEventRecord(ea, nullptr);
    if (e == hipSuccess) {
        launch_nnz_cols(static_cast<const double *>(qY), n, p, static_cast<int *>(qn), nullptr);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(eb, nullptr);
    if (e == hipSuccess) e = hipMemcpy(nnz_out, qn, (size_t)p * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, ea, eb);
    if (ea) (void)hipEventDestroy(ea);
    if (eb) (void)hipEventDestroy(eb);
    if (e != hipSuccess) return fail(nullptr, DCFM_ERR_HIP, "count_nonzero_columns: %s", hipGetErrorString(e));
    if (dev_ms) *dev_ms = ms;
    return DCFM_OK;
}

// P x K x G col-major (j,k,m) at j + P*k + P*K*m  <->  dev [m][j][k] (PP x KP)
static void pk_to_dev(const Dims &d, const double *src, std::vector<double> &dst) {
    const int KP = d.kp;
    dst.assign((size_t)d.G * d.PP * KP, 0.0);
    for (int m = 0; m < d.G; ++m)
        for (int k = 0; k < d.K; ++k)
            for (int j = 0; j < d.P; ++j)
                dst[((size_t)m * d.PP + j) * KP + k] = src[(size_t)j + (size_t)d.P * k + (size_t)d.P * d.K * m];
}
static void pk_from_dev(const Dims &d, const std::vector<double> &src, double *dst) {
    const int KP = d.kp;
    for (int m = 0; m < d.G; ++m)
        for (int k = 0; k < d.K; ++k)
            for (int j = 0; j < d.P; ++j)
                dst[(size_t)j + (size_t)d.P * k + (size_t)d.P * d.K * m] = src[((size_t)m * d.PP + j) * KP + k];
}
// n x K x G col-major (i,k,m) <-> dev [m][i][k] (NP x KP)
static void nk_to_dev(const Dims &d, const double *src, int G, std::vector<double> &dst) {
    const int KP = d.kp;
    dst.assign((size_t)G * d.NP * KP, 0.0);
    for (int m = 0; m < G; ++m)
        for (int k = 0; k < d.K; ++k)
            for (int i = 0; i < d.n; ++i)
                dst[((size_t)m * d.NP + i) * KP + k] = src[(size_t)i + (size_t)d.n * k + (size_t)d.n * d.K * m];
}
static void nk_from_dev(const Dims &d, const std::vector<double> &src, int G, double *dst) {
    const int KP = d.kp;
    for (int m = 0; m < G; ++m)
        for (int k = 0; k < d.K; ++k)
            for (int i = 0; i < d.n; ++i)
                dst[(size_t)i + (size_t)d.n * k + (size_t)d.n * d.K * m] = src[((size_t)m * d.NP + i) * KP + k];
}
// P x G col-major (j,m) <-> dev [m][j] (PP)
static void p_to_dev(const Dims &d, const double *src, std::vector<double> &dst) {
    dst.assign((size_t)d.G * d.PP, 0.0);
    for (int m = 0; m < d.G; ++m)
        for (int j = 0; j < d.P; ++j) dst[(size_t)m * d.PP + j] = src[(size_t)j + (size_t)d.P * m];
}
static void p_from_dev(const Dims &d, const std::vector<double> &src, double *dst) {
    for (int m = 0; m < d.G; ++m)
        for (int j = 0; j < d.P; ++j) dst[(size_t)j + (size_t)d.P * m] = src[(size_t)m * d.PP + j];
}
// K x 1 x g col-major (k,m) <-> dev [m][k] (KP), pads 1
static void k_to_dev(const Dims &d, const double *src, std::vector<double> &dst) {
    const int KP = d.kp;
    dst.assign((size_t)d.g * KP, 1.0);
    for (int m = 0; m < d.g; ++m)
        for (int k = 0; k < d.K; ++k) dst[(size_t)m * KP + k] = src[(size_t)k + (size_t)d.K * m];
}
static void k_from_dev(const Dims &d, const std::vector<double> &src, double *dst) {
    const int KP = d.kp;
    for (int m = 0; m < d.g; ++m)
        for (int k = 0; k < d.K; ++k) dst[(size_t)k + (size_t)d.K * m] = src[(size_t)m * KP + k];
}

static int up(dcfm_handle *h, double *dev, const std::vector<double> &v) {
    HIPC(h, hipMemcpy(dev, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice));
    return DCFM_OK;
}
static int down(dcfm_handle *h, std::vector<double> &v, const double *dev, size_t n) {
    v.resize(n);
    HIPC(h, hipMemcpy(v.data(), dev, n * sizeof(double), hipMemcpyDeviceToHost));
    return DCFM_OK;
}

int dcfm_set_state(dcfm_handle *h, const dcfm_state_view *s) {
    if (!h || !s) return fail(h, DCFM_ERR_INVALID, "null argument");
    if (!s->Lambda || !s->ps || !s->omega || !s->psi || !s->Plam || !s->X || !s->Z || !s->delta || !s->tauh)
        return fail(h, DCFM_ERR_INVALID, "set_state: every member except eta is required");
    const Dims &d = h->d;
    HIPC(h, hipSetDevice(h->cfg.device));
    sync_all(h);
    std::vector<double> v;
    int rc;
    pk_to_dev(d, s->Lambda, v); if ((rc = up(h, h->b.Lam, v))) return rc;
    pk_to_dev(d, s->psi, v);    if ((rc = up(h, h->b.psi, v))) return rc;
    pk_to_dev(d, s->Plam, v);   if ((rc = up(h, h->b.Plam, v))) return rc;
    p_to_dev(d, s->ps, v);      if ((rc = up(h, h->b.ps, v))) return rc;
    p_to_dev(d, s->omega, v);   if ((rc = up(h, h->b.omega, v))) return rc;
    nk_to_dev(d, s->X, 1, v);   if ((rc = up(h, h->b.X, v))) return rc;
    nk_to_dev(d, s->Z, d.G, v); if ((rc = up(h, h->b.Z, v))) return rc;
    h->cur = 0;
    k_to_dev(d, s->delta, v);   if ((rc = up(h, h->b.delta, v))) return rc;
    k_to_dev(d, s->tauh, v);    if ((rc = up(h, h->b.tau, v))) return rc;
    h->plam_valid = true;
    h->have_state = true;
    return reset_numeric(h);
}

static int get_state(dcfm_handle *h, dcfm_state_view *o, bool checked) {
    if (!h || !o) return fail(h, DCFM_ERR_INVALID, "null argument");
    const Dims &d = h->d;
    HIPC(h, hipSetDevice(h->cfg.device));
    sync_all(h);
    if (checked)
        if (int rc = numeric_status(h)) return rc;
    std::vector<double> v;
    int rc;
    const size_t KP = d.kp;
    const size_t npk = (size_t)d.G * d.PP * KP, nnk = (size_t)d.G * d.NP * KP;
    if (o->Lambda) { if ((rc = down(h, v, h->b.Lam, npk))) return rc; pk_from_dev(d, v, o->Lambda); }
    if (o->psi) { if ((rc = down(h, v, h->b.psi, npk))) return rc; pk_from_dev(d, v, o->psi); }
    if (o->Plam) {
        if (h->plam_valid) {
            if ((rc = down(h, v, h->b.Plam, npk))) return rc;
        } else {   // Plam = psi o tau' (dc:176) of the last iteration, formed as k_lambda forms it
            std::vector<double> tau;
            if ((rc = down(h, v, h->b.psi, npk))) return rc;
            if ((rc = down(h, tau, h->b.tau + h->cur * (size_t)d.g * KP, (size_t)d.g * KP))) return rc;
            for (int m = 0; m < d.G; ++m)
                for (int j = 0; j < d.P; ++j)
                    for (int k = 0; k < d.K; ++k) {
                        double &x = v[((size_t)m * d.PP + j) * KP + k];
                        x = x * tau[(size_t)(d.shard0 + m) * KP + k];
                    }
        }
        pk_from_dev(d, v, o->Plam);
    }
    if (o->ps) { if ((rc = down(h, v, h->b.ps, (size_t)d.G * d.PP))) return rc; p_from_dev(d, v, o->ps); }
    if (o->omega) { if ((rc = down(h, v, h->b.omega, (size_t)d.G * d.PP))) return rc; p_from_dev(d, v, o->omega); }
    if (o->X) { if ((rc = down(h, v, h->b.X, (size_t)d.NP * KP))) return rc; nk_from_dev(d, v, 1, o->X); }
    if (o->Z) { if ((rc = down(h, v, h->b.Z, nnk))) return rc; nk_from_dev(d, v, d.G, o->Z); }
    if (o->eta) {
        launch_eta(d, h->b, h->b.W, h->stream);   // W is scratch between iterations
        HIPC(h, hipGetLastError());
        HIPC(h, hipStreamSynchronize(h->stream));
        if ((rc = down(h, v, h->b.W, nnk))) return rc;
        nk_from_dev(d, v, d.G, o->eta);
    }
    const size_t nkg = (size_t)d.g * KP;
    if (o->delta) { if ((rc = down(h, v, h->b.delta + h->cur * nkg, nkg))) return rc; k_from_dev(d, v, o->delta); }
    if (o->tauh) { if ((rc = down(h, v, h->b.tau + h->cur * nkg, nkg))) return rc; k_from_dev(d, v, o->tauh); }
    return DCFM_OK;
}

int dcfm_get_state(dcfm_handle *h, dcfm_state_view *o) { return get_state(h, o, true); }

// forensic read after DCFM_ERR_NUMERIC: the state as the device holds it, non-finite values included
int dcfm_get_state_raw(dcfm_handle *h, dcfm_state_view *o) { return get_state(h, o, false); }

int dcfm_set_draws(dcfm_handle *h, const dcfm_draws_view *dv, int64_t first_iter, int64_t n_iter) {
    if (!h || !dv || n_iter < 1) return fail(h, DCFM_ERR_INVALID, "bad argument");
    if (!dv->NZ || !dv->NX || !dv->NL || !dv->Gpsi || !dv->Gdelta || !dv->Gps)
        return fail(h, DCFM_ERR_INVALID, "set_draws: all six arrays required");
    const Dims &d = h->d;
    HIPC(h, hipSetDevice(h->cfg.device));
    sync_all(h);
    const size_t T = n_iter;
    const size_t nNZ = (size_t)d.K * d.n * d.g * T, nNX = (size_t)d.K * d.n * T,
                 nNL = (size_t)d.K * d.P * d.g * T, nPsi = (size_t)d.P * d.K * d.g * T,
                 nDel = (size_t)d.K * d.g * T, nPs = (size_t)d.P * d.g * T;
    const size_t tot = nNZ + nNX + nNL + nPsi + nDel + nPs;
    if (h->draws_mem) { (void)hipFree(h->draws_mem); h->draws_mem = nullptr; }
    void *q = nullptr;
    HIPC(h, hipMalloc(&q, tot * sizeof(double)));
    h->draws_mem = static_cast<double *>(q);
    double *p = h->draws_mem;
    const double *srcs[6] = {dv->NZ, dv->NX, dv->NL, dv->Gpsi, dv->Gdelta, dv->Gps};
    const size_t cnt[6] = {nNZ, nNX, nNL, nPsi, nDel, nPs};
    const double **dsts[6] = {&h->dr.NZ, &h->dr.NX, &h->dr.NL, &h->dr.Gpsi, &h->dr.Gdelta, &h->dr.Gps};
    // Gpsi: MATLAB P x K x g x T -> device [T][g][P][K] (the loading-row kernels read a row's K gammas)
    std::vector<double> gpsi(nPsi);
    for (size_t t = 0; t < T; ++t)
        for (int m = 0; m < d.g; ++m)
            for (int k = 0; k < d.K; ++k)
                for (int j = 0; j < d.P; ++j)
                    gpsi[((t * d.g + m) * d.P + j) * d.K + k] = dv->Gpsi[j + (size_t)d.P * (k + (size_t)d.K * (m + (size_t)d.g * t))];
    srcs[3] = gpsi.data();
    for (int k = 0; k < 6; ++k) {
        HIPC(h, hipMemcpy(p, srcs[k], cnt[k] * sizeof(double), hipMemcpyHostToDevice));
        *dsts[k] = p;
        p += cnt[k];
    }
    h->dr.first_iter = first_iter;
    h->dr.n_iter = n_iter;
    return DCFM_OK;
}

// Hand the filled Lb[lb] batch to the assembly stream (overlaps the next iterations).
static int flush_batch(dcfm_handle *h) {
    if (h->batch == 0) return DCFM_OK;
    Dims &d = h->d;
    Bufs &b = h->b;
    const int lb = h->lb;
    HIPC(h, hipEventRecord(h->e_batch, h->stream));
    HIPC(h, hipStreamWaitEvent(h->sasm, h->e_batch, 0));
    if (d.coll) {
        KTimer t(h, DCFM_K_COMM, h->sasm);
        const size_t rows = (size_t)d.G * d.P;
        if (!h->loop) NCCLC(h, ncclGroupStart());
        int rc = coll_allgather(h, CH_ASM, b.Lb[lb] + (size_t)d.rank * rows * b.LDB, b.Lb[lb], rows * b.LDB,
                                h->sasm);
        if (rc == DCFM_OK)
            rc = coll_allgather(h, CH_ASM, b.wsum[lb] + (size_t)d.rank * rows, b.wsum[lb], rows, h->sasm);
        if (!h->loop) NCCLC(h, ncclGroupEnd());
        if (rc) return rc;
    }
    // k extent: the batch's columns rounded to the MFMA k-step (4); k_assemble stages whole
    // chunks of ASM_KC columns, so columns [used, round_up(used, ASM_KC)) must be zero
    const int used = h->batch * d.K, kext = round_up(used, 4), kstage = round_up(used, ASM_KC);
    const double effsamp = (double)h->cfg.mcmc / (double)h->cfg.thin;   // dc:45 (Q8)
    // k_save wrote columns [0, used) of every row; only the chunk's tail [used, kstage) can
    // hold an earlier batch's samples: zero just that (not the p x LDB buffer)
    if (kstage > used)
        HIPC(h, hipMemset2DAsync(b.Lb[lb] + used, (size_t)b.LDB * sizeof(double), 0, (size_t)(kstage - used) * sizeof(double),
                                 (size_t)d.p, h->sasm));
    {
        KTimer t(h, DCFM_K_ASSEMBLE, h->sasm);
        launch_assemble(d, b, b.Lb[lb], b.wsum[lb], kext, 1.0 / effsamp, h->sasm);
    }
    HIPC(h, hipGetLastError());
    HIPC(h, hipMemsetAsync(b.wsum[lb], 0, (size_t)d.p * sizeof(double), h->sasm));   // k_save adds into it
    HIPC(h, hipEventRecord(h->e_free[lb], h->sasm));
    h->asm_pending[lb] = true;
    h->lb ^= 1;
    h->batch = 0;
    return DCFM_OK;
}

int dcfm_run(dcfm_handle *h, int64_t first_iter, int64_t n_iter) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    if (!h->have_data || !h->have_state) return fail(h, DCFM_ERR_INVALID, "set_data and set_state first");
    if (first_iter < 1 || n_iter < 0) return fail(h, DCFM_ERR_INVALID, "iterations are 1-based");
    Dims &d = h->d;
    Bufs &b = h->b;
    if (d.coll && !h->comm_ok) return fail(h, DCFM_ERR_INVALID, "dcfm_comm_init first (nranks > 1 or COMM_SELF)");
    if (d.inject) {
        if (!h->dr.NZ) return fail(h, DCFM_ERR_INVALID, "INJECT_DRAWS set but no draws");
        if (first_iter < h->dr.first_iter || first_iter + n_iter > h->dr.first_iter + h->dr.n_iter)
            return fail(h, DCFM_ERR_INVALID, "iterations [%lld,%lld) not covered by injected draws",
                        (long long)first_iter, (long long)(first_iter + n_iter));
    }
    HIPC(h, hipSetDevice(h->cfg.device));
    hipStream_t s = h->stream, ss = h->side, sd = h->sdraw;
    const size_t KW = d.kp;
    const size_t nkg = (size_t)d.g * KW;
    const int64_t end_iter = first_iter + n_iter;
    // K <= 32: the per-shard operators ride in the fused launches on the main stream
    // (k_wcol, k_xdraw); K > 32 (or DCFM_FLAG_UNFUSED): prep and the X operators run on the
    // side stream
    const bool fused = h->fused;
    const bool lamgen = fused && !d.inject;   // k_wcol draws k_lambda's variates (b.ldraw)
    // fused (K <= 32): per iteration t, k_wcol = [Z operators and shard sum of A of t, column
    // sums of t-1] beside the W pass of t, whose tiles draw Z; one rank: the last chunk also
    // factors Xprec.  Several ranks: k_xred and ONE all-gather of [column sums | A sum | X
    // message].  Then k_xdraw = [X operators (several ranks), delta chain of t-1] beside the X
    // draw.  k_wcol also draws the loading-row variates of t (generated chain).  The last
    // iteration's chain runs after the loop (k_delta).
    const bool wc = fused && !d.coll;
    bool delta_pending = false;           // k_lambda of it - 1 ran, its delta chain not yet queued
    auto after_delta = [&]() {            // iteration it - 1 is complete
        h->cur ^= 1;
        if (h->trace_n < h->trace_cap) {                                  // dcfm_set_trace
            launch_trace(d, b, b.tau + h->cur * nkg, h->trace, trace_row(h, h->trace_n), s);
            h->trace_n += 1;
        }
    };
    // generated draws: batches [b0, b0 + DB) aligned to this call's first iteration,
    // queued on sdraw into a slot whose previous batch the sweep has finished with
    int rc_gen = DCFM_OK;
    auto gen_batch = [&](int64_t b0, int busy) -> int {
        const int64_t nb = std::min<int64_t>(h->DB, end_iter - b0);
        for (int sl = 0; sl < 2; ++sl)
            if (h->gen_first[sl] == b0 && h->gen_n[sl] >= nb) return sl;
        int sl = busy >= 0 ? 1 - busy : (h->gen_first[0] <= h->gen_first[1] ? 0 : 1);
        hipError_t e = hipSuccess;
        if (h->used_pending[sl]) {
            e = hipStreamWaitEvent(sd, h->e_used[sl], 0);
            h->used_pending[sl] = false;
        }
        for (int64_t it = b0; e == hipSuccess && it < b0 + nb; ++it) {
            const size_t o = (size_t)(it - b0);
            DrawsDev v = h->gen[sl];
            v.NZ += o * h->draw_iter_sz[0];
            v.NX += o * h->draw_iter_sz[1];
            v.NL += o * h->draw_iter_sz[2];
            v.Gpsi += o * h->draw_iter_sz[3];
            v.Gdelta += o * h->draw_iter_sz[4];
            v.Gps += o * h->draw_iter_sz[5];
            v.first_iter = it;
            v.n_iter = 1;
            KTimer t(h, DCFM_K_DRAWS, sd);
            launch_draws(d, v, it, sd);
        }
        if (e == hipSuccess) e = hipEventRecord(h->e_drawn[sl], sd);
        if (e != hipSuccess) {
            rc_gen = fail(h, DCFM_ERR_HIP, "draws batch at iteration %lld: %s", (long long)b0, hipGetErrorString(e));
            return -1;
        }
        h->gen[sl].first_iter = b0;
        h->gen_first[sl] = b0;
        h->gen_n[sl] = nb;
        return sl;
    };
    // Generated draws (Philox, counter-addressed): the fused K <= 32 chain (any rank count) draws
    // its variates where they are consumed (Z / X normals, the delta gammas) or in the launch
    // before (k_lambda's normals and gammas: the LAMGEN blocks of k_wcol, behind its W tiles); the
    // other paths read k_draws buffers generated a batch ahead on the draw stream
    const bool gen_draws = !d.inject && !fused;
    int slot = -1;
    int64_t batch0 = first_iter, batch_n = 0;
    if (!fused) HIPC(h, hipEventRecord(h->e_lam, s));   // Lambda/omega of the previous iteration are final
    for (int64_t it = first_iter; it < end_iter; ++it) {
        if (gen_draws && (it == first_iter || it == batch0 + batch_n)) {
            batch0 = it;
            batch_n = std::min<int64_t>(h->DB, end_iter - it);
            slot = gen_batch(it, -1);
            if (slot < 0) return rc_gen;
            HIPC(h, hipStreamWaitEvent(s, h->e_drawn[slot], 0));
            if (it + batch_n < end_iter && gen_batch(it + batch_n, slot) < 0) return rc_gen;   // next batch
        }
        const DrawsDev &dr = d.inject ? h->dr : h->gen[gen_draws ? slot : 0];
        if (wc) {   // k_wcol: + the Z draw of the W tiles' rows
            KTimer t(h, DCFM_K_WPASS, s);
            h->wc_ops += 1;
            launch_wcol(d, b, dr, it, true, delta_pending, true, h->wc_ops, s, lamgen);
        } else if (fused) {   // several ranks: k_wcol (W pass + Z draw, no X factorisation), k_xred
                              // (the local X message), then ONE all-gather of [column sums of it - 1
                              // | local A sum | X message]; k_xdraw factors Xprec from the ranks' A
                              // sums, runs the delta chain of it - 1 and draws X
            {
                KTimer t(h, DCFM_K_WPASS, s);
                h->wc_ops += 1;
                launch_wcol(d, b, dr, it, true, delta_pending, true, h->wc_ops, s, lamgen);
            }
            { KTimer t(h, DCFM_K_XRED, s); launch_xred(d, b, s); }
            KTimer t(h, DCFM_K_COMM, s);
            if (int rc = coll_allgather(h, CH_MAIN, b.sloc, b.msg_all, (size_t)d.xstride, s)) return rc;
        } else {
            // side stream: A_m, R_m, Rx from this iteration's incoming Lambda, omega (dc:98-100,112-118)
            HIPC(h, hipStreamWaitEvent(ss, h->e_lam, 0));
            { KTimer t(h, DCFM_K_PREP, ss); launch_prep(d, b, ss); }
            HIPC(h, hipEventRecord(h->e_prep, ss));
            { KTimer t(h, DCFM_K_XCHOL, ss); launch_asum(d, b, ss); }
            if (d.coll) {
                KTimer t(h, DCFM_K_COMM, ss);
                if (int rc = coll_allgather(h, CH_SIDE, b.xa, b.xa_all, KW * KW, ss)) return rc;
            }
            { KTimer t(h, DCFM_K_XCHOL, ss); launch_xchol(d, b, ss); }
            HIPC(h, hipEventRecord(h->e_xchol, ss));
            // main stream
            { KTimer t(h, DCFM_K_WPASS, s);  launch_wpass(d, b, s); }
            HIPC(h, hipStreamWaitEvent(s, h->e_prep, 0));
            { KTimer t(h, DCFM_K_ZDRAW, s);  launch_zdraw(d, b, dr, it, s); }
            { KTimer t(h, DCFM_K_XRED, s);   launch_xred(d, b, s); }
            if (d.coll) {
                KTimer t(h, DCFM_K_COMM, s);
                if (int rc = coll_allgather(h, CH_MAIN, b.xin, b.xall, (size_t)d.NP * KW, s)) return rc;
            }
            HIPC(h, hipStreamWaitEvent(s, h->e_xchol, 0));
        }
        if (fused && d.coll) {   // several ranks: + the X factorisation
            KTimer t(h, DCFM_K_XDRAW, s);
            h->xm_ops += 1;
            launch_xdraw_mr(d, b, dr, it, h->xm_ops, s);
        } else {
            KTimer t(h, DCFM_K_XDRAW, s);
            launch_xdraw(d, b, dr, it, s, wc);
        }
        if (fused) {   // k_cpass + the delta chain of it - 1 (column sums from k_wcol / the gather)
            {
                KTimer t(h, DCFM_K_CPASS, s);
                if (delta_pending)
                    launch_cpass(d, b, s, dr, b.delta + h->cur * nkg, b.tau + h->cur * nkg,
                                 b.delta + (1 - h->cur) * nkg, b.tau + (1 - h->cur) * nkg, it - 1);
                else
                    launch_cpass(d, b, s);
            }
            HIPC(h, hipGetLastError());
            if (delta_pending) after_delta();   // outside the timer: it may launch k_trace_part
            delta_pending = false;
        } else {
            KTimer t(h, DCFM_K_CPASS, s);
            launch_cpass(d, b, s);
        }
        {
            KTimer t(h, DCFM_K_LAMBDA, s);
            // exact residual: k_resid redoes every row below (the guard need not fire)
            const bool exact = h->cfg.flags & DCFM_FLAG_EXACT_RESIDUAL;
            const double kmax = (h->cfg.flags & DCFM_FLAG_GUARD_ALL) ? 0.0 : KAPPA_IDENTITY_MAX;
            launch_lambda(d, b, dr, it, b.tau + h->cur * nkg, h->plam_valid ? b.Plam : nullptr, s, lamgen,
                          exact ? HUGE_VAL : kmax);
        }
        if (h->cfg.flags & DCFM_FLAG_EXACT_RESIDUAL) {   // dc:169's residual for every loading row
            KTimer t(h, DCFM_K_RESID, s);
            launch_resid(d, b, dr, it, s, lamgen);
        } else if (d.kp != KP) {                          // K > 32: the tiles k_lambda_w's guard flagged
            KTimer t(h, DCFM_K_RESID, s);
            launch_resid_flagged(d, b, dr, it, s);
        }
        h->plam_valid = false;
        if (fused) {
            delta_pending = true;     // column sums + delta chain ride in the next iteration's launches
        } else {
            HIPC(h, hipEventRecord(h->e_lam, s));
            { KTimer t(h, DCFM_K_COLSUM, s); launch_colsum(d, b, s); }
            if (d.coll) {
                KTimer t(h, DCFM_K_COMM, s);
                if (int rc = coll_allgather(h, CH_MAIN, b.sloc, b.sall, (size_t)d.G * KW, s)) return rc;
            }
            {
                KTimer t(h, DCFM_K_DELTA, s);
                launch_delta(d, b, dr, it, b.delta + h->cur * nkg, b.tau + h->cur * nkg,
                             b.delta + (1 - h->cur) * nkg, b.tau + (1 - h->cur) * nkg, s);
            }
        }
        if (gen_draws && it == batch0 + batch_n - 1) {      // the batch's last consumer is queued
            HIPC(h, hipEventRecord(h->e_used[slot], s));
            h->used_pending[slot] = true;
        }
        if (!fused) {
            h->cur ^= 1;
            if (h->trace_n < h->trace_cap) {                              // dcfm_set_trace
                launch_trace(d, b, b.tau + h->cur * nkg, h->trace, trace_row(h, h->trace_n), s);
                h->trace_n += 1;
            }
        }
        HIPC(h, hipGetLastError());
        if (it % h->cfg.thin == 0 && it > h->cfg.burnin) {                // dc:180
            if (h->batch == 0 && h->asm_pending[h->lb]) {                 // buffer still being assembled
                HIPC(h, hipStreamWaitEvent(s, h->e_free[h->lb], 0));
                h->asm_pending[h->lb] = false;
            }
            { KTimer t(h, DCFM_K_SAVE, s); launch_save(d, b, b.Lb[h->lb], b.wsum[h->lb], h->batch, s); }
            HIPC(h, hipGetLastError());
            h->batch += 1;
            h->saved += 1;
            if (h->batch == h->B) {
                int rc = flush_batch(h);
                if (rc) return rc;
            }
        }
    }
    if (delta_pending) {   // the last iteration's column sums (+ their gather) and delta chain
        KTimer t(h, DCFM_K_DELTA, s);
        launch_wcol(d, b, h->dr, end_iter - 1, false, true, false, 0, s);
        if (d.coll)
            if (int rc = coll_allgather(h, CH_MAIN, b.sloc, b.msg_all, (size_t)d.xstride, s)) return rc;
        const DrawsDev &dr = d.inject ? h->dr : h->gen[0];   // gammas drawn in place unless injected
        launch_delta(d, b, dr, end_iter - 1, b.delta + h->cur * nkg, b.tau + h->cur * nkg,
                     b.delta + (1 - h->cur) * nkg, b.tau + (1 - h->cur) * nkg, s);
        HIPC(h, hipGetLastError());
        after_delta();
    }
    int rc = flush_batch(h);
    if (rc) return rc;
    launch_finite(d, b, b.tau + h->cur * nkg, h->nan_dev, s);   // sentinel, read at the next sync point
    HIPC(h, hipGetLastError());
    HIPC(h, hipMemcpyAsync(h->nan_host, h->nan_dev, sizeof(int), hipMemcpyDeviceToHost, s));
    if (h->prof) collect_prof(h);
    return DCFM_OK;
}

int dcfm_set_trace(dcfm_handle *h, int64_t capacity) {
    if (!h || capacity < 0) return fail(h, DCFM_ERR_INVALID, "set_trace: bad argument");
    HIPC(h, hipSetDevice(h->cfg.device));
    HIPC(h, hipStreamSynchronize(h->stream));
    if (h->trace) (void)hipFree(h->trace);
    h->trace = nullptr;
    h->trace_cap = h->trace_n = 0;
    if (capacity == 0) return DCFM_OK;
    const size_t nd = trace_scratch_doubles(h->d.G) + (size_t)capacity * h->d.G * 4;
    if (hipMalloc(&h->trace, nd * sizeof(double)) != hipSuccess)
        return fail(h, DCFM_ERR_ALLOC, "set_trace: %lld rows", (long long)capacity);
    HIPC(h, hipMemset(h->trace, 0, trace_scratch_doubles(h->d.G) * sizeof(double)));   // tickets start at 0
    h->trace_cap = capacity;
    return DCFM_OK;
}

int dcfm_get_trace(dcfm_handle *h, double *out, int64_t *count) {
    if (!h || !count) return fail(h, DCFM_ERR_INVALID, "get_trace: null argument");
    HIPC(h, hipSetDevice(h->cfg.device));
    HIPC(h, hipStreamSynchronize(h->stream));
    *count = h->trace_n;
    if (out && h->trace_n) {
        const int G = h->d.G;
        std::vector<double> rows((size_t)h->trace_n * G * 4);
        HIPC(h, hipMemcpy(rows.data(), trace_row(h, 0), rows.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int64_t t = 0; t < h->trace_n; ++t)
            for (int q = 0; q < 4; ++q) {
                double acc = 0.0;
                for (int m = 0; m < G; ++m) acc += rows[((size_t)t * G + m) * 4 + q];   // shard order
                out[t * 4 + q] = acc;
            }
    }
    return DCFM_OK;
}

int dcfm_synchronize(dcfm_handle *h) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    HIPC(h, hipSetDevice(h->cfg.device));
    HIPC(h, hipStreamSynchronize(h->stream));
    HIPC(h, hipStreamSynchronize(h->side));
    HIPC(h, hipStreamSynchronize(h->sdraw));
    HIPC(h, hipStreamSynchronize(h->sasm));
    return numeric_status(h);
}

int64_t dcfm_saved_samples(const dcfm_handle *h) { return h ? h->saved : -1; }

int dcfm_get_sigma_cols(dcfm_handle *h, int64_t col0, int64_t ncols, double *out) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    Dims &d = h->d;
    const int root = 0;
    int code = DCFM_OK;
    if (!out && d.rank == root) code = fail(h, DCFM_ERR_INVALID, "null output on the root rank");
    else if (col0 < 0 || ncols < 0 || col0 + ncols > d.p)
        code = fail(h, DCFM_ERR_INVALID, "columns [%lld, %lld) outside 0..p = %d", (long long)col0,
                    (long long)(col0 + ncols), d.p);
    // every failure before the gather -- arguments, device, state, scratch allocation -- is folded
    // into `code` and agreed on: every rank enters the gather, or none (no rank left blocked in it)
    if (code == DCFM_OK) {
        const hipError_t e = hipSetDevice(h->cfg.device);
        if (e != hipSuccess) code = fail(h, DCFM_ERR_HIP, "get_sigma_cols: %s", hipGetErrorString(e));
    }
    sync_all(h);
    if (code == DCFM_OK) code = numeric_status(h);
    const int nr = d.nranks;
    const long long p = d.p, c0 = col0, c1 = col0 + ncols;
    // every rank's packed-window count for this stripe (known to all ranks: no size exchange)
    std::vector<long long> cnt(nr), base(nr);
    long long tot = 0;
    const bool is_root = d.rank == root;
    void *q = nullptr;
    if (code == DCFM_OK && ncols > 0) {
        for (int k = 0; k < nr; ++k) {
            const long long R0 = std::min<long long>(p, (long long)h->Tb[k] * ASM_TILE);
            const long long R1 = std::min<long long>(p, (long long)h->Tb[k + 1] * ASM_TILE);
            cnt[k] = win_off(c1, c0, R0, R1);
            base[k] = tot;
            tot += cnt[k];
        }
        if (tot != p * ncols) code = fail(h, DCFM_ERR_INVALID, "sigma_cols: windows cover %lld of %lld", tot, p * ncols);
    }
    if (code == DCFM_OK && ncols > 0) {
        // root: [recv (all ranks' windows, own part packed in place) | dense stripe]; others: own windows
        const size_t ndev = is_root ? (nr > 1 ? 2 * (size_t)tot : (size_t)tot) : (size_t)std::max<long long>(cnt[d.rank], 1);
        const hipError_t e = hipMalloc(&q, ndev * sizeof(double));
        if (e != hipSuccess) {
            q = nullptr;
            code = fail(h, DCFM_ERR_ALLOC, "get_sigma_cols: %zu doubles of scratch: %s", ndev, hipGetErrorString(e));
        }
    }
    if (int rc = agree(h, code)) {
        if (q) (void)hipFree(q);
        return rc;
    }
    if (ncols == 0) return DCFM_OK;
    double *buf = static_cast<double *>(q);
    double *mine = is_root ? buf + base[d.rank] : buf;
    int rc = DCFM_OK;
    launch_sigma_pack(h->b.Sigma, d.p, h->b.T0, h->b.T1, (int)col0, (int)ncols, mine, h->stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) rc = fail(h, DCFM_ERR_HIP, "sigma_pack: %s", hipGetErrorString(e));
    double *dense = buf;   // one rank: its windows are the dense stripe
    if (rc == DCFM_OK && nr > 1) {
        rc = coll_gather(h, mine, buf, base, cnt, root, h->stream);
        if (rc == DCFM_OK && is_root) {
            dense = buf + tot;
            void *qt = nullptr;
            e = hipMalloc(&qt, (size_t)nr * sizeof(long long) + (size_t)(nr + 1) * sizeof(int));
            if (e == hipSuccess) {
                long long *dbase = static_cast<long long *>(qt);
                int *dTb = reinterpret_cast<int *>(dbase + nr);
                e = hipMemcpyAsync(dbase, base.data(), nr * sizeof(long long), hipMemcpyHostToDevice, h->stream);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(dTb, h->Tb.data(), (nr + 1) * sizeof(int), hipMemcpyHostToDevice, h->stream);
                if (e == hipSuccess) {
                    launch_sigma_unpack(buf, d.p, (int)col0, (int)ncols, dTb, dbase, nr, dense, h->stream);
                    e = hipGetLastError();
                }
                if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
                (void)hipFree(qt);
            }
            if (e != hipSuccess) rc = fail(h, DCFM_ERR_HIP, "sigma_unpack: %s", hipGetErrorString(e));
        }
    }
    if (rc == DCFM_OK && is_root) {
        e = hipMemcpyAsync(out, dense, (size_t)tot * sizeof(double), hipMemcpyDeviceToHost, h->stream);
        if (e != hipSuccess) rc = fail(h, DCFM_ERR_HIP, "get_sigma_cols: %s", hipGetErrorString(e));
    }
    if (rc == DCFM_OK) {
        e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) rc = fail(h, DCFM_ERR_HIP, "get_sigma_cols: %s", hipGetErrorString(e));
    }
    (void)hipFree(buf);
    return rc;
}

int dcfm_sigma_block(const dcfm_handle *h, int64_t out[3]) {
    if (!h || !out) return fail(nullptr, DCFM_ERR_INVALID, "null argument");
    const int64_t p = h->d.p;
    out[0] = std::min<int64_t>(p, (int64_t)h->b.T0 * ASM_TILE);
    out[1] = std::min<int64_t>(p, (int64_t)h->b.T1 * ASM_TILE);
    out[2] = (int64_t)(tri(h->b.T1) - tri(h->b.T0)) * ASM_TILE * ASM_TILE * (int64_t)sizeof(double);
    return DCFM_OK;
}

int dcfm_get_sigma(dcfm_handle *h, double *out) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    if (!out && h->d.rank == 0) return fail(h, DCFM_ERR_INVALID, "null output on the root rank");
    const int64_t p = h->d.p;
    const int64_t chunk = std::max<int64_t>(32, std::min<int64_t>(p, ((int64_t)1 << 28) / p));   // <= 2 GiB stripes
    for (int64_t c = 0; c < p; c += chunk) {
        const int rc = dcfm_get_sigma_cols(h, c, std::min(chunk, p - c), out ? out + (size_t)c * p : nullptr);
        if (rc) return rc;
    }
    return DCFM_OK;
}

// ---------------------------------------------------------------------------
// Error of Sigmaout against a truth U U' + diag(s) (north_star
// check 2), without Sigmaout leaving the device.  Frobenius norms come from the first
// pass of k_sigma_err; the operator norm of M = Sigmaout - Sigma0 is the largest
// |eigenvalue| of the Lanczos tridiagonal T_m (symmetric M; full reorthogonalisation,
// twice, on the host: p x m doubles), found by Sturm-sequence bisection.
// ---------------------------------------------------------------------------
static int sturm_below(const std::vector<double> &a, const std::vector<double> &b, double x) {
    int cnt = 0;
    double q = 1.0;
    for (size_t i = 0; i < a.size(); ++i) {
        q = a[i] - x - (i ? b[i - 1] * b[i - 1] / q : 0.0);
        if (q == 0.0) q = -1e-300;
        if (q < 0.0) ++cnt;
    }
    return cnt;
}
static double tridiag_extreme(const std::vector<double> &a, const std::vector<double> &b, bool largest) {
    const size_t m = a.size();
    double lo = 0.0, hi = 0.0;
    for (size_t i = 0; i < m; ++i) {   // Gershgorin interval
        const double rad = (i ? std::fabs(b[i - 1]) : 0.0) + (i + 1 < m ? std::fabs(b[i]) : 0.0);
        lo = i ? std::min(lo, a[i] - rad) : a[i] - rad;
        hi = i ? std::max(hi, a[i] + rad) : a[i] + rad;
    }
    for (int it = 0; it < 200 && hi - lo > 0.0; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        const int c = sturm_below(a, b, mid);
        if (largest ? (c == (int)m) : (c >= 1)) hi = mid;
        else lo = mid;
    }
    return 0.5 * (lo + hi);
}
static uint64_t splitmix64(uint64_t &x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int dcfm_sigma_error(dcfm_handle *h, const double *U, int32_t r, const double *sdiag, int32_t iters,
                     uint64_t seed, double out[3]) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    int code = DCFM_OK;
    if (!sdiag || !out || (r > 0 && !U)) code = fail(h, DCFM_ERR_INVALID, "null argument");
    else if (r < 0 || r > 32) code = fail(h, DCFM_ERR_INVALID, "truth rank r = %d outside 0..32", r);
    else if (iters < 0) code = fail(h, DCFM_ERR_INVALID, "iters = %d < 0", iters);
    if (code == DCFM_OK) {
        const hipError_t e = hipSetDevice(h->cfg.device);
        if (e != hipSuccess) code = fail(h, DCFM_ERR_HIP, "sigma_error: %s", hipGetErrorString(e));
    }
    sync_all(h);
    if (code == DCFM_OK) code = numeric_status(h);
    const Dims &d = h->d;
    const int p = d.p;
    const size_t P = (size_t)p;
    const int m = std::min<int>(iters, p);
    double *dev = nullptr;
    const size_t ns = (size_t)sigma_err_splits(p);
    if (code == DCFM_OK) {   // scratch before agree(): an allocation failure fails the call on every rank
        void *q = nullptr;
        const size_t nd = P * (size_t)std::max(r, 1) + 5 * P + 3 * ns * P;
        const hipError_t e = hipMalloc(&q, nd * sizeof(double));
        if (e != hipSuccess) code = fail(h, DCFM_ERR_ALLOC, "sigma_error: %zu doubles of scratch: %s", nd, hipGetErrorString(e));
        else dev = static_cast<double *>(q);
    }
    if (int rc = agree(h, code)) {   // the all-reduces below run on every rank, or on none
        if (dev) (void)hipFree(dev);
        return rc;
    }
    // U, s, v, then the summed outputs y | fro | tru (contiguous), then the split partials
    double *dU = dev, *ds = dU + P * std::max(r, 1), *dv = ds + P, *dy = dv + P, *dfro = dy + P, *dtru = dfro + P;
    double *py = dtru + P, *pfro = py + ns * P, *ptru = pfro + ns * P;
    int rc = DCFM_OK;
    auto hip_ok = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == DCFM_OK) rc = fail(h, DCFM_ERR_HIP, "sigma_error %s: %s", what, hipGetErrorString(e));
        return rc == DCFM_OK;
    };
    if (r > 0) hip_ok(hipMemcpy(dU, U, P * r * sizeof(double), hipMemcpyHostToDevice), "upload U");
    hip_ok(hipMemcpy(ds, sdiag, P * sizeof(double), hipMemcpyHostToDevice), "upload s");
    std::vector<double> V, y(P), fro(P), tru(P), alpha, beta;
    // one pass: y = M v (v may be null: norms only); collective over ranks
    auto pass = [&](const double *vh, bool first) {
        if (rc) return false;
        if (vh && !hip_ok(hipMemcpyAsync(dv, vh, P * sizeof(double), hipMemcpyHostToDevice, h->stream), "upload v"))
            return false;
        launch_sigma_err(h->b.Sigma, p, dU, r, ds, vh ? dv : nullptr, h->b.T0, h->b.T1, first, vh ? py : nullptr,
                         pfro, ptru, dy, h->stream);
        if (!hip_ok(hipGetLastError(), "launch")) return false;
        if (d.coll) {
            if (vh && (rc = coll_allreduce_sum(h, CH_ASM, dy, P, h->stream))) return false;
            if (first && (rc = coll_allreduce_sum(h, CH_ASM, dfro, P, h->stream))) return false;
            if (first && (rc = coll_allreduce_sum(h, CH_ASM, dtru, P, h->stream))) return false;
        }
        if (vh) hip_ok(hipMemcpyAsync(y.data(), dy, P * sizeof(double), hipMemcpyDeviceToHost, h->stream), "y");
        if (first) {
            hip_ok(hipMemcpyAsync(fro.data(), dfro, P * sizeof(double), hipMemcpyDeviceToHost, h->stream), "fro");
            hip_ok(hipMemcpyAsync(tru.data(), dtru, P * sizeof(double), hipMemcpyDeviceToHost, h->stream), "tru");
        }
        return hip_ok(hipStreamSynchronize(h->stream), "sync");
    };
    auto dot = [&](const double *a, const double *b) {
        double acc = 0.0;
        for (size_t i = 0; i < P; ++i) acc += a[i] * b[i];
        return acc;
    };
    if (m == 0) {
        pass(nullptr, true);
    } else {
        V.assign(P * (size_t)(m + 1), 0.0);
        uint64_t st = seed ^ 0x5DEECE66Dull;
        for (size_t i = 0; i < P; i += 2) {   // Box-Muller normals: a rotation-invariant start
            const double u1 = ((splitmix64(st) >> 11) + 1.0) * 0x1.0p-53, u2 = (splitmix64(st) >> 11) * 0x1.0p-53;
            const double rr = std::sqrt(-2.0 * std::log(u1));
            V[i] = rr * std::cos(6.283185307179586 * u2);
            if (i + 1 < P) V[i + 1] = rr * std::sin(6.283185307179586 * u2);
        }
        const double n0 = std::sqrt(dot(V.data(), V.data()));
        for (size_t i = 0; i < P; ++i) V[i] /= n0;
        double bprev = 0.0;
        for (int j = 0; j < m; ++j) {
            double *vj = V.data() + P * j, *vn = V.data() + P * (j + 1);
            if (!pass(vj, j == 0)) break;
            const double a = dot(y.data(), vj);
            const double *vp = j ? vj - P : vj;
            const double bp = j ? bprev : 0.0;
            for (size_t i = 0; i < P; ++i) vn[i] = y[i] - a * vj[i] - bp * vp[i];
            for (int rep = 0; rep < 2; ++rep)
                for (int i2 = 0; i2 <= j; ++i2) {
                    const double *vi = V.data() + P * i2;
                    const double c = dot(vn, vi);
                    for (size_t i = 0; i < P; ++i) vn[i] -= c * vi[i];
                }
            const double bn = std::sqrt(dot(vn, vn));
            alpha.push_back(a);
            double scale = std::fabs(a);
            for (double x : alpha) scale = std::max(scale, std::fabs(x));
            if (bn <= 1e-13 * std::max(scale, 1e-300)) break;   // invariant subspace: T is exact
            beta.push_back(bn);
            for (size_t i = 0; i < P; ++i) vn[i] /= bn;
            bprev = bn;
        }
    }
    if (rc == DCFM_OK) {
        double fs = 0.0, ts = 0.0;
        for (size_t i = 0; i < P; ++i) {
            fs += fro[i];
            ts += tru[i];
        }
        out[0] = std::sqrt(fs);
        out[1] = std::sqrt(ts);
        out[2] = 0.0;
        if (!alpha.empty()) {
            beta.resize(alpha.size() - 1);
            out[2] = std::max(std::fabs(tridiag_extreme(alpha, beta, true)),
                              std::fabs(tridiag_extreme(alpha, beta, false)));
        }
    }
    (void)hipFree(dev);
    return rc;
}

int dcfm_set_profiling(dcfm_handle *h, int enable) {
    return dcfm_set_profiling_mask(h, enable ? 0xFFFFFFFFu : 0u);
}

int dcfm_set_profiling_mask(dcfm_handle *h, uint32_t mask) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    collect_prof(h);
    h->prof_mask = mask;
    h->prof_stride = 1;
    std::fill(h->prof_seq, h->prof_seq + DCFM_K_COUNT, (int64_t)0);
    const bool enable = mask != 0;
    h->prof = enable;
    if (enable) {
        std::fill(h->kms, h->kms + DCFM_K_COUNT, 0.0);
        std::fill(h->kcnt, h->kcnt + DCFM_K_COUNT, 0);
    }
    return DCFM_OK;
}

int dcfm_set_profiling_stride(dcfm_handle *h, int32_t stride) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    if (stride < 1) return fail(h, DCFM_ERR_INVALID, "profiling stride %d < 1", (int)stride);
    h->prof_stride = stride;
    std::fill(h->prof_seq, h->prof_seq + DCFM_K_COUNT, (int64_t)0);
    return DCFM_OK;
}

int dcfm_get_kernel_stats(dcfm_handle *h, double ms[DCFM_K_COUNT], int64_t launches[DCFM_K_COUNT]) {
    if (!h) return fail(h, DCFM_ERR_INVALID, "null handle");
    collect_prof(h);
    for (int k = 0; k < DCFM_K_COUNT; ++k) {
        if (ms) ms[k] = h->kms[k];
        if (launches) launches[k] = h->kcnt[k];
    }
    return DCFM_OK;
}

int dcfm_rng_fill(int device, uint64_t seed, int kind, double shape, int32_t site, int32_t shard,
                  int64_t iter, int64_t count, double *out) {
    if (count < 0) return fail(nullptr, DCFM_ERR_INVALID, "rng_fill: bad argument");
    return dcfm_rng_fill_rows(device, seed, kind, shape, site, shard, iter, (count + 31) / 32, 32, count, out);
}

int dcfm_rng_fill_rows(int device, uint64_t seed, int kind, double shape, int32_t site, int32_t shard,
                       int64_t iter, int64_t rows, int32_t width, int64_t count, double *out) {
    if (!out || count < 0 || rows < 0 || width < 1 || width > (1 << 23) || count > rows * (int64_t)width ||
        (kind != 0 && kind != 1) || (kind == 1 && !(shape > 0.0)))
        return fail(nullptr, DCFM_ERR_INVALID, "rng_fill: bad argument");
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail(nullptr, DCFM_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e));
    void *q = nullptr;
    e = hipMalloc(&q, std::max<int64_t>(count, 1) * sizeof(double));
    if (e != hipSuccess) return fail(nullptr, DCFM_ERR_ALLOC, "hipMalloc: %s", hipGetErrorString(e));
    launch_rng_fill(seed, kind, shape, site, shard, iter, count, width, static_cast<double *>(q), nullptr);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, q, count * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(q);
    if (e != hipSuccess) return fail(nullptr, DCFM_ERR_HIP, "rng_fill: %s", hipGetErrorString(e));
    return DCFM_OK;
}

}  // extern "C"
