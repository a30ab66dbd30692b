// Dev harness (not product): times the loading-row kernel variants at a BASELINE shape on
// consistent synthetic inputs (E = eta'eta, C = Y'eta, yy = diag Y'Y per shard, so SS >= 0)
// and checks every variant against the library's k_lambda (gen = 1) on the same state.
// Build: see tools/lambench/build.sh.  Run: lambench [g P n K reps]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "linalg.h"
#include "lam_variants.h"

using namespace dcfm;

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); exit(1); } \
    } while (0)

static double *dnew(size_t n) {
    void *p = nullptr;
    CK(hipMalloc(&p, std::max<size_t>(n, 1) * 8));
    CK(hipMemset(p, 0, std::max<size_t>(n, 1) * 8));
    return (double *)p;
}
static void up(double *d, const std::vector<double> &h) { CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice)); }
static std::vector<double> down(const double *d, size_t n) {
    std::vector<double> h(n);
    CK(hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost));
    return h;
}

int main(int argc, char **argv) {
    const int g = argc > 1 ? atoi(argv[1]) : 64, P = argc > 2 ? atoi(argv[2]) : 312;
    const int n = argc > 3 ? atoi(argv[3]) : 1000, K = argc > 4 ? atoi(argv[4]) : 30;
    const int reps = argc > 5 ? atoi(argv[5]) : 50;
    Dims d{};
    d.n = n; d.P = P; d.g = g; d.K = K; d.G = g; d.nranks = 1; d.rank = 0; d.shard0 = 0;
    d.NP = (n + 127) / 128 * 128; d.PP = (P + 31) / 32 * 32; d.p = P * g; d.kp = KP;
    d.rho = 0.5; d.sr = std::sqrt(0.5); d.s1r = std::sqrt(0.5);
    d.as_ = 1; d.bs = 0.3; d.df = 3; d.ad1 = 2; d.bd1 = 1; d.ad2 = 2; d.bd2 = 1;
    d.seed = 12345; d.inject = 0; d.sgap = 0; d.xstride = KP * KP;
    const size_t G = g, PP = d.PP;
    std::mt19937_64 rng(7);
    std::normal_distribution<double> N01;
    std::uniform_real_distribution<double> U01(0.0, 1.0);
    std::vector<double> hE(G * KP * KP, 0.0), hC(G * PP * KP, 0.0), hyy(G * PP, 0.0);
    std::vector<double> eta((size_t)n * K), Y((size_t)n * P), Wt((size_t)K * P);
    for (size_t m = 0; m < G; ++m) {
        for (auto &x : eta) x = N01(rng);
        for (auto &x : Wt) x = U01(rng) < 0.7 ? 0.0 : N01(rng);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < P; ++j) {
                double s = 0.3 * N01(rng);
                for (int k = 0; k < 10 && k < K; ++k) s += eta[(size_t)i * K + k] * Wt[(size_t)k * P + j];
                Y[(size_t)i * P + j] = s;
            }
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b) {
                double s = 0;
                for (int i = 0; i < n; ++i) s += eta[(size_t)i * K + a] * eta[(size_t)i * K + b];
                hE[(m * KP + a) * KP + b] = s;
            }
        for (int j = 0; j < P; ++j) {
            double yyj = 0;
            for (int i = 0; i < n; ++i) yyj += Y[(size_t)i * P + j] * Y[(size_t)i * P + j];
            hyy[m * PP + j] = yyj;
            for (int k = 0; k < K; ++k) {
                double s = 0;
                for (int i = 0; i < n; ++i) s += Y[(size_t)i * P + j] * eta[(size_t)i * K + k];
                hC[(m * PP + j) * KP + k] = s;
            }
        }
    }
    std::vector<double> hpsi(G * PP * KP, 0.0), hps(G * PP, 0.0), htau((size_t)g * KP, 1.0);
    for (size_t m = 0; m < G; ++m)
        for (int j = 0; j < P; ++j) {
            hps[m * PP + j] = 0.5 + 2.0 * U01(rng);
            for (int k = 0; k < K; ++k) hpsi[(m * PP + j) * KP + k] = 0.2 + 2.0 * U01(rng);
        }
    for (int m = 0; m < g; ++m) {
        double t = 1.0;
        for (int k = 0; k < K; ++k) { t *= 0.8 + 1.5 * U01(rng); htau[(size_t)m * KP + k] = t; }
    }
    Bufs b{};
    b.C = dnew(hC.size()); up(b.C, hC);
    b.E = dnew(hE.size()); up(b.E, hE);
    b.yy = dnew(hyy.size()); up(b.yy, hyy);
    b.Lam = dnew(G * PP * KP); b.psi = dnew(G * PP * KP); b.ps = dnew(G * PP); b.omega = dnew(G * PP);
    b.cpart = dnew(G * PP * KP);
    double *tau = dnew(htau.size()); up(tau, htau);
    // one iteration of draws (k_draws layout [T = 1][g][P][K])
    DrawsDev dr{};
    dr.NZ = dnew((size_t)K * n * g); dr.NX = dnew((size_t)K * n); dr.NL = dnew((size_t)K * P * g);
    dr.Gpsi = dnew((size_t)K * P * g); dr.Gdelta = dnew((size_t)K * g); dr.Gps = dnew((size_t)P * g);
    const int64_t iter = 3;
    dr.first_iter = iter; dr.n_iter = 1;
    launch_draws(d, dr, iter, nullptr);
    CK(hipDeviceSynchronize());
    auto reset = [&]() { up(b.psi, hpsi); up(b.ps, hps); CK(hipMemset(b.Lam, 0, G * PP * KP * 8)); };
    auto outputs = [&]() {
        std::vector<std::vector<double>> o;
        o.push_back(down(b.Lam, G * PP * KP));
        o.push_back(down(b.psi, G * PP * KP));
        o.push_back(down(b.ps, G * PP));
        o.push_back(down(b.omega, G * PP));
        o.push_back(down(b.cpart, G * PP * KP));
        return o;
    };
    const char *names[5] = {"Lam", "psi", "ps", "omega", "cpart"};
    // reference: the library kernel, variates from the draw buffers
    reset();
    launch_lambda(d, b, dr, iter, tau, nullptr, nullptr, false);
    CK(hipDeviceSynchronize());
    auto ref = outputs();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto &&launch) {
        reset();
        launch();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        auto o = outputs();
        double worst = 0.0;
        for (int f = 0; f < 5; ++f) {
            double mx = 0.0, df = 0.0;
            for (size_t i = 0; i < o[f].size(); ++i) {
                mx = std::max(mx, std::fabs(ref[f][i]));
                df = std::max(df, std::fabs(o[f][i] - ref[f][i]));
            }
            const double rel = df / std::max(mx, 1e-300);
            worst = std::max(worst, rel);
            if (!(rel < 1e-11)) printf("   %s: field %s rel diff %.3e\n", name, names[f], rel);
        }
        reset();
        for (int w = 0; w < 5; ++w) launch();
        CK(hipEventRecord(e0, nullptr));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %9.2f us   max rel diff vs ref %.2e\n", name, 1000.0 * ms / reps, worst);
        fflush(stdout);
    };
    printf("shape g=%d P=%d n=%d K=%d (%d rows)\n", g, P, n, K, g * P);
    run("lib k_lambda", [&] { launch_lambda(d, b, dr, iter, tau, nullptr, nullptr, false); });
    run_variants(d, b, dr, iter, tau, run);
    return 0;
}
