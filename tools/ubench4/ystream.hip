// Dev microbenchmark (not product): how fast can the c3 Y array (64 x 1024 x 320 fp64, 168 MB)
// be streamed on one MI355X with the access patterns of the two Y passes, against a plain
// contiguous read?  Each kernel sums what it reads (one store per wave, so nothing is dead code).
//   flat     : grid-stride, 16 B per lane, consecutive lanes consecutive addresses
//   cpass    : k_cpass's map — block = (shard, 32-column tile), 4 waves split the 1024 rows,
//              lane (r, q) reads Y[4s + q][c0 + 2r .. +1], 2 batches of 4 rows in flight
//   wpass    : the W pass's map — wave = 32 rows of a shard, lane (r, q) reads rows r, r + 16 at
//              columns 8t + 2q .. +1, a ring of 4 chunks in flight
//   rowslab  : block = (shard, 64 rows), each wave streams whole 2,560-B rows (a row per 160 lanes)
// Build: hipcc -O3 --offload-arch=gfx950 ystream.hip -o ystream     Run: ./ystream [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct d2 { double x, y; };
constexpr int G = 64, NP = 1024, PP = 320;

__global__ __launch_bounds__(256) void k_flat(const double *__restrict__ Y, size_t n2, double *out) {
    const d2 *p = reinterpret_cast<const d2 *>(Y);
    double s = 0.0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        const d2 v = p[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_cpass_pat(const double *__restrict__ Y, double *out) {
    const int nt = PP / 32;
    const int m = blockIdx.x / nt, tile = blockIdx.x % nt;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    const double *Yp = Y + (size_t)m * NP * PP + tile * 32 + 2 * r;
    const int s0 = wave * (NP / 16), nsw = NP / 16;
    double acc = 0.0;
    d2 a[4], b[4];
    auto load = [&](int s, d2 (&v)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const d2 *>(Yp + (size_t)(4 * (s + u) + q) * PP);
    };
    load(s0, a);
    for (int bb = 0; bb < nsw / 4; bb += 2) {
        if (bb + 1 < nsw / 4) load(s0 + 4 * (bb + 1), b);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += a[u].x * a[u].y;
        if (bb + 2 < nsw / 4) load(s0 + 4 * (bb + 2), a);
        if (bb + 1 < nsw / 4)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += b[u].x * b[u].y;
    }
    if (acc == 12345.678) out[blockIdx.x] = acc;
}

template <int RING>
__global__ __launch_bounds__(256) void k_wpass_pat(const double *__restrict__ Y, double *out) {
    const int nrb = NP / 128;
    const int m = blockIdx.x / nrb, rb = blockIdx.x % nrb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    const int i0 = rb * 128 + wave * 32;
    const double *Y0 = Y + ((size_t)m * NP + i0 + r) * PP + 2 * q, *Y1 = Y0 + 16 * PP;
    double acc = 0.0;
    d2 v0[RING], v1[RING];
#pragma unroll
    for (int k = 0; k < RING - 1; ++k) { v0[k] = *reinterpret_cast<const d2 *>(Y0 + 8 * k); v1[k] = *reinterpret_cast<const d2 *>(Y1 + 8 * k); }
    for (int t = 0; t < PP / 8; t += RING) {
#pragma unroll
        for (int k = 0; k < RING; ++k) {
            const int tn = t + k + RING - 1;
            if (tn < PP / 8) {
                v0[(k + RING - 1) % RING] = *reinterpret_cast<const d2 *>(Y0 + 8 * tn);
                v1[(k + RING - 1) % RING] = *reinterpret_cast<const d2 *>(Y1 + 8 * tn);
            }
            acc += v0[k].x * v1[k].y + v0[k].y * v1[k].x;
        }
    }
    if (acc == 12345.678) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_rowslab(const double *__restrict__ Y, double *out) {
    // block = 64 rows of one shard (64 x 2,560 B = 160 KB contiguous); thread t reads 16-B pieces
    // t, t + 256, ... of that contiguous range
    const d2 *p = reinterpret_cast<const d2 *>(Y + (size_t)blockIdx.x * 64 * PP);
    constexpr int N2 = 64 * PP / 2;
    double acc = 0.0;
    d2 v[8];
    for (int i = threadIdx.x; i < N2; i += 256 * 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (i + 256 * k < N2) ? p[i + 256 * k] : d2{0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k].x * v[k].y;
    }
    if (acc == 12345.678) out[blockIdx.x] = acc;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const size_t n = (size_t)G * NP * PP;
    double *Y, *out;
    CK(hipMalloc(&Y, n * 8));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(Y, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto &&launch) {
        for (int w = 0; w < 5; ++w) launch();
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1000.0 * ms / reps;
        printf("%-22s %8.2f us  %7.0f GB/s\n", name, us, n * 8 / (us * 1e-6) / 1e9);
    };
    for (int nb : {1024, 2048, 4096, 8192})
        run(nb == 1024 ? "flat 1024 blocks" : nb == 2048 ? "flat 2048 blocks" : nb == 4096 ? "flat 4096 blocks" : "flat 8192 blocks",
            [&] { hipLaunchKernelGGL(k_flat, dim3(nb), dim3(256), 0, nullptr, Y, n / 2, out); });
    run("cpass pattern", [&] { hipLaunchKernelGGL(k_cpass_pat, dim3(G * PP / 32), dim3(256), 0, nullptr, Y, out); });
    run("wpass pattern ring4", [&] { hipLaunchKernelGGL(k_wpass_pat<4>, dim3(G * NP / 128), dim3(256), 0, nullptr, Y, out); });
    run("wpass pattern ring8", [&] { hipLaunchKernelGGL(k_wpass_pat<8>, dim3(G * NP / 128), dim3(256), 0, nullptr, Y, out); });
    run("row slabs", [&] { hipLaunchKernelGGL(k_rowslab, dim3(G * NP / 64), dim3(256), 0, nullptr, Y, out); });
    return 0;
}
