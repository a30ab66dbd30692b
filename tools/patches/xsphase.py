"""Dev instrumentation (never shipped), applied after stamps.py: s_memrealtime marks of the
k_wcol shard-sum role (per chunk block) and of the last arrival's X factorisation, read back
with dcfm_debug_xs (tools/stamps.py prints them when present)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old, s.count(old))
    s = s.replace(old, new)
rep("""template <bool PUB = false>
__device__ __forceinline__ void xchol_factor(""", """__device__ unsigned long long g_xs[64][8];
template <bool PUB = false>
__device__ __forceinline__ void xchol_factor(""")
M = lambda k: f"if (threadIdx.x == 0 && j < 64) g_xs[j][{k}] = __builtin_amdgcn_s_memrealtime();"
rep("""            wait_count(chunk_ctr + j, ops_epoch * (unsigned long long)chunk);
            double vs[NU];""", f"""            {M(0)}
            wait_count(chunk_ctr + j, ops_epoch * (unsigned long long)chunk);
            {M(1)}
            double vs[NU];""")
rep("""                if (!last_arrival(b.ticket, (unsigned)nxs, smem)) return;
            }
            double xs[NU];""", f"""                {M(2)}
                if (!last_arrival(b.ticket, (unsigned)nxs, smem)) return;
            }}
            {M(3)}
            double xs[NU];""")
rep("""            for (int u = 0; u < NU; ++u) xprec_store(d, smem, t + 256 * u, xs[u]);
            __syncthreads();
            xchol_factor(d, b.XM, smem);              // Xprec""", f"""            for (int u = 0; u < NU; ++u) xprec_store(d, smem, t + 256 * u, xs[u]);
            __syncthreads();
            {M(4)}
            xchol_factor(d, b.XM, smem);
            {M(6)}
            __syncthreads();
            {M(7)}
            //""")
rep("""    if (wave == 0) {                       // Ux = Lx^{-1} = Rx^{-T}
        chol_inv32(Sm, Us, Wk, lds_l, lds_u, lane);
    }
    __syncthreads();""", """    if (wave == 0) {                       // Ux = Lx^{-1} = Rx^{-T}
        chol_inv32(Sm, Us, Wk, lds_l, lds_u, lane);
    }
    __syncthreads();
    if (!PUB && threadIdx.x == 0) g_xs[63][5] = __builtin_amdgcn_s_memrealtime();""")
rep("""extern "C" int dcfm_debug_stamps(""", """extern "C" int dcfm_debug_xs(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(dcfm::g_xs), sizeof(dcfm::g_xs)) == hipSuccess ? 0 : 1;
}
extern "C" int dcfm_debug_stamps(""")
open(f, "w").write(s)
