"""Dev instrumentation (never shipped): per-phase shader-clock totals of k_lambda_w, kept in
registers and added once per block (lane 0), read back with dcfm_debug_phases (tools/ltphase.py).
Phases: 0 loads + Q build, 3 trailing (+ staging), 6 chol_inv16, 1 v / U reads, 2 panel,
4 back solve, 7 epilogue (5 = 0)."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels_wide.hip"
s = p.read_text()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old, s.count(old))
    s = s.replace(old, new)
rep("""template <int NB>
__host__ __device__ constexpr int utix""", """__device__ unsigned long long g_phase[64][8];
#define PH_MARK(i) do { __builtin_amdgcn_s_waitcnt(0); const unsigned long long _t = __builtin_amdgcn_s_memtime(); \\
    ph_acc[i] += _t - ph_t; ph_t = _t; } while (0)
template <int NB>
__host__ __device__ constexpr int utix""")
rep("""    const int lane = threadIdx.x, c16 = lane & 15, q = lane >> 4;
    const int K = d.K;
    const double *Em = E + (size_t)m * KW * KW;
    const size_t rowoff = ((size_t)m * d.PP + j) * KW;
    const double psj = ps[(size_t)m * d.PP + j];
    // ---- every load""", """    const int lane = threadIdx.x, c16 = lane & 15, q = lane >> 4;
    const int K = d.K;
    unsigned long long ph_t = __builtin_amdgcn_s_memtime();
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
    const double *Em = E + (size_t)m * KW * KW;
    const size_t rowoff = ((size_t)m * d.PP + j) * KW;
    const double psj = ps[(size_t)m * d.PP + j];
    // ---- every load""")
rep("""    // ---- blocked factorisation with the forward solve
    static_for<NB>([&](auto JC) {
        constexpr int J = decltype(JC)::value, tJ = utix<NB>(J, J);""", """    // ---- blocked factorisation with the forward solve
    PH_MARK(0);
    static_for<NB>([&](auto JC) {
        constexpr int J = decltype(JC)::value, tJ = utix<NB>(J, J);""")
rep("""        for (int g = 0; g < 4; ++g) Sd[(q + 4 * g) * LD + c16] = T[tJ][g];
        __syncthreads();""", """        for (int g = 0; g < 4; ++g) Sd[(q + 4 * g) * LD + c16] = T[tJ][g];
        __syncthreads();
        PH_MARK(3);""")
rep("""        chol_inv16_p<LD>(Sd, 0, Ud, lds_l, lds_u, lane);
        __syncthreads();""", """        chol_inv16_p<LD>(Sd, 0, Ud, lds_l, lds_u, lane);
        __syncthreads();
        PH_MARK(6);""")
rep("""            for (int g = 0; g < 4; ++g) vb[16 * J + q + 4 * g] = vj[g];        // v_J for the back solve
        }""", """            for (int g = 0; g < 4; ++g) vb[16 * J + q + 4 * g] = vj[g];        // v_J for the back solve
        }
        PH_MARK(1);""")
rep("""        static_for<NB>([&](auto KC) {                     // trailing T_{Kc,I} -= R_{J,Kc}' R_{J,I}""", """        PH_MARK(2);
        static_for<NB>([&](auto KC) {                     // trailing T_{Kc,I} -= R_{J,Kc}' R_{J,I}""")
rep("""    // ---- w = v + z (dc:142 normrnd), back solve R x = w (dc:144):
    //      x_J = U_JJ' (w_J - sum_{I>J} R_{J,I} x_I); lane (c16, .) holds x_I[c16] in xr[I]""", """    PH_MARK(3);
    PH_MARK(4);
    // ---- w = v + z (dc:142 normrnd), back solve R x = w (dc:144):
    //      x_J = U_JJ' (w_J - sum_{I>J} R_{J,I} x_I); lane (c16, .) holds x_I[c16] in xr[I]""")
rep("""    // ---- epilogue: Lambda_j, psi_j (dc:150), cpart (dc:156), SS_j (dc:169), ps_j, omega_j""", """    PH_MARK(7);
    // ---- epilogue: Lambda_j, psi_j (dc:150), cpart (dc:156), SS_j (dc:169), ps_j, omega_j""")
rep("""        omega[(size_t)m * d.PP + j] = 1.0 / psn;                 // dc:171 (Q1)
    }
}

""", """        omega[(size_t)m * d.PP + j] = 1.0 / psn;                 // dc:171 (Q1)
    }
    PH_MARK(5);
    if (lane == 0) {
        for (int i = 0; i < 8; ++i) atomicAdd(&g_phase[blockIdx.x & 63][i], ph_acc[i]);
    }
}

""")
s += """
extern "C" int dcfm_debug_phases(unsigned long long *out, int reset) {
    static unsigned long long z[64 * 8];
    if (reset) { for (int i = 0; i < 512; ++i) z[i] = 0; return hipMemcpyToSymbol(HIP_SYMBOL(dcfm::wide::g_phase), z, sizeof(z)) == hipSuccess ? 0 : 1; }
    if (hipMemcpyFromSymbol(z, HIP_SYMBOL(dcfm::wide::g_phase), sizeof(z)) != hipSuccess) return 1;
    for (int i = 0; i < 8; ++i) { out[i] = 0; for (int b = 0; b < 64; ++b) out[i] += z[b * 8 + i]; }
    return 0;
}
"""
rep("""    const double yyj = yy[(size_t)m * d.PP + j], Gps = dr.Gps[drow];   // dc:169-170
    d4 T[NT];""", """    const double yyj = yy[(size_t)m * d.PP + j], Gps = dr.Gps[drow];   // dc:169-170
    { double sink = zr[0] + Gr[0] + trr[0] + cr[0] + pr[0] + yyj + Gps + psj;
      asm volatile("" :: "v"(sink)); }
    PH_MARK(5);
    d4 T[NT];""")
p.write_text(s)
