"""Dev instrumentation (never shipped): per-phase shader-clock totals of k_lambda_t, summed
over blocks by thread 0 (global atomics), read back with dcfm_debug_phases (tools/ltphase.py).
Phases: 0 loads+Q build, 1 first diagonal factor, 2 panel, 3 trailing (+ look-ahead factor),
4 back solve, 5 epilogue; 6 = time inside diag_factor (owner wave, every call)."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels_wide.hip"
s = p.read_text()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old, s.count(old))
    s = s.replace(old, new)
rep("""#ifndef DCFM_LT_MINW""", """__device__ unsigned long long g_phase[64][8];
#define PH_MARK(i) do { __builtin_amdgcn_s_waitcnt(0); const unsigned long long _t = __builtin_amdgcn_s_memtime(); \\
    ph_acc[i] += _t - ph_t; ph_t = _t; } while (0)
#ifndef DCFM_LT_MINW""")
rep("""    const int K = d.K;
    constexpr int nb = NB, NT = NTM;""", """    const int K = d.K;
    unsigned long long ph_t = __builtin_amdgcn_s_memtime();
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
    constexpr int nb = NB, NT = NTM;""")
rep("""    auto diag_factor = [&](int J, int os) {      // whole owner wave: U_JJ, v_J; keeps U_JJ in acc
        double *U = Ud + (J & 1) * TZ;""", """    auto diag_factor = [&](int J, int os) {      // whole owner wave: U_JJ, v_J; keeps U_JJ in acc
        const unsigned long long df0 = __builtin_amdgcn_s_memtime();
        double *U = Ud + (J & 1) * TZ;""")
rep("""                for (int g = 0; g < 4; ++g) acc[sl][g] = U[(q + 4 * g) * LD + c16];   // U_JJ, C/D layout
            }
    };""", """                for (int g = 0; g < 4; ++g) acc[sl][g] = U[(q + 4 * g) * LD + c16];   // U_JJ, C/D layout
            }
        __builtin_amdgcn_s_waitcnt(0);
        ph_acc[6] += __builtin_amdgcn_s_memtime() - df0;
    };""")
rep("""    if (wave == 0) diag_factor(0, 0);               // tile (0, 0) is tile 0: wave 0, slot 0
    __syncthreads();""", """    PH_MARK(0);
    if (wave == 0) diag_factor(0, 0);               // tile (0, 0) is tile 0: wave 0, slot 0
    __syncthreads();
    PH_MARK(1);""")
rep("""            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        if (J + 1 < nb) {""", """            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        PH_MARK(2);
        if (J + 1 < nb) {""")
rep("""                __builtin_amdgcn_sched_barrier(0);   // one slot's operands live at a time
            }
        }
        __syncthreads();
    }""", """                __builtin_amdgcn_sched_barrier(0);   // one slot's operands live at a time
            }
        }
        __syncthreads();
        PH_MARK(3);
    }""")
rep("""    // ---- epilogue: Lambda_j, psi_j (dc:150), and SS_j""", """    PH_MARK(4);
    // ---- epilogue: Lambda_j, psi_j (dc:150), and SS_j""")
rep("""        omega[(size_t)m * d.PP + j] = 1.0 / psn;                 // dc:171 (Q1)
    }
}""", """        omega[(size_t)m * d.PP + j] = 1.0 / psn;                 // dc:171 (Q1)
    }
    PH_MARK(5);
    if (t == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(&g_phase[blockIdx.x & 63][i], ph_acc[i]);
    if (t == 0) atomicAdd(&g_phase[blockIdx.x & 63][7], __builtin_amdgcn_s_memrealtime() - rt0);
    if (lane == 0) atomicAdd(&g_phase[blockIdx.x & 63][6], ph_acc[6]);
}""")
s += """
extern "C" int dcfm_debug_phases(unsigned long long *out, int reset) {
    static unsigned long long z[64 * 8];
    if (reset) { for (int i = 0; i < 512; ++i) z[i] = 0; return hipMemcpyToSymbol(HIP_SYMBOL(dcfm::wide::g_phase), z, sizeof(z)) == hipSuccess ? 0 : 1; }
    if (hipMemcpyFromSymbol(z, HIP_SYMBOL(dcfm::wide::g_phase), sizeof(z)) != hipSuccess) return 1;
    for (int i = 0; i < 8; ++i) { out[i] = 0; for (int b = 0; b < 64; ++b) out[i] += z[b * 8 + i]; }
    return 0;
}
"""
p.write_text(s)
