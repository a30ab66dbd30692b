"""A/B: k_assemble's per-chunk barriers wait for LDS only (s_waitcnt lgkmcnt(0); s_barrier),
so the tile's old-Sigma loads stay in flight across the staging barrier."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels.hip"
s = p.read_text()
old = """    lstore(0);
    __syncthreads();
    for (int kc = 0, buf = 0; kc < kext; kc += AKC, buf ^= 1) {"""
assert s.count(old) == 1
s = s.replace(old, """    lstore(0);
    asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    for (int kc = 0, buf = 0; kc < kext; kc += AKC, buf ^= 1) {""")
old = """        if (more) lstore(buf ^ 1);
        __syncthreads();
    }"""
assert s.count(old) == 1
s = s.replace(old, """        if (more) lstore(buf ^ 1);
        asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    }""")
p.write_text(s)
