"""A/B timing only (wrong numbers): k_zxchol without the delta-chain blocks' work."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = """        if (m < d.g)
            delta_shard(d, sall, da.delta_in, da.tau_in, da.delta_out, da.tau_out, dr, da.iter, m, threadIdx.x & 63);"""
assert old in s
s = s.replace(old, "")
open(f, "w").write(s)
