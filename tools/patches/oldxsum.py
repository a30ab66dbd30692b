"""A/B: the pre-canonical A sum in k_deltaops (plain accumulate, not the tree)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "        const double acc = tree_sum(A + (size_t)m0 * KP * KP + e, chunk, (size_t)KP * KP);"
new = """        double acc = 0.0;
#pragma unroll 8
        for (int m = m0; m < m0 + chunk; ++m) acc += A[(size_t)m * KP * KP + e];"""
assert old in s
s = s.replace(old, new)
old = "        xa[e] = tree_sum_f<double>(nxs, [&](int jj) { return (jj == j) ? v[u] : ld_agent(xpart + (size_t)jj * KP * KP + e); });"
new = """        double acc = 0.0;
        for (int jj = 0; jj < nxs; ++jj) acc += (jj == j) ? v[u] : ld_agent(xpart + (size_t)jj * KP * KP + e);
        xa[e] = acc;"""
assert old in s
s = s.replace(old, new)
open(f, "w").write(s)
