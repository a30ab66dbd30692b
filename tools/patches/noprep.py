"""Dev A/B: prep_gram's loads in the committed rounds of 4 chunks (HEAD) instead of one round."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
i = s.index("    // latency-bound: a wave's chunks tt, tt + 4, ... are requested in rounds of UB")
j = s.index("            if (tt + 4 * u < nt) mm(wj[u], l[u]);\n    }\n", i) + len("            if (tt + 4 * u < nt) mm(wj[u], l[u]);\n    }\n")
s = s[:i] + """    const int nt = d.PP >> 3;
    int tt = wave;
    for (; tt + 12 < nt; tt += 16) {
        d2 wj[4];
        double l[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ld(tt + 4 * u, wj[u], l[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) mm(wj[u], l[u]);
    }
    for (; tt < nt; tt += 4) {
        d2 wj;
        double l[4];
        ld(tt, wj, l);
        mm(wj, l);
    }
""" + s[j:]
open(f, "w").write(s)
