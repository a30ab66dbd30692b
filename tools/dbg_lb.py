import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import __graft_entry__ as ge
dcfm = ge.load_package()
from test_gpu_loopback import _run_ranks, make_case, state_dict, stacked_draws
def one(c, g, K, burnin, mcmc, thin):
    N = burnin + mcmc
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True)
    smp.set_data(c["Yd"]); smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
    smp.set_draws(stacked_draws(c["src"], 1, N), 1, N); smp.run(1, N)
    st = smp.get_state(); st["Sig"] = smp.get_sigma(); smp.close(); return st
for (n,g,K,nobs,p) in [(2,4,5,40,60),(4,8,6,50,96)]:
    c = make_case(nobs, p, g, K, seed=3)
    out, N = _run_ranks(dcfm, c, g, K, 1, 4, 2, n)
    o = one(c, g, K, 1, 4, 2)
    for f in ("X","delta","tauh","Sig"):
        a, b = out[0][f], o[f]
        print(n, f, np.max(np.abs(a-b)), np.argwhere(a!=b)[:3].tolist())
    for f in ("Lambda","ps","omega"):
        both = np.concatenate([out[r][f] for r in range(n)], axis=-1)
        print(n, f, np.max(np.abs(both - o[f])))
