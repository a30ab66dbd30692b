"""The multi-rank sweep on ONE GPU: n handles (ranks 0..n-1) joined by the in-process
loopback communicator (dcfm_comm_init_loopback), each driven by its own host thread.
Every collective of the RCCL path (X message and shard sums of A all-gathers, column
sums for delta, the assembly batch all-gather, the Sigma all-reduce) runs with the same
call order and semantics, so this is the parity test of the decomposition itself: with
injected draws the n-rank chain must match the single-process oracle to the 1e-10 bar
of tests/test_gpu_parity.py, and the replicated quantities (X, delta, tau, Sigmaout)
must be bitwise identical on all ranks.
"""
import threading

import numpy as np
import pytest

from helpers import make_case, rel_err, stacked_draws, state_dict
from oracle import dc_oracle as F

pytestmark = pytest.mark.gpu


def _run_ranks(dcfm, c, g, K, burnin, mcmc, thin, n):
    N = burnin + mcmc
    G = g // n
    draws = stacked_draws(c["src"], 1, N)
    smps = [dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True,
                         nranks=n, rank=r, device=0) for r in range(n)]
    try:
        dcfm.Sampler.comm_loopback(smps)
        for r, smp in enumerate(smps):
            smp.set_data(c["Yd"][:, :, r * G:(r + 1) * G])
            st = state_dict(c["st"], r * G, G)
            smp.set_state({f: st[f] for f in st if f != "eta"})
            smp.set_draws(draws, 1, N)
        out, errs = [None] * n, []

        def work(r):
            try:
                smps[r].run(1, N)
                got = smps[r].get_state()
                got["Sig"] = smps[r].get_sigma()          # collective
                out[r] = got
            except Exception as e:                        # surfaced below
                errs.append(e)

        ths = [threading.Thread(target=work, args=(r,)) for r in range(n)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in ths), "a rank did not finish"
        assert not errs, errs
        return out, N
    finally:
        for smp in smps:
            smp.close()


@pytest.mark.parametrize("n,g,K,nobs,p", [(2, 4, 5, 40, 60), (4, 8, 6, 50, 96), (2, 4, 40, 60, 120)])
def test_loopback_ranks_match_oracle(dcfm, n, g, K, nobs, p):
    burnin, mcmc, thin = 1, 4, 2
    c = make_case(nobs, p, g, K, seed=13)
    out, N = _run_ranks(dcfm, c, g, K, burnin, mcmc, thin, n)
    ref = c["st"].copy()
    S_ref = F.run_chain(c["Yd"], ref, c["rho"], c["hyper"], c["src"].iteration, 1, N, burnin, mcmc, thin)
    for f in ("Sig", "X", "delta", "tauh"):
        for r in range(1, n):
            assert np.array_equal(out[0][f], out[r][f]), f"{f} differs between ranks 0 and {r}"
    assert rel_err(out[0]["Sig"], S_ref) < 1e-10
    for f in ("X", "delta", "tauh"):
        assert rel_err(out[0][f], getattr(ref, f)) < 1e-10, f
    for f in ("Lambda", "ps", "omega", "psi", "Plam", "Z", "eta"):
        both = np.concatenate([out[r][f] for r in range(n)], axis=-1)
        assert rel_err(both, getattr(ref, f)) < 1e-10, f
