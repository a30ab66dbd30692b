"""GPU: per-iteration chain trace (dcfm_set_trace, trace.hip) against the same summaries
of the oracle chain's state after each iteration (same injected draws), narrow and wide
paths, one rank and two loopback ranks (rows add).  Bar: 1e-10 relative, as the state."""
import threading

import numpy as np
import pytest

from helpers import make_case, stacked_draws, state_dict
from oracle import dc_oracle as F

pytestmark = pytest.mark.gpu

TOL = 1e-10


def _oracle_rows(c, N):
    ref = c["st"].copy()
    rows = []
    S = None
    for it in range(1, N + 1):
        S = F.run_chain(c["Yd"], ref, c["rho"], c["hyper"], c["src"].iteration, it, 1, 0, N, 1, Sigmaout=S)
        rows.append([np.sum(ref.Lambda ** 2), np.sum(ref.omega), np.sum(np.log(ref.ps)),
                     np.sum(np.log(ref.tauh))])
    return np.array(rows)


@pytest.mark.parametrize("shape", [(40, 48, 4, 5), (37, 57, 3, 7), (45, 141, 3, 40)])
def test_trace_matches_oracle(dcfm, shape):
    n, p, g, K = shape
    c = make_case(n, p, g, K)
    N = 4
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 0, N, 1, inject_draws=True)
    try:
        smp.set_data(c["Yd"])
        smp.set_state(state_dict(c["st"]))
        smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
        smp.set_trace(N - 1)                 # capacity bound: the last iteration is not recorded
        smp.run(1, N)
        tr = smp.get_trace()
    finally:
        smp.close()
    want = _oracle_rows(c, N)
    assert tr.shape == (N - 1, 4)
    err = np.max(np.abs(tr - want[:N - 1]) / np.maximum(np.abs(want[:N - 1]), 1e-300))
    assert err < TOL, (tr, want)


def test_trace_two_loopback_ranks_add_up(dcfm):
    c = make_case(33, 72, 6, 3)
    N, R, gl = 3, 2, 3
    draws = stacked_draws(c["src"], 1, N)
    smps = [dcfm.Sampler(c["n"], c["P"], 6, 3, c["rho"], 0, N, 1, nranks=R, rank=r, inject_draws=True)
            for r in range(R)]
    try:
        dcfm.Sampler.comm_loopback(smps)
        for r, s in enumerate(smps):
            s.set_data(c["Yd"][:, :, r * gl:(r + 1) * gl])
            s.set_state(dcfm.local_state(state_dict(c["st"]), r * gl, gl))
            s.set_draws(draws, 1, N)
            s.set_trace(N)
        errs = []

        def go(s):
            try:
                s.run(1, N)
                s.synchronize()
            except Exception as e:          # noqa: BLE001 - surfaced below
                errs.append(e)
        th = [threading.Thread(target=go, args=(s,)) for s in smps]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
        assert not errs, errs
        tr = sum(s.get_trace() for s in smps)
    finally:
        for s in smps:
            s.close()
    want = _oracle_rows(c, N)
    err = np.max(np.abs(tr - want) / np.abs(want))
    assert err < TOL


def test_trace_off_by_default_and_resettable(dcfm):
    c = make_case(40, 48, 4, 5)
    smp = dcfm.Sampler(c["n"], c["P"], 4, 5, c["rho"], 0, 6, 1)
    try:
        smp.set_data(c["Yd"])
        smp.set_state(state_dict(c["st"]))
        smp.run(1, 2)
        assert smp.get_trace().shape == (0, 4)
        smp.set_trace(10)
        smp.run(3, 4)
        tr = smp.get_trace()
        assert tr.shape == (4, 4) and np.all(np.isfinite(tr))
        smp.set_trace(0)
        assert smp.get_trace().shape == (0, 4)
    finally:
        smp.close()
