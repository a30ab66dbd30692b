"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces its committed fixtures (regression pin).
GPU: the HIP path, fed the fixture's inputs and draws, reproduces every
iteration's state and the final Sigmaout to 1e-10 relative.
"""
from pathlib import Path

import numpy as np
import pytest

from helpers import rel_err
from oracle import dc_oracle as F

GOLDEN = sorted((Path(__file__).parent / "golden").glob("*.npz"))
STATE = ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "eta", "delta", "tauh")


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def init_state(fx):
    return F.SamplerState(**{f: fx[f"init_{f}"].copy() for f in STATE})


def draws_fn(fx):
    from oracle.draws import IterDraws

    def get(t):
        return IterDraws(*(fx[f"draw_{f}"][..., t - 1] for f in ("NZ", "NX", "NL", "Gpsi", "Gdelta", "Gps")))
    return get


@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_oracle_reproduces_fixture(path):
    fx = load(path)
    n, p, g, K, burnin, mcmc, thin, seed = (int(v) for v in fx["meta"])
    rho = float(fx["rho"])
    Yk, n2, p2, P, K2, keep = F.preprocess(fx["Y"], g, K * g)
    assert np.array_equal(keep, fx["keep"])
    Yd = F.standardize(F.partition(Yk, g, fx["varind"]))
    assert np.array_equal(Yd, fx["Yd"])
    st = init_state(fx)
    rec = []
    S = F.run_chain(Yd, st, rho, F.Hyper(), draws_fn(fx), 1, burnin + mcmc, burnin, mcmc, thin, record=rec)
    for t, s in enumerate(rec, start=1):
        for f in STATE:
            assert rel_err(getattr(s, f), fx[f"it{t}_{f}"]) < 1e-13, (t, f)
    assert rel_err(S, fx["Sigmaout"]) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_gpu_matches_fixture(dcfm, path):
    fx = load(path)
    n, p, g, K, burnin, mcmc, thin, seed = (int(v) for v in fx["meta"])
    rho = float(fx["rho"])
    N = burnin + mcmc
    P = p // g
    smp = dcfm.Sampler(n, P, g, K, rho, burnin, mcmc, thin, inject_draws=True)
    try:
        smp.set_data(fx["Yd"])
        smp.set_state({f: fx[f"init_{f}"] for f in STATE if f != "eta"})
        smp.set_draws({f: fx[f"draw_{f}"] for f in ("NZ", "NX", "NL", "Gpsi", "Gdelta", "Gps")}, 1, N)
        for t in range(1, N + 1):
            smp.run(t, 1)
            got = smp.get_state()
            for f in STATE:
                assert rel_err(got[f], fx[f"it{t}_{f}"]) < 1e-10, (t, f)
        assert rel_err(smp.get_sigma(), fx["Sigmaout"]) < 1e-10
    finally:
        smp.close()
