"""GPU: on-device initial state (dcfm_init_state, init.hip; dc:68-87).

Pinned against the host formula of dc:68-87 (driver.initial_state) applied to the same
standard variates, reproduced through dcfm_rng_fill at the documented counters (sites 7-12,
iteration 0, variate e = MATLAB linear index inside the shard's array).  The arithmetic is
the same scalings and the same cumprod order, so the bar is 1e-14 relative."""
import numpy as np
import pytest

from helpers import rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-14
FIELDS = ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "eta", "delta", "tauh")


def _host_init(dcfm, n, P, g, K, rho, seed):
    h = dcfm.Hyper()
    f = lambda kind, cnt, site, shard, shape=1.0: dcfm.rng_fill(kind, cnt, seed=seed, shape=shape, site=site,
                                                               shard=shard, iteration=0)

    class Init:
        pass
    init = Init()
    init.ps0 = np.stack([f("gamma", P, 7, m, h.as_) for m in range(g)], axis=1)[:, None, :]
    init.X0 = f("normal", n * K, 8, 0).reshape(n, K, order="F")
    init.psi0 = np.stack([f("gamma", P * K, 9, m, h.df / 2).reshape(P, K, order="F") for m in range(g)], axis=2)
    init.Z0 = np.stack([f("normal", n * K, 10, m).reshape(n, K, order="F") for m in range(g)], axis=2)
    init.delta0 = np.empty((K, g))
    for m in range(g):
        init.delta0[0, m] = f("gamma", 1, 11, m, h.ad1)[0]
        if K > 1:
            init.delta0[1:, m] = f("gamma", K, 12, m, h.ad2)[1:]
    return dcfm.initial_state(n, P, K, g, rho, h, init)


@pytest.mark.parametrize("n,P,g,K", [(37, 19, 3, 7), (40, 12, 4, 1), (45, 47, 3, 40)])
def test_init_state_matches_host_formula(dcfm, n, P, g, K):
    rho, seed = 0.5, 1234
    smp = dcfm.Sampler(n, P, g, K, rho, 0, 2, 1, seed=seed)
    try:
        smp.init_state()
        got = smp.get_state()
    finally:
        smp.close()
    want = _host_init(dcfm, n, P, g, K, rho, seed)
    for f in FIELDS:
        if f == "Lambda":
            assert not np.any(got[f])
            continue
        assert rel_err(got[f], want[f]) < TOL, f


def test_init_state_two_ranks_hold_slices_of_one_rank(dcfm):
    n, P, g, K, seed = 33, 20, 6, 5, 77
    one = dcfm.Sampler(n, P, g, K, 0.5, 0, 1, 1, seed=seed)
    try:
        one.init_state()
        ref = one.get_state()
    finally:
        one.close()
    gl = g // 2
    for r in range(2):
        smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 1, 1, seed=seed, nranks=2, rank=r)
        try:
            smp.init_state()
            got = smp.get_state()
        finally:
            smp.close()
        for f in FIELDS:
            want = ref[f] if f in ("X", "delta", "tauh") else ref[f][..., r * gl:(r + 1) * gl]
            np.testing.assert_array_equal(got[f], want, err_msg=f)


def test_chain_from_device_init_equals_chain_from_its_upload(dcfm):
    """init_state then run == set_state(the same state) then run (on-device Philox draws)."""
    n, P, g, K, seed, N = 40, 24, 4, 6, 5, 6
    from helpers import make_case
    Yd = make_case(n, P * g, g, K)["Yd"]
    out = []
    init = None
    for mode in ("device", "upload"):
        smp = dcfm.Sampler(n, P, g, K, 0.5, 2, N - 2, 1, seed=seed)
        try:
            smp.set_data(Yd)
            if mode == "device":
                smp.init_state()
                init = smp.get_state()
            else:
                smp.set_state({f: init[f] for f in init if f != "eta"})
            smp.run(1, N)
            st = smp.get_state()
            st["Sigma"] = smp.get_sigma()
            out.append(st)
        finally:
            smp.close()
    for f in out[0]:
        assert rel_err(out[0][f], out[1][f]) < 1e-13, f
