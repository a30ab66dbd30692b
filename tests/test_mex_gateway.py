"""The MATLAB side of the boundary: matlab/dcfm_mex.c compiled with gcc
against a mock of the MEX / mx API (tests/mexmock; no MATLAB exists here or on the GPU box)
and driven the way MATLAB would call it.

CPU: the gateway type-checks with -Wall -Wextra -Werror, and rejects malformed calls
(wrong argument count, class, element count, bad handle, invalid config) before the
library sees a pointer.  GPU: a whole chain through the gateway — create, set_data,
set_state, set_draws, run, get_state, get_sigma — equals the same chain through the
Python host twin bit for bit, and a wrong-sized array is refused rather than over-read.
"""
import numpy as np
import pytest

from helpers import make_case, stacked_draws, state_dict
from mexmock import driver as mm


@pytest.fixture(scope="module")
def mex(tmp_path_factory):
    return mm.Mex(mm.build(tmp_path_factory.mktemp("mexmock")))


def _cfg(**kw):
    c = dict(n=30.0, P=10.0, g=4.0, K=3.0, rho=0.5, burnin=1.0, mcmc=2.0, thin=1.0, inject=1.0)
    c.update(kw)
    return c


def test_gateway_typechecks():
    mm.syntax_check()


def test_malformed_calls_are_rejected(mex):
    with pytest.raises(mm.MexError) as e:
        mex.call(3.0)                              # command not a string
    assert e.value.id == "dcfm:cmd"
    with pytest.raises(mm.MexError) as e:
        mex.call("frobnicate")
    assert e.value.id == "dcfm:cmd"
    with pytest.raises(mm.MexError) as e:
        mex.call("create")                         # missing cfg
    assert e.value.id == "dcfm:nargs"
    with pytest.raises(mm.MexError) as e:
        mex.call("create", 1.0)                    # cfg not a struct
    assert e.value.id == "dcfm:cfg"
    with pytest.raises(mm.MexError) as e:
        mex.call("create", _cfg(rho=np.array([0.5, 0.5])))   # non-scalar field
    assert e.value.id == "dcfm:cfg"
    with pytest.raises(mm.MexError) as e:
        mex.call("create", _cfg(rho=1.5))          # library validation, before any device call
    assert e.value.id == "dcfm:create" and "rho" in e.value.msg
    for cmd in ("run", "get_sigma", "set_data", "destroy"):
        with pytest.raises(mm.MexError) as e:
            mex.call(cmd, 7.0, *([1.0, 1.0] if cmd == "run" else [np.zeros(3)] if cmd == "set_data" else []))
        assert e.value.id == "dcfm:handle", cmd
    assert mex.locks() == 0


def test_malformed_calls_under_address_and_ub_sanitizers(tmp_path):
    """SURVEY §5 (race detection / sanitizers): the gateway and the mock MEX runtime built with
    -fsanitize=address,undefined (host code only; GPU sanitizers are unavailable on the pool)
    run the malformed-call suite (tests/mexmock/asan_main.c) with leak checking on: every call
    is rejected with its error id and no out-of-bounds access, use after free, leak or undefined
    behaviour is reported."""
    import os
    import subprocess
    exe = tmp_path / "mex_asan"
    cmd = ["gcc", *mm.FLAGS, "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", str(mm.ROOT / "matlab" / "dcfm_mex.c"),
           str(mm.ROOT / "tests" / "mexmock" / "mexmock.c"), str(mm.ROOT / "tests" / "mexmock" / "asan_main.c"),
           f"-L{mm.PKG}", "-ldcfm", f"-Wl,-rpath,{mm.PKG}", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_create_without_gpu_reports_the_hip_error(mex, gpu_available):
    if gpu_available:
        pytest.skip("a GPU is present")
    with pytest.raises(mm.MexError) as e:
        mex.call("create", _cfg())
    assert e.value.id == "dcfm:create"


@pytest.mark.gpu
def test_chain_through_the_gateway_matches_the_host_twin(mex, dcfm):
    n, p, g, K = 40, 48, 4, 5
    burnin, mcmc, thin = 1, 3, 2
    N = burnin + mcmc
    c = make_case(n, p, g, K, seed=11)
    P = c["P"]
    st = state_dict(c["st"])
    d = stacked_draws(c["src"], 1, N)
    h = mex.call("create", _cfg(n=float(n), P=float(P), g=float(g), K=float(K), rho=c["rho"],
                                burnin=float(burnin), mcmc=float(mcmc), thin=float(thin)))
    try:
        # wrong sizes are refused before the library reads them
        with pytest.raises(mm.MexError) as e:
            mex.call("set_data", h, c["Yd"][:, :, :2])
        assert e.value.id == "dcfm:arg"
        with pytest.raises(mm.MexError) as e:
            mex.call("set_data", h, c["Yd"], 1.0)
        assert e.value.id == "dcfm:nargs"
        mex.call("set_data", h, c["Yd"])
        mex.call("set_state", h, st["Lambda"], st["ps"], st["omega"], st["psi"], st["Plam"], st["X"], st["Z"],
                 st["delta"], st["tauh"])
        with pytest.raises(mm.MexError) as e:
            mex.call("set_draws", h, d["NZ"][:-1], d["NX"], d["NL"], d["Gpsi"], d["Gdelta"], d["Gps"], 1.0, float(N))
        assert e.value.id == "dcfm:arg"
        mex.call("set_draws", h, d["NZ"], d["NX"], d["NL"], d["Gpsi"], d["Gdelta"], d["Gps"], 1.0, float(N))
        mex.call("run", h, 1.0, float(N))
        got = mex.call("get_state", h, nlhs=10)
        S = mex.call("get_sigma", h)
        with pytest.raises(mm.MexError) as e:
            mex.call("get_sigma", h, float(p + 1))        # a caller-supplied p cannot resize the output
        assert e.value.id == "dcfm:arg"
    finally:
        mex.call("destroy", h)
    assert mex.locks() == 0

    smp = dcfm.Sampler(n, P, g, K, c["rho"], burnin, mcmc, thin, inject_draws=True)
    try:
        smp.set_data(c["Yd"])
        smp.set_state({f: v for f, v in st.items() if f != "eta"})
        smp.set_draws(d, 1, N)
        smp.run(1, N)
        ref = smp.get_state()
        S_ref = smp.get_sigma()
    finally:
        smp.close()
    names = ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "eta", "delta", "tauh")
    for name, a in zip(names, got):
        assert np.array_equal(a.reshape(-1, order="F"), np.asarray(ref[name]).reshape(-1, order="F")), name
    assert S.shape == (p, p) and np.array_equal(S, S_ref)
