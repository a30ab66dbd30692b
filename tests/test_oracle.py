"""CPU tests of the oracle restatement: MATLAB semantics, quirks, closed-form conditionals,
faithful loop vs vectorised form.  (Parity with MATLAB itself is unpinned: no MATLAB here.)"""
import numpy as np
import pytest

import oracle
from helpers import make_case, rel_err
from oracle import dc_oracle as F
from oracle import vectorised as V


def test_cholcov_is_upper_with_RtR():
    r = np.random.default_rng(0)
    B = r.standard_normal((6, 6))
    A = B @ B.T + 6 * np.eye(6)
    R = F.cholcov(A)
    assert np.allclose(np.tril(R, -1), 0)
    assert np.allclose(R.T @ R, A, rtol=1e-13, atol=1e-12)
    # cholcov rejects asymmetric input (MATLAB returns [] and the reference would fail)
    A2 = A.copy()
    A2[0, 1] += 1e-3
    with pytest.raises(ValueError):
        F.cholcov(A2)


def test_chol_lower_uses_lower_triangle():
    r = np.random.default_rng(1)
    B = r.standard_normal((5, 5))
    A = B @ B.T + 5 * np.eye(5)
    Ab = A.copy()
    Ab[np.triu_indices(5, 1)] = 99.0          # garbage upper triangle is ignored
    L = F.chol_lower(Ab)
    assert np.allclose(L @ L.T, A, rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize("K,g,axis", [(3, 4, 0), (1, 4, 2), (1, 1, None)])
def test_cumprod_first_nonsingleton_dim(K, g, axis):
    d = np.random.default_rng(2).uniform(0.5, 2, size=(K, 1, g))
    got = F.matlab_cumprod_delta(d)
    want = d.copy() if axis is None else np.cumprod(d, axis=axis)
    assert np.array_equal(got, want)


def test_preprocess_zero_columns_and_integrality():
    Y, _ = oracle.synth.make_data(10, 14, k0=2, zero_cols=2)
    Yk, n, p, P, K, keep = F.preprocess(Y, 3, 6)
    assert p == 12 and P == 4 and K == 2 and Yk.shape == (10, 12)
    assert np.all(np.count_nonzero(Yk, axis=0) > 0)
    with pytest.raises(ValueError):
        F.preprocess(Y, 5, 10)            # P = 12/5 not integral (dc:41)


def test_standardize_moments():
    Y, _ = oracle.synth.make_data(30, 12, k0=2)
    Yd = F.standardize(F.partition(Y, 3, np.arange(12)))
    assert np.allclose(Yd.mean(axis=0), 0, atol=1e-14)
    assert np.allclose(Yd.var(axis=0, ddof=1), 1, rtol=1e-13)


def test_lambda_row_is_the_gaussian_full_conditional():
    """With z = 0 the draw (dc:141-144) is the conditional mean Q^{-1} b."""
    c = make_case(25, 12, 2, 3, seed=5)
    st = c["st"]
    st.Lambda[...] = np.random.default_rng(3).standard_normal(st.Lambda.shape)
    F.update_eta(st, c["rho"])
    d = c["src"].iteration(1)
    d.NL[...] = 0.0
    F.update_Lambda(st, c["Yd"], d)
    for m in range(2):
        eta = st.eta[:, :, m]
        for j in range(c["P"]):
            Q = np.diag(st.Plam[j, :, m]) + st.ps[j, 0, m] * (eta.T @ eta)
            b = st.ps[j, 0, m] * (eta.T @ c["Yd"][:, j, m])
            assert np.allclose(st.Lambda[j, :, m], np.linalg.solve(Q, b), rtol=1e-10, atol=1e-12)


def test_Z_mean_uses_RRt_quirk_Q2():
    """dc:104: mean = (R R')^{-1} b with R = cholcov(Zprec) upper, not Zprec^{-1} b."""
    c = make_case(20, 12, 2, 3, seed=6)
    st = c["st"]
    rng = np.random.default_rng(4)
    st.Lambda[...] = rng.standard_normal(st.Lambda.shape)
    d = c["src"].iteration(1)
    d.NZ[...] = 0.0
    F.update_Z(st, c["Yd"], c["rho"], d)
    rho = c["rho"]
    m = 0
    Lam, om = st.Lambda[:, :, m], st.omega[:, m]
    Zprec = np.eye(3) + (1 - rho) * ((Lam * om[:, None]).T @ Lam)
    R = np.linalg.cholesky(Zprec).T
    i = 0
    bz = np.sqrt(1 - rho) * ((Lam * om[:, None]).T @ (c["Yd"][i, :, m] - np.sqrt(rho) * Lam @ st.X[i]))
    assert np.allclose(st.Z[i, :, m], np.linalg.solve(R @ R.T, bz), rtol=1e-10)
    assert not np.allclose(st.Z[i, :, m], np.linalg.solve(Zprec, bz), rtol=1e-6)


def test_delta_chain_reads_shard1_delta_quirk_Q4():
    """dc:161: for shard m >= 2 the h >= 2 update uses shard 1's already-updated delta_h."""
    c = make_case(15, 18, 3, 3, seed=7)
    st = c["st"]
    st.Lambda[...] = np.random.default_rng(5).standard_normal(st.Lambda.shape)
    d = c["src"].iteration(1)
    F.update_psi(st, c["hyper"], d)
    a = st.copy()
    F.update_delta_tau(a, c["hyper"], d)
    # recompute shard 2's h=2 step by hand with shard 1's new delta_2
    hyper = c["hyper"]
    b = st.copy()
    colsum = (b.psi[:, :, 1] * b.Lambda[:, :, 1] ** 2).sum(axis=0)
    d2 = b.delta[:, 0, 1].copy()
    t = np.cumprod(d2)
    bd = hyper.bd1 + 0.5 / d2[0] * np.sum(t * colsum)
    d2[0] = (1 / bd) * d.Gdelta[0, 1]
    t = np.cumprod(d2)
    bd = hyper.bd2 + 0.5 / a.delta[1, 0, 0] * np.sum(t[1:] * colsum[1:])
    assert np.isclose(a.delta[1, 0, 1], (1 / bd) * d.Gdelta[1, 1], rtol=1e-13)


@pytest.mark.parametrize("n,p,g,K", [(20, 24, 3, 2), (20, 24, 3, 1), (15, 12, 1, 3), (30, 40, 4, 5)])
def test_faithful_vs_vectorised(n, p, g, K):
    c = make_case(n, p, g, K, seed=9)
    s1, s2 = c["st"].copy(), c["st"].copy()
    S1 = F.run_chain(c["Yd"], s1, c["rho"], c["hyper"], c["src"].iteration, 1, 6, 2, 4, 2)
    S2 = V.full(V.run_chain(c["Yd"], s2, c["rho"], c["hyper"], c["src"].iteration, 1, 6, 2, 4, 2))
    for f, a in s1.as_dict().items():
        assert rel_err(getattr(s2, f), a) < 1e-12, f
    assert rel_err(S2, S1) < 1e-12


def test_faithful_vs_vectorised_at_c1_shape():
    """The vectorised oracle that the BASELINE-shape GPU parity tests use
    (tests/test_gpu_parity_configs.py) agrees with the faithful per-row loop at c1's shape
    (p = 1,000, n = 100, g = 4, K = 5), the largest the faithful loop runs in seconds."""
    c = make_case(100, 1000, 4, 5, seed=29, k0=10)
    s1, s2 = c["st"].copy(), c["st"].copy()
    S1 = F.run_chain(c["Yd"], s1, c["rho"], c["hyper"], c["src"].iteration, 1, 2, 1, 1, 1)
    S2 = V.full(V.run_chain(c["Yd"], s2, c["rho"], c["hyper"], c["src"].iteration, 1, 2, 1, 1, 1))
    for f, a in s1.as_dict().items():
        assert rel_err(getattr(s2, f), a) < 1e-12, f
    assert rel_err(S2, S1) < 1e-12


@pytest.mark.parametrize("name,n,p,g,K,iters", [("c2", 500, 5000, 8, 20, 2), ("c3", 1000, 19968, 64, 30, 1)])
def test_faithful_vs_vectorised_at_baseline_shapes(name, n, p, g, K, iters):
    """The vectorised oracle the BASELINE-shape GPU parity tests compare against is pinned to
    the faithful per-row loop (the reference's loop structure, dc:97-177) AT those shapes, with
    absolute bars: every iteration starts both restatements from the same state, and
    tests/helpers.stagewise_errors checks the stages before the loading solve and after it at
    1e-12 relative (ps / omega per row, unscaled, against the faithful residual update) and the
    loading draw by its per-row backward error (<= 1e-14) -- at c2's
    second iteration cond(Q_j) ~ 1e7 makes the two restatements' Lambda differ by ~1e-9 in
    forward error while both solve their systems to machine precision."""
    from helpers import stagewise_errors
    c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
    D = V.Data(c["Yd"])
    st = c["st"].copy()
    for it in range(1, iters + 1):
        d = c["src"].iteration(it)
        faithful = st.copy()
        F.gibbs_iteration(faithful, c["Yd"], c["rho"], c["hyper"], d)
        errs, bw, _ = stagewise_errors(st, faithful.as_dict(), D, c["rho"], c["hyper"], d)
        for f, e in errs.items():
            assert e < 1e-12, (name, it, f, e)
        assert bw < 1e-14, (name, it, bw)
        # the vectorised chain with dc:169's residual (the GPU's DCFM_FLAG_EXACT_RESIDUAL
        # reference): its ps / omega against the faithful update on its own eta and Lambda
        vec = st.copy()
        V.gibbs_iteration(vec, D, c["rho"], c["hyper"], d, direct=True)
        errs, bw, _ = stagewise_errors(st, vec.as_dict(), D, c["rho"], c["hyper"], d)
        assert errs["ps"] < 1e-12 and errs["omega"] < 1e-12, (name, it, errs["ps"], errs["omega"])
        st = vec


def test_posterior_mean_recovers_truth():
    """End-to-end statistical sanity of the oracle chain's Sigmaout against the synthetic truth.

    The reference model (quirks included: Q1 uses variances where the Z/X
    conditionals need precisions, Q3's g*I prior) is biased, so this bounds the
    error loosely instead of asserting it beats the sample covariance."""
    n, p, g, K = 200, 40, 4, 5
    c = make_case(n, p, g, K, seed=10, k0=3)
    Sig = V.full(V.run_chain(c["Yd"], c["st"], c["rho"], c["hyper"], c["src"].iteration, 1, 300, 100, 200, 2))
    truth = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
    err = oracle.synth.cov_errors(Sig, truth)
    assert np.all(np.isfinite(Sig)) and err["fro_rel"] < 0.8, err
    assert np.allclose(np.diag(Sig), 1.0, atol=0.25)           # standardised units (dc:57-59)


def test_truth_factors_match_dense_truth():
    """driver.truth_factors (the low-rank form dcfm_sigma_error takes) equals the dense
    truth in Sigmaout's coordinates (kept columns, varind order, standardised; dc:36-59)."""
    import __graft_entry__ as ge
    dcfm = ge.load_package()
    from helpers import make_case
    c = make_case(50, 90, 3, 4, seed=5, k0=4, zero_cols=3)
    _, _, Lam0, sig2 = oracle.synth.make_data(50, 90, k0=4, zero_cols=3, factors=True)
    U, s = dcfm.truth_factors(Lam0, sig2, c["Y"], c["keep"], c["init"].varind)
    dense = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
    np.testing.assert_allclose(U @ U.T + np.diag(s), dense, rtol=1e-13, atol=1e-13)


def test_unpermute_sigma_restores_input_order():
    """driver.unpermute_sigma undoes the output coordinates (Q7): the dense truth in
    Sigmaout's permuted, standardised space maps back to Sigma0 on the kept columns."""
    import __graft_entry__ as ge
    dcfm = ge.load_package()
    from helpers import make_case
    c = make_case(40, 60, 4, 4, seed=9, k0=3, zero_cols=4)
    S_out = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
    cols = dcfm.output_columns(c["keep"], c["init"].varind)
    sd = c["Y"][:, cols].std(axis=0, ddof=1)
    back = dcfm.unpermute_sigma(S_out, c["keep"], c["init"].varind, 60, sd=sd, fill=np.nan)
    keep = np.asarray(c["keep"])
    np.testing.assert_allclose(back[np.ix_(keep, keep)], c["Sigma0"][np.ix_(keep, keep)], rtol=1e-13, atol=1e-13)
    dropped = np.setdiff1d(np.arange(60), keep)
    assert dropped.size and np.all(np.isnan(back[dropped]))
