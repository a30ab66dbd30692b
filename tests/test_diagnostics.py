"""Convergence diagnostics across chains (host logic, no GPU): split-R-hat and ESS of
<pkg>/diagnostics.py against known-answer cases and a plain-loop restatement of BDA3 §11.4."""
import numpy as np


def _rhat_loops(x):
    """Split-R-hat of one quantity, x: chains x iterations, written out with loops."""
    n = x.shape[1] // 2
    halves = []
    for c in x:
        halves += [c[:n], c[len(c) - n:]]
    m = len(halves)
    means = [sum(h) / n for h in halves]
    grand = sum(means) / m
    B = n / (m - 1) * sum((mu - grand) ** 2 for mu in means)
    W = sum(sum((v - mu) ** 2 for v in h) / (n - 1) for h, mu in zip(halves, means)) / m
    return ((n - 1) / n * W + B / n) / W


def test_rhat_matches_loop_restatement(dcfm):
    x = np.random.default_rng(0).standard_normal((3, 41))
    got = dcfm.diagnostics.split_rhat(x)[0]
    assert abs(got - np.sqrt(_rhat_loops(x))) < 1e-12


def test_iid_chains_mix(dcfm):
    x = np.random.default_rng(1).standard_normal((4, 1000, 2))
    r = dcfm.diagnostics.split_rhat(x)
    e = dcfm.diagnostics.ess(x)
    assert np.all(r < 1.02)
    assert np.all((e > 0.7 * 4000) & (e < 1.3 * 4000)), e


def test_shifted_chain_flags_nonconvergence(dcfm):
    x = np.random.default_rng(2).standard_normal((4, 500))
    x[1] += 3.0
    assert dcfm.diagnostics.split_rhat(x)[0] > 1.5


def test_trending_chain_flags_nonconvergence(dcfm):
    """Split halves catch a drift inside a single chain (1 chain = 2 halves)."""
    t = np.linspace(0.0, 5.0, 400)
    x = (t + np.random.default_rng(3).standard_normal(400))[None, :]
    assert dcfm.diagnostics.split_rhat(x)[0] > 1.5


def test_ar1_ess(dcfm):
    phi, m, n = 0.9, 4, 4000
    r = np.random.default_rng(4)
    x = np.empty((m, n))
    x[:, 0] = r.standard_normal(m) / np.sqrt(1 - phi ** 2)
    for t in range(1, n):
        x[:, t] = phi * x[:, t - 1] + r.standard_normal(m)
    want = m * n * (1 - phi) / (1 + phi)
    got = dcfm.diagnostics.ess(x)[0]
    assert 0.6 * want < got < 1.4 * want, (got, want)


def test_summarize_fields(dcfm):
    x = np.random.default_rng(5).standard_normal((2, 50, 4))
    s = dcfm.diagnostics.summarize(x)
    assert set(s) == set(dcfm.diagnostics.TRACE_FIELDS)
    assert all(set(v) == {"rhat", "ess"} for v in s.values())
