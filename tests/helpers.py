"""Shared setup for parity tests: oracle chain + matching GPU sampler inputs."""
from __future__ import annotations

import numpy as np

import oracle
from oracle import dc_oracle as F

STATE_CMP = ("Lambda", "X", "Z", "eta", "ps", "omega", "psi", "Plam", "delta", "tauh")


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b).reshape(a.shape)
    den = float(np.max(np.abs(b))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / max(den, 1e-300)


def make_case(n, p, g, K, *, rho=0.5, seed=3, k0=4, zero_cols=0, dense_truth=True):
    Y, Sigma0 = oracle.synth.make_data(n, p, k0=k0, zero_cols=zero_cols, dense_truth=dense_truth)
    hyper = F.Hyper()
    Yk, n, pk, P, K_, keep = F.preprocess(Y, g, K * g)
    src = oracle.DrawSource(seed, n, pk, g, K, hyper)
    init = src.init()
    Yd = F.standardize(F.partition(Yk, g, init.varind))
    st = F.initialise(n, P, K, g, rho, hyper, init)
    return dict(Y=Y, Sigma0=Sigma0, Yd=Yd, st=st, src=src, init=init, hyper=hyper, n=n, p=pk,
                P=P, K=K, g=g, rho=rho, keep=keep)


def state_dict(st, s0=0, gl=None):
    out = {}
    for f in STATE_CMP:
        a = getattr(st, f)
        if gl is not None and f not in ("X", "delta", "tauh"):
            a = a[..., s0:s0 + gl]
        out[f] = a
    return out


def stacked_draws(src, first, n_iter):
    ds = [src.iteration(t) for t in range(first, first + n_iter)]
    return ds[0].stacked(ds[1:])


def sigma_stripe_from_lower(SigLower, c0, c1):
    """Columns [c0, c1) of the symmetric matrix whose lower triangle is SigLower (p x p)."""
    lo = SigLower[:, c0:c1]
    up = SigLower[c0:c1, :].T
    r = np.arange(SigLower.shape[0])[:, None]
    c = np.arange(c0, c1)[None, :]
    return np.where(r >= c, lo, up)
