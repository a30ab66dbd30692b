"""Injected random-draw source (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

The reference consumes MATLAB's global stream through ``randperm``, ``normrnd``
(= ``randn``) and ``gamrnd`` (= ``b .* randg(a)``) — SURVEY.md Appendix B.
Every gamma shape it uses is >= 1 and data independent; only the scales depend
on the state.  So a run is fully determined by buffers of *standard* normal and
*standard* gamma variates.  This module produces those buffers (seeded NumPy,
not MATLAB's mt19937ar) in the reference's consumption layout, with MATLAB
array shapes:

  init  (dc:50,69,71,73,80,83)
    varind  p        randperm(p), 0-based here
    ps0     P x 1 x g randg(as)                    (dc:69, scaled by 1/bs)
    X0      n x K     randn                        (dc:71)
    psi0    P x K x g randg(df/2)                  (dc:73, scaled by 2/df)
    Z0      n x K x g randn, per shard             (dc:80)
    delta0  K x g     [randg(ad1); randg(ad2,K-1)] (dc:83, scaled by bd1 / bd2)

  per iteration (dc:104,126,142,150,158,163,170)
    NZ      K x n x g normals, for m, for i: randn(K,1)     (dc:104)
    NX      K x n     normals, for i: randn(K,1)            (dc:126)
    NL      K x P x g normals, for m, for j: randn(K,1)     (dc:142)
    Gpsi    P x K x g randg(df/2 + 0.5)                     (dc:150)
    Gdelta  K x g     h=1: randg(ad1 + P*K/2); h>=2: randg(ad2 + P*(K-h+1)/2)  (dc:158,163)
    Gps     P x g     randg(as + n/2)                       (dc:170)

The C-ABI ``dcfm_set_draws`` takes exactly these arrays (column-major), one
trailing iteration dimension added.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def gamma_shapes(n: int, P: int, K: int, hyper) -> dict:
    """Standard-gamma shapes of every gamma site (dc:69,73,83,150,157,161,170)."""
    h1 = np.arange(1, K + 1)
    dshape = np.where(h1 == 1, hyper.ad1 + 0.5 * P * K, hyper.ad2 + 0.5 * P * (K - h1 + 1))
    return {
        "ps0": float(hyper.as_),
        "psi0": float(hyper.df / 2.0),
        "delta0": np.where(h1 == 1, hyper.ad1, hyper.ad2).astype(float),
        "psi": float(hyper.df / 2.0 + 0.5),
        "delta": dshape.astype(float),
        "ps": float(hyper.as_ + 0.5 * n),
    }


@dataclass
class InitDraws:
    varind: np.ndarray
    ps0: np.ndarray
    X0: np.ndarray
    psi0: np.ndarray
    Z0: np.ndarray
    delta0: np.ndarray


@dataclass
class IterDraws:
    NZ: np.ndarray
    NX: np.ndarray
    NL: np.ndarray
    Gpsi: np.ndarray
    Gdelta: np.ndarray
    Gps: np.ndarray

    def stacked(self, others=()):
        """Stack this and further IterDraws along a trailing iteration axis."""
        seq = [self, *others]
        return {f: np.stack([getattr(d, f) for d in seq], axis=-1)
                for f in ("NZ", "NX", "NL", "Gpsi", "Gdelta", "Gps")}


class DrawSource:
    """Seeded source of standard variates in reference consumption layout.

    Iteration ``t`` (1-based, as ``iter`` in dc:90) always yields the same
    draws for the same seed, independent of which other iterations were drawn.
    """

    def __init__(self, seed: int, n: int, p: int, g: int, K: int, hyper):
        if p % g:
            raise ValueError("p must be divisible by g (dc:41)")
        self.seed = int(seed)
        self.n, self.p, self.g, self.K = n, p, g, K
        self.P = p // g
        self.hyper = hyper
        self.shapes = gamma_shapes(n, self.P, K, hyper)

    def _rng(self, *tag):
        return np.random.Generator(np.random.PCG64(np.random.SeedSequence([self.seed, *tag])))

    def init(self) -> InitDraws:
        n, p, g, K, P = self.n, self.p, self.g, self.K, self.P
        r = self._rng(0, 0)
        varind = r.permutation(p)
        ps0 = r.standard_gamma(self.shapes["ps0"], size=(P, 1, g))
        X0 = r.standard_normal((n, K))
        psi0 = r.standard_gamma(self.shapes["psi0"], size=(P, K, g))
        Z0 = np.empty((n, K, g))
        delta0 = np.empty((K, g))
        for m in range(g):
            Z0[:, :, m] = r.standard_normal((n, K))
            delta0[0, m] = r.standard_gamma(self.hyper.ad1)
            if K > 1:
                delta0[1:, m] = r.standard_gamma(self.hyper.ad2, size=K - 1)
        return InitDraws(varind, ps0, X0, psi0, Z0, delta0)

    def iteration(self, it: int) -> IterDraws:
        n, g, K, P = self.n, self.g, self.K, self.P
        r = self._rng(1, int(it))
        NZ = r.standard_normal((K, n, g))
        NX = r.standard_normal((K, n))
        NL = r.standard_normal((K, P, g))
        Gpsi = r.standard_gamma(self.shapes["psi"], size=(P, K, g))
        Gdelta = np.empty((K, g))
        for h in range(K):
            Gdelta[h, :] = r.standard_gamma(self.shapes["delta"][h], size=g)
        Gps = r.standard_gamma(self.shapes["ps"], size=(P, g))
        return IterDraws(NZ, NX, NL, Gpsi, Gdelta, Gps)
