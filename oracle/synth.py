"""Synthetic sparse-factor data + truth-error metrics (TEST INFRASTRUCTURE ONLY).

The reference ships no data or generator.  This is the
builder-defined generator of SURVEY §8d:

  Lambda0 (p x k0) with N(0,1) entries, a fraction ``sparsity`` of them zeroed;
  sigma0^2 ~ U(0.2, 1);  Sigma0 = Lambda0 Lambda0' + diag(sigma0^2);
  Y (n x p) = F Lambda0' + E,  F ~ N(0, I_k0),  E ~ N(0, diag sigma0^2).

Errors are measured in the reference's OUTPUT space (quirk Q7, dc:36-39,50-59,
186-195): Sigmaout is in the order (kept columns)[varind] and in standardised
units, so the truth is permuted the same way and scaled by the sample standard
deviations.
"""
from __future__ import annotations

import numpy as np

DATA_SEED = 20161209


def make_data(n: int, p: int, k0: int = 10, sparsity: float = 0.7, seed: int = DATA_SEED,
              zero_cols: int = 0, factors: bool = False, dense_truth: bool = True):
    """Y (n x p) and Sigma0; with ``factors`` also (Lambda0, sigma0^2) of Sigma0.
    ``dense_truth=False`` returns None for Sigma0 (p x p: 3.2 GB at p = 20k)."""
    r = np.random.Generator(np.random.PCG64(seed))
    Lam0 = r.standard_normal((p, k0))
    Lam0[r.random((p, k0)) < sparsity] = 0.0
    sig2 = r.uniform(0.2, 1.0, size=p)
    F = r.standard_normal((n, k0))
    E = r.standard_normal((n, p)) * np.sqrt(sig2)[None, :]
    Y = F @ Lam0.T + E
    Sigma0 = Lam0 @ Lam0.T + np.diag(sig2) if dense_truth else None
    if zero_cols:
        cols = r.choice(p, size=zero_cols, replace=False)
        Y[:, cols] = 0.0
    if factors:
        return Y, Sigma0, Lam0, sig2
    return Y, Sigma0


def truth_in_output_space(Sigma0: np.ndarray, Y: np.ndarray, keep: np.ndarray, varind: np.ndarray):
    """Sigma0 restricted to kept columns, permuted by varind, standardised (dc:38,50-59)."""
    S = Sigma0[np.ix_(keep, keep)][np.ix_(varind, varind)]
    sd = Y[:, keep][:, varind].std(axis=0, ddof=1)
    return S / sd[:, None] / sd[None, :]


def cov_errors(Sigma_hat: np.ndarray, Sigma_true: np.ndarray):
    """Frobenius and operator-norm error of a covariance estimate."""
    D = Sigma_hat - Sigma_true
    fro = float(np.linalg.norm(D, "fro"))
    op = float(np.max(np.abs(np.linalg.eigvalsh((D + D.T) / 2))))
    return {"fro": fro, "op": op, "fro_rel": fro / float(np.linalg.norm(Sigma_true, "fro"))}
