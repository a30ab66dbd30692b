"""Convergence diagnostics across chains on the per-iteration chain
trace the device records (``Sampler.set_trace`` / dcfm_set_trace).

The reference runs one chain and keeps no trace (divideconquer.m:180-196 accumulates only
Sigmaout); config c4 runs 8 parallel chains (BASELINE configs[3]), so the build adds the
standard between/within-chain checks on scalar summaries of each chain's state:

* ``split_rhat`` — potential scale reduction factor on split chains (Gelman et al.,
  Bayesian Data Analysis 3rd ed., §11.4): each chain is cut in halves, and
  R = sqrt(((n-1)/n W + B/n) / W) with B, W the between / within variances of the halves.
* ``ess`` — effective sample size over all chains (BDA3 §11.5: combined autocorrelation
  from the variogram, summed over Geyer's initial positive sequence of lag pairs).

Inputs are arrays of shape (chains, iterations) or (chains, iterations, quantities).
"""
from __future__ import annotations

import numpy as np

TRACE_FIELDS = ("lambda_fro2", "tr_omega", "sum_log_ps", "sum_log_tau")


def _as3(x):
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 2:
        x = x[:, :, None]
    if x.ndim != 3:
        raise ValueError("traces must be (chains, iterations[, quantities])")
    return x


def _split(x):
    n = x.shape[1] // 2
    if n < 2:
        raise ValueError("need at least 4 iterations per chain")
    return np.concatenate([x[:, :n], x[:, x.shape[1] - n:]], axis=0)     # (2m, n, q)


def split_rhat(traces) -> np.ndarray:
    """Split-R-hat per quantity (BDA3 §11.4); values near 1 mean the chains mix."""
    x = _split(_as3(traces))
    n = x.shape[1]
    means = x.mean(axis=1)                                  # (2m, q)
    B = n * means.var(axis=0, ddof=1)
    W = x.var(axis=1, ddof=1).mean(axis=0)
    var_plus = (n - 1) / n * W + B / n
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.sqrt(var_plus / W)


def ess(traces) -> np.ndarray:
    """Effective sample size per quantity over all split chains (BDA3 §11.5)."""
    x = _split(_as3(traces))
    m, n, q = x.shape
    means = x.mean(axis=1)
    B = n * means.var(axis=0, ddof=1)
    W = x.var(axis=1, ddof=1).mean(axis=0)
    var_plus = (n - 1) / n * W + B / n
    out = np.empty(q)
    for k in range(q):
        if not var_plus[k] > 0:
            out[k] = np.nan
            continue
        rho = []
        for t in range(1, n):
            vt = np.mean((x[:, t:, k] - x[:, :-t, k]) ** 2)          # variogram V_t
            rho.append(1.0 - vt / (2.0 * var_plus[k]))
        # Geyer: sum pairs rho_{2s-1} + rho_{2s} while they stay positive (rho_0 = 1 first)
        r = np.concatenate([[1.0], np.asarray(rho)])
        total = 0.0
        for s in range(0, len(r) - 1, 2):
            pair = r[s] + r[s + 1]
            if pair < 0:
                break
            total += pair
        out[k] = m * n / max(2.0 * total - 1.0, 1e-12)
    return out


def summarize(traces, fields=TRACE_FIELDS) -> dict:
    """{field: {"rhat": R, "ess": E}} for a (chains, iterations, 4) device trace."""
    r, e = split_rhat(traces), ess(traces)
    return {f: {"rhat": float(r[i]), "ess": float(e[i])} for i, f in enumerate(fields)}
