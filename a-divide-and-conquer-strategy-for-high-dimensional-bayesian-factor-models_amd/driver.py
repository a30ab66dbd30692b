"""Host twin of the reference driver and public entry point.

``divideconquer(Y, g, k, BURNIN, MCMC, thin, rho)`` mirrors the reference
function ``Sigmaout = divideconquer(Y,g,k,BURNIN,MCMC,thin,rho)``
(divideconquer.m:1): same arguments, same meaning, same output (the p x p
posterior-mean covariance in the permuted, standardised coordinates of
dc:186-195, quirk Q7).  The driver half (dc:29-87: zero-column removal,
P = p/g and K = k/g integrality, partition by randperm, standardisation,
hyper-parameters, initial draws) runs here on the host, as it does in MATLAB;
the hot loop (dc:90-197) runs on the GPU through the C ABI.

Differences a user should know:
  * The reference seeds nothing (no ``rng`` call); here ``seed`` selects both
    the host init draws (NumPy PCG64) and the on-device Philox stream.
  * ``init_draws`` / ``iter_draws`` inject standard variates (SURVEY
    Appendix B layout) instead — this is how the parity tests drive it.
  * ``return_info=True`` additionally returns varind (the permutation, which
    the reference never returns) and the kept-column index.
"""
from __future__ import annotations

import time

import numpy as np

from .sampler import Hyper, Sampler, count_nonzero_columns


def preprocess(Y, g, k):
    """dc:29-41. Returns (Y_kept, n, p, P, K, keep)."""
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim != 2:
        raise ValueError("Y must be n x p (rows are observations, dc:30)")
    n, p = Y.shape
    keep = np.flatnonzero(np.count_nonzero(Y, axis=0) != 0)     # dc:31-38
    Y = Y[:, keep]
    p = keep.size                                                # dc:39
    if g < 1 or p % g or k % g:
        raise ValueError(f"P = p/g = {p}/{g} and K = k/g = {k}/{g} must be integers (dc:41)")
    return Y, n, p, p // g, k // g, keep


def preprocess_device(Y, g, k, device=0):
    """dc:29-41 with the column scan on the GPU (dcfm_count_nonzero_columns): returns
    (n, p, P, K, keep) — the kept width and index; the data itself is not copied, since
    dcfm_set_data_raw gathers the kept columns on the device through ``shard_columns``."""
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim != 2:
        raise ValueError("Y must be n x p (rows are observations, dc:30)")
    n = Y.shape[0]
    keep = np.flatnonzero(count_nonzero_columns(Y, device=device) != 0)    # dc:31-38
    p = keep.size                                                          # dc:39
    if g < 1 or p % g or k % g:
        raise ValueError(f"P = p/g = {p}/{g} and K = k/g = {k}/{g} must be integers (dc:41)")
    return n, p, p // g, k // g, keep


def shard_columns(keep, varind, P, s0, gl):
    """Input column of every (local shard, position) of shards [s0, s0+gl): dc:50-54's
    Y(:, varind((m-1)*P+1 : m*P)) after the zero-column removal (dc:36), 0-based, shard-major
    — the ``cols`` argument of dcfm_set_data_raw."""
    return np.asarray(keep, dtype=np.int64)[np.asarray(varind)[s0 * P:(s0 + gl) * P]]


def partition_standardize(Y, g, varind):
    """dc:48-59: Yd(:,:,m) = Y(:,varind(block m)); centre; scale by 1./sqrt(var)."""
    n, p = Y.shape
    P = p // g
    Yd = np.empty((n, P, g))
    for m in range(g):
        Yd[:, :, m] = Y[:, varind[m * P:(m + 1) * P]]
    Md = Yd.mean(axis=0, keepdims=True)
    VYd = Yd.var(axis=0, ddof=1, keepdims=True)
    if np.any(VYd == 0):
        raise ValueError("a constant non-zero column has zero variance (dc:59 would divide by zero, Q13)")
    return (Yd - Md) * (1.0 / np.sqrt(VYd))


class _HostInitDraws:
    """Standard variates for dc:50-83 from NumPy (the reference uses MATLAB's stream)."""

    def __init__(self, seed, n, p, g, K, hyper: Hyper):
        r = np.random.Generator(np.random.PCG64(np.random.SeedSequence([int(seed), 0, 0])))
        P = p // g
        self.varind = r.permutation(p)
        self.ps0 = r.standard_gamma(hyper.as_, size=(P, 1, g))
        self.X0 = r.standard_normal((n, K))
        self.psi0 = r.standard_gamma(hyper.df / 2.0, size=(P, K, g))
        self.Z0 = np.empty((n, K, g))
        self.delta0 = np.empty((K, g))
        for m in range(g):
            self.Z0[:, :, m] = r.standard_normal((n, K))
            self.delta0[0, m] = r.standard_gamma(hyper.ad1)
            if K > 1:
                self.delta0[1:, m] = r.standard_gamma(hyper.ad2, size=K - 1)


class _HostVarind:
    """dc:50 varind = randperm(p) alone (the first draw of _HostInitDraws' stream)."""

    def __init__(self, seed, p):
        r = np.random.Generator(np.random.PCG64(np.random.SeedSequence([int(seed), 0, 0])))
        self.varind = r.permutation(p)


def initial_state(n, P, K, g, rho, hyper: Hyper, init) -> dict:
    """dc:68-87 from standard variates ``init`` (fields varind, ps0, X0, psi0, Z0, delta0)."""
    ps = (1.0 / hyper.bs) * np.asarray(init.ps0)                 # dc:69
    X = np.array(init.X0, dtype=float)                           # dc:71
    psi = (2.0 / hyper.df) * np.asarray(init.psi0)               # dc:73
    Z = np.array(init.Z0, dtype=float)                           # dc:80
    delta = np.empty((K, 1, g))
    delta[0, 0, :] = hyper.bd1 * init.delta0[0, :]               # dc:83
    delta[1:, 0, :] = hyper.bd2 * init.delta0[1:, :]
    tauh = np.cumprod(delta, axis=0)                             # dc:85 (per shard)
    Plam = psi * np.transpose(tauh, (1, 0, 2))                   # dc:86
    eta = np.sqrt(rho) * X[:, :, None] + np.sqrt(1 - rho) * Z   # dc:81
    return {
        "Lambda": np.zeros((P, K, g)), "ps": ps, "omega": ps[:, 0, :].copy(),   # dc:70,84 (Q1)
        "psi": psi, "Plam": Plam, "X": X, "Z": Z, "eta": eta, "delta": delta, "tauh": tauh,
    }


def local_state(state: dict, s0: int, gl: int) -> dict:
    """Slice the per-shard fields to shards [s0, s0+gl); X, delta, tauh stay whole."""
    out = {}
    for f, a in state.items():
        if f in ("X", "delta", "tauh"):
            out[f] = a
        else:
            out[f] = a[..., s0:s0 + gl]
    return out


def divideconquer(Y, g, k, BURNIN, MCMC, thin, rho, *, seed=0, hyper: Hyper = Hyper(),
                  init_draws=None, iter_draws=None, nranks=1, rank=0, device=0, comm_uid=None,
                  asm_batch=0, return_info=False, device_ingest=True, device_init=True):
    """Sigmaout = divideconquer(Y,g,k,BURNIN,MCMC,thin,rho)   (divideconquer.m:1).

    ``device_ingest`` (default): the zero-column scan and the partition/standardisation
    (dc:31-59) run on the GPU (dcfm_count_nonzero_columns, dcfm_set_data_raw); False
    keeps them on the host (NumPy) and uploads Yd.  ``device_init`` (default, unless
    ``init_draws`` are injected): the initial state of dc:68-87 is drawn on the GPU from
    the Philox stream (dcfm_init_state); only varind (dc:50) is drawn on the host.

    Multi-GPU: call on every rank with the same arguments plus nranks/rank/device
    and the 128-byte RCCL id (``Sampler.unique_id()`` on rank 0, broadcast by
    the caller).  Every rank returns the full Sigmaout.
    """
    t0 = time.perf_counter()                                     # dc:29 tic
    if device_ingest:
        Y = np.asarray(Y, dtype=np.float64)
        n, p, P, K, keep = preprocess_device(Y, g, k, device=device)
    else:
        Yk, n, p, P, K, keep = preprocess(Y, g, k)
    N = BURNIN + MCMC                                            # dc:45
    on_device_init = device_init and init_draws is None
    if init_draws is not None:
        init = init_draws
    elif on_device_init:                                         # dc:50 only; dc:68-87 on the GPU
        init = _HostVarind(seed, p)
    else:
        init = _HostInitDraws(seed, n, p, g, K, hyper)
    if not device_ingest:
        Yd = partition_standardize(Yk, g, np.asarray(init.varind))
    state = None if on_device_init else initial_state(n, P, K, g, rho, hyper, init)
    gl = g // nranks
    s0 = rank * gl
    smp = Sampler(n, P, g, K, rho, BURNIN, MCMC, thin, hyper=hyper, seed=seed, nranks=nranks,
                  rank=rank, device=device, inject_draws=iter_draws is not None, asm_batch=asm_batch)
    try:
        if nranks > 1:
            if comm_uid is None:
                raise ValueError("nranks > 1 needs comm_uid (Sampler.unique_id() from rank 0)")
            smp.comm_init(comm_uid)
        if device_ingest:                                        # dc:48-59 on the device
            smp.set_data_raw(Y, shard_columns(keep, init.varind, P, s0, gl))
        else:
            smp.set_data(Yd[:, :, s0:s0 + gl])
        if state is None:
            smp.init_state()
        else:
            smp.set_state(local_state(state, s0, gl))
        if iter_draws is not None:
            smp.set_draws(iter_draws, 1, N)
        smp.run(1, N)                                            # dc:90-197
        Sigmaout = smp.get_sigma()
    finally:
        smp.close()
    elapsed = time.perf_counter() - t0                           # dc:200 toc
    if return_info:
        return Sigmaout, {"varind": np.asarray(init.varind), "keep": keep, "n": n, "p": p, "P": P,
                          "K": K, "N": N, "seconds": elapsed}
    return Sigmaout


def truth_factors(Lam0, sig2, Y, keep, varind):
    """Truth Sigma0 = Lam0 Lam0' + diag(sig2) as (U, s) in Sigmaout's coordinates: kept
    columns (dc:36-39), permuted by varind (dc:50-54), standardised by the sample
    standard deviations (dc:57-59), so Sigma0_out = U U' + diag(s) — the low-rank form
    dcfm_sigma_error takes."""
    Y = np.asarray(Y, dtype=np.float64)
    cols = np.asarray(keep)[np.asarray(varind)]
    sd = Y[:, cols].std(axis=0, ddof=1)
    U = np.asarray(Lam0, dtype=np.float64)[cols] / sd[:, None]
    s = np.asarray(sig2, dtype=np.float64)[cols] / (sd * sd)
    return U, s


def output_columns(keep, varind):
    """Input column index of each Sigmaout row/column: kept columns (dc:36-39) in the
    varind order of the partition (dc:50-54) — Sigmaout's coordinates (quirk Q7)."""
    return np.asarray(keep)[np.asarray(varind)]


def unpermute_sigma(S, keep, varind, p_orig, sd=None, fill=0.0):
    """Sigmaout back in the input's column order: S[a, b] goes to (cols[a], cols[b]) with
    cols = output_columns(keep, varind); rows/columns of dropped (all-zero, dc:36-39)
    columns get ``fill``.  With ``sd`` (the sample standard deviations of the kept
    columns in Sigmaout's order, dc:57) the standardisation is undone: S_ab sd_a sd_b.
    The reference returns the permuted, standardised matrix and leaves this to the
    caller."""
    S = np.asarray(S, dtype=np.float64)
    cols = output_columns(keep, varind)
    if sd is not None:
        sd = np.asarray(sd, dtype=np.float64)
        S = S * sd[:, None] * sd[None, :]
    out = np.full((p_orig, p_orig), fill, dtype=np.float64)
    out[np.ix_(cols, cols)] = S
    return out
