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


def loading_backward_error(lam_mat, Q, b, L, z):
    """Per-row backward error of a loading draw (dc:142-144): the exact draw solves
    Q_j lam_j = b_j + L_j z_j, so || Q_j lam_j - b_j - L_j z_j || / (||Q_j|| ||lam_j|| + ||b_j||
    + ||L_j|| ||z_j||) is ~ machine epsilon for any backward-stable solve, whatever cond(Q_j).
    lam_mat: P x K x g (MATLAB layout); the systems g x P x ... (oracle.vectorised.loading_systems).
    Returns the worst row."""
    lam = np.moveaxis(np.asarray(lam_mat, dtype=np.float64), 2, 0)          # g x P x K
    r = np.einsum("mjkl,mjl->mjk", Q, lam) - b - np.einsum("mjkl,mjl->mjk", L, z)
    nq = np.linalg.norm(Q, axis=(-2, -1), ord=2)
    nl = np.linalg.norm(L, axis=(-2, -1), ord=2)
    den = nq * np.linalg.norm(lam, axis=-1) + np.linalg.norm(b, axis=-1) + nl * np.linalg.norm(z, axis=-1)
    return float(np.max(np.linalg.norm(r, axis=-1) / den))


def stagewise_errors(start, got, Yd, rho, hyper, draws, check_lambda=None):
    """Stage-wise parity of one Gibbs iteration (absolute bars, no comparison of two
    implementations' rounding): from the oracle state `start` at the iteration's start,
      * the stages before the loading solve (Z, X, eta; dc:97-134) vs the oracle's, relative;
      * the loading draw (dc:137-144) as the per-row backward error of got's Lambda against the
        oracle's systems (Q_j, b_j, L_j, z_j) built from got's eta -- cond(Q_j) reaches ~1e7 at
        c1/c2, where two restatements' forward errors differ by cond x eps (see
        tests/test_gpu_parity_configs.py);
      * every later stage (psi, delta/tau, Plam; dc:149-165, 174-177) vs the oracle update applied
        to got's own Lambda, relative;
      * ps, omega (dc:168-172) per row, unscaled relative, vs the faithful loop's update
        (oracle/dc_oracle.py update_ps: the reference's direct residual Yd - eta Lambda') applied
        to got's own eta and Lambda.  The library meets this with DCFM_FLAG_EXACT_RESIDUAL at
        every shape; its default SS identity cancels where SS_j is small against its terms
        (resid.hip header), e.g. 1.3e-10 at config c2's second iteration.
    `got` maps state fields to MATLAB-layout arrays (Sampler.get_state, or an oracle state's
    as_dict()).  Returns ({field: rel err}, lambda backward error, the oracle state after the
    iteration with got's Lambda)."""
    from oracle import vectorised as V
    D = V._as_data(Yd)
    st = start.copy()
    V.update_ZX(st, D, rho, draws)
    V.update_eta(st, rho)
    errs = {f: rel_err(got[f], getattr(st, f)) for f in ("X", "Z", "eta")}
    for f in ("X", "Z", "eta"):        # the later stages from got's own inputs
        getattr(st, f)[...] = np.asarray(got[f], dtype=np.float64).reshape(getattr(st, f).shape)
    E, C, Q, b, L, z = V.loading_systems(st, D, draws)
    bw = loading_backward_error(got["Lambda"], Q, b, L, z)
    V.update_Lambda_psi_delta_ps(st, D, hyper, draws, lam_given=got["Lambda"])
    V.update_Plam(st)
    for f in ("psi", "delta", "tauh", "Plam"):
        errs[f] = rel_err(got[f], getattr(st, f))
    F.update_ps(st, D.Yd, hyper, draws)      # dc:169-171 as written, on got's eta and Lambda
    for f in ("ps", "omega"):
        errs[f] = elem_rel_err(got[f], getattr(st, f))
    return errs, bw, st


def elem_rel_err(a, b):
    """max_i |a_i - b_i| / |b_i| (per element, unscaled)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64).reshape(a.shape)
    return float(np.max(np.abs(a - b) / np.abs(b))) if b.size else 0.0


def residual_rounding_bound(got, Yd):
    """Per-row bound on the rounding error of dc:169's residual evaluation at the state `got` (MATLAB
    layout), relative to ps_j: Ytil_ij = Yd_ij - sum_k eta_ik Lambda_jk carries |delta_ij| <= (K + 1) eps
    M_ij, M_ij = |Yd_ij| + sum_k |eta_ik Lambda_jk|, so SS_j = sum_i Ytil_ij^2 carries <= 2 (K + 1) eps
    sum_i |Ytil_ij| M_ij, and ps_j = Gps / (bs + SS_j / 2) at most the same relative error.  Two correct
    evaluations (any summation order) differ by at most twice that.  Returns g x P (the ps layout's
    shards x rows); ~1e-14 at a stationary state, far larger inside the reference's X excursions, where
    eta Lambda' cancels against Yd."""
    from oracle import vectorised as V
    D = V._as_data(Yd)
    eta = np.moveaxis(np.asarray(got["eta"], dtype=np.float64), 2, 0)          # g x n x K
    lam = np.moveaxis(np.asarray(got["Lambda"], dtype=np.float64), 2, 0)       # g x P x K
    K = lam.shape[-1]
    R = D.Ys - eta @ np.swapaxes(lam, 1, 2)
    M = np.abs(D.Ys) + np.abs(eta) @ np.swapaxes(np.abs(lam), 1, 2)
    SS = np.einsum("mij,mij->mj", R, R)
    return 4.0 * (K + 1) * np.finfo(np.float64).eps * np.einsum("mij,mij->mj", np.abs(R), M) / SS


def scaled_rel_err(a, b, bound, tol):
    """max_i |a_i - b_i| / |b_i| / max(tol, bound_i) * tol: the per-element relative error, each measured
    against the larger of tol and that element's own rounding bound (< tol passes)."""
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    bd = np.maximum(tol, np.asarray(bound, dtype=np.float64).reshape(-1))
    return float(np.max(np.abs(a - b) / np.abs(b) / bd) * tol) if b.size else 0.0
