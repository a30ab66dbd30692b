"""Vectorised restatement of the dc:90-196 sweep (TEST INFRASTRUCTURE ONLY).

Same mathematics and quirks as :mod:`oracle.dc_oracle` (see its header and
oracle/__init__.py: parity unpinned), batched over shards/rows so the host
BLAS does the work.  Uses:

* as a cross-check of the faithful loop (agreement to ~1e-12 relative), which
  also checks the algebraic identities below (the HIP kernels use them too);
* as the ``cpu_baseline`` in bench.py ("port", not MATLAB): the strongest CPU
  form of the reference algorithm we can time on the GPU box.

Identities used (exact in real arithmetic; rounding-level differences only):
  Zmsg' (Y_i - sqrt(rho) L X_i)  = W_i - sqrt(rho) A X_i           W = Y (w o L), A = (w o L)' L
  sum_m Xmsg'(Y_i - sqrt(1-rho) L Z_i) = sum_m W_i - sqrt(1-rho) A' Z_i ... (A' = L'(w o L))
  sum_i (Y_ij - eta_i L_j')^2 = yy_j - 2 L_j.C_j + L_j E L_j'      C = eta'Y, E = eta'eta
  Sigma = rho L L' + (1-rho) blkdiag(L_r L_r') + diag(w)           (dc:184-192 block loop)

It operates on the same :class:`oracle.dc_oracle.SamplerState` (MATLAB shapes);
``Ys`` is the shard-major contiguous copy of Yd (g x n x P).
"""
from __future__ import annotations

import numpy as np
from scipy.linalg.blas import dsyrk, dtrsv

from .dc_oracle import Hyper, SamplerState, matlab_cumprod_delta
from .draws import IterDraws


class Data:
    """Yd in shard-major contiguous layout + per-column sums of squares."""

    def __init__(self, Yd):
        self.Yd = Yd
        self.Ys = np.ascontiguousarray(np.moveaxis(Yd, 2, 0))        # g x n x P
        self.yy = np.einsum("mij,mij->mj", self.Ys, self.Ys)          # g x P


def _as_data(Yd):
    return Yd if isinstance(Yd, Data) else Data(Yd)


def _chol_upper_from_upper(A):
    """cholcov on a stack (..., K, K): upper factor from the upper triangle."""
    S = np.triu(A) + np.swapaxes(np.triu(A, 1), -1, -2)
    return np.swapaxes(np.linalg.cholesky(S), -1, -2)


def _solve(M, B):
    return np.linalg.solve(M, B)


def update_ZX(st: SamplerState, D: Data, rho, d: IterDraws):
    """dc:97-129 (Z then X), Y read once for W."""
    g, n, P = D.Ys.shape
    K = st.Lambda.shape[1]
    Lg = np.ascontiguousarray(np.moveaxis(st.Lambda, 2, 0))         # g x P x K
    w = st.omega.T                                                   # g x P
    Lw = Lg * w[:, :, None]                                          # Zmsg, dc:98
    A = np.swapaxes(Lw, 1, 2) @ Lg                                   # g x K x K, dc:99
    W = D.Ys @ Lw                                                    # g x n x K  (Y pass)
    # Z (dc:99-107): R = cholcov(I + (1-rho) A), Z = R'\(R\bz + eps)
    R = _chol_upper_from_upper(np.eye(K)[None] + (1 - rho) * A)
    bz = np.sqrt(1 - rho) * (W - np.sqrt(rho) * (st.X[None] @ np.swapaxes(A, 1, 2)))   # g x n x K
    v = _solve(R, np.swapaxes(bz, 1, 2))                             # g x K x n
    eps = np.moveaxis(d.NZ, 2, 0)                                    # g x K x n
    Z = _solve(np.swapaxes(R, 1, 2), v + eps)                        # g x K x n
    st.Z[...] = np.moveaxis(np.swapaxes(Z, 1, 2), 0, 2)
    # X (dc:112-128)
    Zg = np.swapaxes(Z, 1, 2)                                        # g x n x K
    sumx1 = A.sum(axis=0)
    Xprec = g * np.eye(K) + rho * sumx1
    Rx = _chol_upper_from_upper(Xprec)
    sumx2 = (W - np.sqrt(1 - rho) * (Zg @ np.swapaxes(A, 1, 2))).sum(axis=0)   # n x K
    bx = np.sqrt(rho) * sumx2
    vx = np.linalg.solve(Rx, bx.T)
    st.X[...] = np.linalg.solve(Rx.T, vx + d.NX).T


def update_eta(st: SamplerState, rho):
    st.eta[...] = np.sqrt(rho) * st.X[:, :, None] + np.sqrt(1 - rho) * st.Z


def loading_systems(st: SamplerState, D: Data, d: IterDraws):
    r"""The loading rows' systems of dc:137-144 from the state after the eta update:
    E (g x K x K, dc:138), C = eta'Y (g x P x K), Q_j = ps_j E + diag(Plam_j) (dc:141),
    b_j = ps_j C_j, L_j = chol(Q_j, 'lower') (dc:142) and the draws z_j (all g x P x ...).
    Lambda_j = L_j' \ (L_j \ b_j + z_j) solves Q_j Lambda_j = b_j + L_j z_j exactly."""
    D = _as_data(D)
    K = st.Lambda.shape[1]
    eta = np.ascontiguousarray(np.moveaxis(st.eta, 2, 0))          # g x n x K
    E = np.swapaxes(eta, 1, 2) @ eta                                 # g x K x K, dc:138
    C = np.swapaxes(D.Ys, 1, 2) @ eta                                # g x P x K  (Y pass)
    ps = st.ps[:, 0, :].T                                            # g x P (previous it., Q11)
    Q = ps[:, :, None, None] * E[:, None, :, :]
    idx = np.arange(K)
    Q[:, :, idx, idx] += np.moveaxis(st.Plam, 2, 0)
    b = ps[:, :, None] * C
    L = np.linalg.cholesky(Q)                                        # dc:142
    z = np.moveaxis(d.NL, (0, 1, 2), (2, 1, 0))                      # g x P x K
    return E, C, Q, b, L, z


def _loading_solve(L, b, z):
    """Lambda_j = L_j' \\ (L_j \\ b_j + z_j) (dc:143-144) for a stack of lower factors (g x P x K x K).
    Small K: batched LAPACK solves; K >= 64 (c4): two triangular solves per row (BLAS dtrsv), which
    skips the batched solver's O(K^3) factorisation of an already triangular matrix."""
    g, P, K = b.shape
    if K < 64:
        v = np.linalg.solve(L, b[..., None])[..., 0]
        return np.linalg.solve(np.swapaxes(L, -1, -2), (v + z)[..., None])[..., 0]
    lam = np.empty_like(b)
    for m in range(g):
        for j in range(P):
            Lj = L[m, j]
            v = dtrsv(Lj, b[m, j], lower=1)
            lam[m, j] = dtrsv(Lj, v + z[m, j], lower=1, trans=1)
    return lam


def residual_ss(D: Data, st: SamplerState, lam):
    """dc:169 as the reference writes it: sum_i (Yd - eta Lambda')_ij^2 per shard (g x P)."""
    g, n, P = D.Ys.shape
    SS = np.empty((g, P))
    for m in range(g):                                               # one BLAS GEMM per shard
        R = D.Ys[m] - np.ascontiguousarray(st.eta[:, :, m]) @ lam[m].T   # n x P
        SS[m] = np.einsum("ij,ij->j", R, R)
    return SS


def update_Lambda_psi_delta_ps(st: SamplerState, D: Data, hyper: Hyper, d: IterDraws, lam_given=None,
                               direct=False):
    """dc:136-172 batched; SS_j by the identity (no residual pass over Y), or with ``direct``
    by dc:169's residual (residual_ss: the library's DCFM_FLAG_EXACT_RESIDUAL).  ``lam_given``
    (P x K x g, MATLAB layout) replaces the loading draw: the rest of the update is then
    applied to that Lambda (stage-wise parity checks of an implementation's later stages)."""
    g, n, P = D.Ys.shape
    E, C, Q, b, L, z = loading_systems(st, D, d)
    if lam_given is None:
        lam = _loading_solve(L, b, z)                                # g x P x K
    else:
        lam = np.ascontiguousarray(np.moveaxis(np.asarray(lam_given, dtype=np.float64), 2, 0))
    st.Lambda[...] = np.moveaxis(lam, 0, 2)
    # psi (dc:150)
    tau = st.tauh[:, 0, :][None, :, :]
    st.psi[...] = (1.0 / (hyper.df / 2 + 0.5 * (st.Lambda ** 2 * tau))) * d.Gpsi
    # delta / tau (dc:155-165)
    update_delta_tau(st, hyper, d)
    # ps (dc:169-171): SS = yy - 2 lam.C + lam E lam'  (or the residual itself)
    if direct:
        SS = residual_ss(D, st, lam)
    else:
        SS = D.yy - 2.0 * np.einsum("mjk,mjk->mj", lam, C) + np.einsum("mjk,mkl,mjl->mj", lam, E, lam)
    st.ps[:, 0, :] = ((1.0 / (hyper.bs + 0.5 * SS)) * d.Gps.T).T
    st.omega[...] = 1.0 / st.ps[:, 0, :]


def update_delta_tau(st: SamplerState, hyper: Hyper, d: IterDraws):
    """dc:154-165: sequential scalar chain, kept as in the faithful loop (Q4, Q5)."""
    P, K, g = st.Lambda.shape
    colsum = (st.psi * st.Lambda ** 2).sum(axis=0)                   # K x g
    delta, tauh = st.delta, st.tauh
    for m in range(g):
        cs = colsum[:, m]
        bd = hyper.bd1 + (0.5 * (1.0 / delta[0, 0, m])) * np.sum(tauh[:, 0, m] * cs)
        delta[0, 0, m] = (1.0 / bd) * d.Gdelta[0, m]
        tauh[...] = matlab_cumprod_delta(delta)
        for h in range(1, K):
            bd = hyper.bd2 + (0.5 * (1.0 / delta[h, 0, 0])) * np.sum(tauh[h:, 0, m] * cs[h:])
            delta[h, 0, m] = (1.0 / bd) * d.Gdelta[h, m]
            tauh[:, :, m] = np.cumprod(delta[:, :, m], axis=0)


def update_Plam(st: SamplerState):
    st.Plam[...] = st.psi * st.tauh[:, 0, :][None, :, :]


def gibbs_iteration(st: SamplerState, Yd, rho, hyper: Hyper, d: IterDraws, direct=False):
    D = _as_data(Yd)
    update_ZX(st, D, rho, d)
    update_eta(st, rho)
    update_Lambda_psi_delta_ps(st, D, hyper, d, direct=direct)
    update_Plam(st)
    return st


def assemble_lower(SigLower, st: SamplerState, rho, effsamp):
    """dc:184-194 into the LOWER triangle of SigLower (Fortran order), via SYRK.

    Sigmaout is symmetric by construction, so the dc:195 symmetrisation is the
    identity here; the full matrix is lower + lower' - diag (see ``full``).
    """
    P, K, g = st.Lambda.shape
    L = np.asfortranarray(np.moveaxis(st.Lambda, 2, 0).reshape(P * g, K))
    SigLower[...] = dsyrk(rho / effsamp, L, beta=1.0, c=SigLower, lower=1, overwrite_c=1)
    for r in range(g):
        s = slice(r * P, (r + 1) * P)
        Lr = st.Lambda[:, :, r]
        blk = ((1 - rho) / effsamp) * (Lr @ Lr.T) + np.diag(st.omega[:, r] / effsamp)
        SigLower[s, s] += np.tril(blk)
    return SigLower


def full(SigLower):
    return np.tril(SigLower) + np.tril(SigLower, -1).T


def run_chain(Yd, st: SamplerState, rho, hyper: Hyper, draws, first_iter, n_iter,
              burnin, mcmc, thin, SigLower=None, direct=False):
    """Returns the lower-triangle accumulator (Fortran order); ``full()`` mirrors it.
    ``direct``: SS_j of dc:169 by the residual itself (see update_Lambda_psi_delta_ps)."""
    D = _as_data(Yd)
    g, n, P = D.Ys.shape
    effsamp = mcmc / thin
    if SigLower is None:
        SigLower = np.zeros((P * g, P * g), order="F")
    for it in range(first_iter, first_iter + n_iter):
        gibbs_iteration(st, D, rho, hyper, draws(it), direct=direct)
        if it % thin == 0 and it > burnin:
            assemble_lower(SigLower, st, rho, effsamp)
    return SigLower
