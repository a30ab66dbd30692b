"""Vectorised restatement of the dc:90-196 sweep (TEST INFRASTRUCTURE ONLY).

Same mathematics and quirks as :mod:`oracle.dc_oracle` (see its header and
oracle/__init__.py: parity unpinned), batched over shards/rows so the host
BLAS does the work.  Uses:

* as a cross-check of the faithful loop (agreement to ~1e-12 relative);
* as the ``cpu_baseline`` in bench.py ("port", not MATLAB): it is the
  strongest CPU form of the reference algorithm we can time on the GPU box.

It operates on the same :class:`oracle.dc_oracle.SamplerState` (MATLAB shapes).
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import solve_triangular

from .dc_oracle import Hyper, SamplerState, matlab_cumprod_delta
from .draws import IterDraws


def _sym_upper(A):
    return np.triu(A) + np.swapaxes(np.triu(A, 1), -1, -2)


def _batched_tri_solve(L, B, lower: bool, trans: bool = False):
    """Solve op(L) x = b for a stack of triangular L (..., K, K), b (..., K)."""
    M = np.swapaxes(L, -1, -2) if trans else L
    return np.linalg.solve(M, B[..., None])[..., 0]


def update_Z(st: SamplerState, Yd, rho, d: IterDraws):
    """dc:97-108, batched over rows."""
    n, P, g = Yd.shape
    K = st.Lambda.shape[1]
    for m in range(g):
        Lam = st.Lambda[:, :, m]
        Zmsg = Lam * st.omega[:, m][:, None]
        Zprec = np.eye(K) + (1 - rho) * (Zmsg.T @ Lam)
        R = np.linalg.cholesky(_sym_upper(Zprec)).T                       # cholcov: upper
        Rz = Yd[:, :, m] - X_times(st.X, np.sqrt(rho) * Lam)             # n x P
        bz = np.sqrt(1 - rho) * (Rz @ Zmsg)                              # n x K
        vz = solve_triangular(R, bz.T, lower=False)                      # R \ b   (K x n)
        mz = solve_triangular(R.T, vz, lower=True)                       # R' \ v  (Q2)
        yz = solve_triangular(R.T, d.NZ[:, :, m], lower=True)
        st.Z[:, :, m] = (mz + yz).T


def X_times(X, LamScaled):
    return X @ LamScaled.T


def update_X(st: SamplerState, Yd, rho, d: IterDraws):
    """dc:111-129, batched over rows (cross-shard sums kept)."""
    n, P, g = Yd.shape
    K = st.Lambda.shape[1]
    LamW = st.Lambda * st.omega[:, None, :]                              # P x K x g
    sumx1 = np.einsum("pkm,plm->kl", LamW, st.Lambda)
    Xprec = g * np.eye(K) + rho * sumx1
    R = np.linalg.cholesky(_sym_upper(Xprec)).T
    sumx2 = np.zeros((n, K))
    for m in range(g):
        Rx = Yd[:, :, m] - st.Z[:, :, m] @ (np.sqrt(1 - rho) * st.Lambda[:, :, m]).T
        sumx2 += Rx @ LamW[:, :, m]
    bx = np.sqrt(rho) * sumx2
    vx = solve_triangular(R, bx.T, lower=False)
    mx = solve_triangular(R.T, vx, lower=True)
    yx = solve_triangular(R.T, d.NX, lower=True)
    st.X[:, :] = (mx + yx).T


def update_eta(st: SamplerState, rho):
    st.eta[...] = np.sqrt(rho) * st.X[:, :, None] + np.sqrt(1 - rho) * st.Z


def update_Lambda(st: SamplerState, Yd, d: IterDraws):
    """dc:136-146, all rows of all shards in one batched Cholesky."""
    n, P, g = Yd.shape
    K = st.Lambda.shape[1]
    E = np.einsum("nkm,nlm->mkl", st.eta, st.eta)                       # g x K x K
    C = np.einsum("nkm,npm->mpk", st.eta, Yd)                           # g x P x K
    ps = st.ps[:, 0, :].T                                               # g x P
    Q = ps[:, :, None, None] * E[:, None, :, :]
    idx = np.arange(K)
    Q[:, :, idx, idx] += np.moveaxis(st.Plam, 2, 0)                     # g x P x K
    b = ps[:, :, None] * C
    L = np.linalg.cholesky(Q)
    v = _batched_tri_solve(L, b, lower=True)
    mlam = _batched_tri_solve(L, v, lower=False, trans=True)
    z = np.moveaxis(d.NL, (0, 1, 2), (2, 1, 0))                         # g x P x K
    ylam = _batched_tri_solve(L, z, lower=False, trans=True)
    st.Lambda[...] = np.moveaxis(ylam + mlam, 0, 2)


def update_psi(st: SamplerState, hyper: Hyper, d: IterDraws):
    tau = st.tauh[:, 0, :][None, :, :]                                  # 1 x K x g
    scale = 1.0 / (hyper.df / 2 + 0.5 * (st.Lambda ** 2 * tau))
    st.psi[...] = scale * d.Gpsi


def update_delta_tau(st: SamplerState, hyper: Hyper, d: IterDraws):
    """dc:154-165: the sequential chain is scalar work; kept as in the faithful loop."""
    P, K, g = st.Lambda.shape
    colsum = (st.psi * st.Lambda ** 2).sum(axis=0)                      # K x g
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


def update_ps(st: SamplerState, Yd, hyper: Hyper, d: IterDraws):
    n, P, g = Yd.shape
    for m in range(g):
        Ytil = Yd[:, :, m] - st.eta[:, :, m] @ st.Lambda[:, :, m].T
        st.ps[:, 0, m] = (1.0 / (hyper.bs + 0.5 * np.einsum("ij,ij->j", Ytil, Ytil))) * d.Gps[:, m]
    st.omega[...] = 1.0 / st.ps[:, 0, :]


def update_Plam(st: SamplerState):
    st.Plam[...] = st.psi * st.tauh[:, 0, :][None, :, :]


def gibbs_iteration(st: SamplerState, Yd, rho, hyper: Hyper, d: IterDraws):
    update_Z(st, Yd, rho, d)
    update_X(st, Yd, rho, d)
    update_eta(st, rho)
    update_Lambda(st, Yd, d)
    update_psi(st, hyper, d)
    update_delta_tau(st, hyper, d)
    update_ps(st, Yd, hyper, d)
    update_Plam(st)
    return st


def assemble_into(Sigmaout, st: SamplerState, rho, effsamp):
    """dc:182-195 as one GEMM: rho*L*L' + (1-rho)*blkdiag(L_r L_r') + diag(omega)."""
    P, K, g = st.Lambda.shape
    L = np.moveaxis(st.Lambda, 2, 0).reshape(P * g, K)
    Sigma = (rho * L) @ L.T
    for r in range(g):
        s = slice(r * P, (r + 1) * P)
        Lr = st.Lambda[:, :, r]
        Sigma[s, s] = Lr @ Lr.T + np.diag(st.omega[:, r])
    Sigmaout += Sigma / effsamp
    Sigmaout += Sigmaout.T
    Sigmaout *= 0.5
    return Sigmaout


def run_chain(Yd, st: SamplerState, rho, hyper: Hyper, draws, first_iter, n_iter,
              burnin, mcmc, thin, Sigmaout=None):
    n, P, g = Yd.shape
    effsamp = mcmc / thin
    if Sigmaout is None:
        Sigmaout = np.zeros((P * g, P * g))
    for it in range(first_iter, first_iter + n_iter):
        gibbs_iteration(st, Yd, rho, hyper, draws(it))
        if it % thin == 0 and it > burnin:
            Sigmaout = assemble_into(Sigmaout, st, rho, effsamp)
    return Sigmaout
