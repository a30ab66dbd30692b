"""Faithful-loop restatement of divideconquer.m (TEST INFRASTRUCTURE ONLY).

Header, scope and parity status: see oracle/__init__.py (parity unpinned: no
MATLAB/Octave here, no reference fixtures).  ``dc:L`` = line L of the
reference's ``divideconquer.m``.

Arrays keep the reference's MATLAB shapes (``Lambda`` is P x K x g, ``Yd`` is
n x P x g, ...) so every line below reads like the line it restates.  Loops
over shards, rows and factor indices are kept where the reference loops, and
scalar*matrix*vector products are evaluated left to right as MATLAB does.
Random variates come from an injected :class:`oracle.draws.IterDraws`.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

import numpy as np
from scipy.linalg import solve_triangular

from .draws import DrawSource, InitDraws, IterDraws


@dataclass(frozen=True)
class Hyper:
    """Hard-coded hyper-parameters, dc:62-65."""
    as_: float = 1.0   # dc:62 (``as`` is a Python keyword)
    bs: float = 0.3    # dc:62
    df: float = 3.0    # dc:63
    ad1: float = 2.0   # dc:64
    bd1: float = 1.0   # dc:64
    ad2: float = 2.0   # dc:65
    bd2: float = 1.0   # dc:65


@dataclass
class SamplerState:
    """The hot loop's read/write set, MATLAB shapes.

    ``omega`` is diag(Omega) (dc:75,84,171): the reference keeps a dense P x P
    matrix and only ever uses its diagonal.  Quirk Q1: it holds ``ps`` at init
    (dc:84) and ``1./ps`` after every ps-update (dc:171).
    """
    Lambda: np.ndarray  # P x K x g
    ps: np.ndarray      # P x 1 x g
    omega: np.ndarray   # P x g
    psi: np.ndarray     # P x K x g   (psijh)
    Plam: np.ndarray    # P x K x g
    X: np.ndarray       # n x K
    Z: np.ndarray       # n x K x g
    eta: np.ndarray     # n x K x g
    delta: np.ndarray   # K x 1 x g
    tauh: np.ndarray    # K x 1 x g

    def copy(self) -> "SamplerState":
        return SamplerState(**{k: np.array(v, copy=True) for k, v in self.__dict__.items()})

    def as_dict(self) -> dict:
        return dict(self.__dict__)


# ---------------------------------------------------------------------------
# MATLAB built-in semantics used by the reference
# ---------------------------------------------------------------------------

def cholcov(A: np.ndarray) -> np.ndarray:
    """MATLAB ``cholcov`` for a symmetric positive-definite A (dc:100,118).

    Returns the UPPER factor R with R'R = A, computed by ``chol`` on the upper
    triangle.  MATLAB returns [] when A is asymmetric beyond
    n*10*eps(max|diag|); the reference would then fail at ``Lz\\bz``, so we raise.
    """
    n = A.shape[0]
    tol = 10.0 * np.spacing(np.max(np.abs(np.diag(A))))
    if not np.all(np.abs(A - A.T) < n * tol):
        raise ValueError("cholcov: matrix not symmetric within tolerance (reference returns [])")
    U = np.triu(A)
    S = U + np.triu(A, 1).T
    return np.linalg.cholesky(S).T


def chol_lower(A: np.ndarray) -> np.ndarray:
    """MATLAB ``chol(A,'lower')`` (dc:142): uses the lower triangle of A."""
    Lo = np.tril(A)
    S = Lo + np.tril(A, -1).T
    return np.linalg.cholesky(S)


def matlab_cumprod_delta(delta: np.ndarray) -> np.ndarray:
    """``cumprod(delta)`` on the K x 1 x g array (dc:158), quirk Q5.

    MATLAB runs cumprod along the first non-singleton dimension: the factor
    dimension when K >= 2, the shard dimension when K == 1 and g > 1.
    """
    K, _, g = delta.shape
    if K > 1:
        return np.cumprod(delta, axis=0)
    if g > 1:
        return np.cumprod(delta, axis=2)
    return delta.copy()


# ---------------------------------------------------------------------------
# Driver half (dc:29-87) — stays on the host in the product as well
# ---------------------------------------------------------------------------

def preprocess(Y: np.ndarray, g: int, k: int):
    """dc:29-42: drop all-zero columns; P = p/g, K = k/g must be integral."""
    Y = np.asarray(Y, dtype=np.float64)
    n, p = Y.shape                                   # dc:30
    nnzcol = np.count_nonzero(Y, axis=0)             # dc:31-34
    keep = np.flatnonzero(nnzcol != 0)               # dc:36,38 setdiff(1:p, zerocol)
    Y = Y[:, keep]
    p = keep.size                                    # dc:39
    if p % g or k % g:
        raise ValueError(f"P = p/g = {p}/{g} and K = k/g = {k}/{g} must be integers (dc:41)")
    return Y, n, p, p // g, k // g, keep


def partition(Y: np.ndarray, g: int, varind: np.ndarray) -> np.ndarray:
    """dc:48-54: Yd(:,:,m) = Y(:, varind((m-1)P+1 : mP))."""
    n, p = Y.shape
    P = p // g
    Yd = np.zeros((n, P, g))
    for m in range(g):
        Yd[:, :, m] = Y[:, varind[m * P:(m + 1) * P]]
    return Yd


def standardize(Yd: np.ndarray) -> np.ndarray:
    """dc:56-59: centre each column, scale by 1./sqrt(var) (n-1 normalisation)."""
    Md = Yd.mean(axis=0, keepdims=True)
    VYd = Yd.var(axis=0, ddof=1, keepdims=True)
    Yd = Yd - Md
    return Yd * (1.0 / np.sqrt(VYd))


def initialise(n: int, P: int, K: int, g: int, rho: float, hyper: Hyper,
               init: InitDraws) -> SamplerState:
    """dc:68-87 with injected standard variates."""
    ps = (1.0 / hyper.bs) * init.ps0                       # dc:69 gamrnd(as,1/bs)
    Lambda = np.zeros((P, K, g))                           # dc:70
    eta = np.zeros((n, K, g))
    Z = np.zeros((n, K, g))                                # dc:71
    X = np.array(init.X0, dtype=float, copy=True)
    psi = (2.0 / hyper.df) * init.psi0                     # dc:73 gamrnd(df/2,2/df)
    delta = np.zeros((K, 1, g))                            # dc:74
    omega = np.zeros((P, g))                               # dc:75
    tauh = np.zeros((K, 1, g))                             # dc:76
    Plam = np.zeros((P, K, g))                             # dc:77
    for m in range(g):                                     # dc:79
        Z[:, :, m] = init.Z0[:, :, m]                      # dc:80
        eta[:, :, m] = np.sqrt(rho) * X + np.sqrt(1 - rho) * Z[:, :, m]   # dc:81
        d = np.empty(K)
        d[0] = hyper.bd1 * init.delta0[0, m]               # dc:83 gamrnd(ad1,bd1)
        d[1:] = hyper.bd2 * init.delta0[1:, m]             # dc:83 gamrnd(ad2,bd2,[K-1,1])
        delta[:, 0, m] = d
        omega[:, m] = ps[:, 0, m]                          # dc:84 Omega = diag(ps)  (Q1)
        tauh[:, 0, m] = np.cumprod(delta[:, 0, m])         # dc:85
        Plam[:, :, m] = psi[:, :, m] * tauh[:, 0, m][None, :]   # dc:86
    return SamplerState(Lambda, ps, omega, psi, Plam, X, Z, eta, delta, tauh)


# ---------------------------------------------------------------------------
# Hot loop body (dc:90-178) — what the HIP library replaces
# ---------------------------------------------------------------------------

def update_Z(st: SamplerState, Yd, rho, d: IterDraws):
    """dc:97-108: shard-specific factor Z (quirk Q2: R'\\(R\\b) with upper R)."""
    n, P, g = Yd.shape
    K = st.Lambda.shape[1]
    for m in range(g):
        Lam = st.Lambda[:, :, m]
        om = st.omega[:, m]
        Zmsg = Lam * om[:, None]                                   # dc:98
        Zprec = np.eye(K) + ((1 - rho) * Zmsg.T) @ Lam             # dc:99
        Lz = cholcov(Zprec)                                        # dc:100
        for i in range(n):                                         # dc:101
            Rz = Yd[i, :, m] - (np.sqrt(rho) * Lam) @ st.X[i, :]   # dc:102
            bz = (np.sqrt(1 - rho) * Zmsg.T) @ Rz                  # dc:103
            vz = solve_triangular(Lz, bz, lower=False)             # dc:104 Lz\bz
            mz = solve_triangular(Lz.T, vz, lower=True)            # dc:104 Lz'\vz
            zz = d.NZ[:, i, m]                                     # dc:104 normrnd
            yz = solve_triangular(Lz.T, zz, lower=True)            # dc:105
            st.Z[i, :, m] = mz + yz                                # dc:106


def update_X(st: SamplerState, Yd, rho, d: IterDraws):
    """dc:111-129: shared factor X; prior term g*I (Q3); sums over all shards."""
    n, P, g = Yd.shape
    K = st.Lambda.shape[1]
    sumx1 = 0.0                                                    # dc:112
    for m in range(g):                                             # dc:113
        Xmsg = st.Lambda[:, :, m] * st.omega[:, m][:, None]        # dc:114
        sumx1 = sumx1 + Xmsg.T @ st.Lambda[:, :, m]                # dc:115
    Xprec = g * np.eye(K) + rho * sumx1                            # dc:117
    Lx = cholcov(Xprec)                                            # dc:118
    for i in range(n):                                             # dc:119
        sumx2 = 0.0                                                # dc:120
        for m in range(g):                                         # dc:121
            Lam = st.Lambda[:, :, m]
            Rx = Yd[i, :, m] - (np.sqrt(1 - rho) * Lam) @ st.Z[i, :, m]   # dc:122
            sumx2 = sumx2 + (Lam * st.omega[:, m][:, None]).T @ Rx        # dc:123
        bx = np.sqrt(rho) * sumx2                                  # dc:125
        vx = solve_triangular(Lx, bx, lower=False)                 # dc:126
        mx = solve_triangular(Lx.T, vx, lower=True)
        zx = d.NX[:, i]
        yx = solve_triangular(Lx.T, zx, lower=True)                # dc:127
        st.X[i, :] = mx + yx                                       # dc:128


def update_eta(st: SamplerState, rho):
    """dc:131-134."""
    g = st.eta.shape[2]
    for m in range(g):
        st.eta[:, :, m] = np.sqrt(rho) * st.X + np.sqrt(1 - rho) * st.Z[:, :, m]


def update_Lambda(st: SamplerState, Yd, d: IterDraws):
    """dc:136-146: row-wise loadings; uses Plam and ps of the previous iteration (Q11)."""
    n, P, g = Yd.shape
    for m in range(g):                                             # dc:137
        eta = st.eta[:, :, m]
        eta2 = eta.T @ eta                                         # dc:138
        for j in range(P):                                         # dc:140
            Qlam = np.diag(st.Plam[j, :, m]) + st.ps[j, 0, m] * eta2     # dc:141
            blam = st.ps[j, 0, m] * (eta.T @ Yd[:, j, m])          # dc:141
            Llam = chol_lower(Qlam)                                # dc:142
            zlam = d.NL[:, j, m]                                   # dc:142
            vlam = solve_triangular(Llam, blam, lower=True)        # dc:143
            mlam = solve_triangular(Llam.T, vlam, lower=False)
            ylam = solve_triangular(Llam.T, zlam, lower=False)
            st.Lambda[j, :, m] = ylam + mlam                       # dc:144


def update_psi(st: SamplerState, hyper: Hyper, d: IterDraws):
    """dc:148-152: psi_jh = (1./(df/2 + 0.5*lambda^2*tau_h)) .* randg(df/2+0.5)."""
    g = st.psi.shape[2]
    for m in range(g):
        scale = 1.0 / (hyper.df / 2 + 0.5 * (st.Lambda[:, :, m] ** 2 * st.tauh[:, 0, m][None, :]))
        st.psi[:, :, m] = scale * d.Gpsi[:, :, m]


def update_delta_tau(st: SamplerState, hyper: Hyper, d: IterDraws):
    """dc:154-165 with quirks Q4 (``delta(h)`` = shard 1's delta_h) and Q5 (cumprod dim)."""
    P, K, g = st.Lambda.shape
    delta, tauh = st.delta, st.tauh
    for m in range(g):                                             # dc:155
        mat = st.psi[:, :, m] * st.Lambda[:, :, m] ** 2            # dc:156
        colsum = mat.sum(axis=0)
        bd = hyper.bd1 + (0.5 * (1.0 / delta[0, 0, m])) * np.sum(tauh[:, 0, m] * colsum)  # dc:157
        delta[0, 0, m] = (1.0 / bd) * d.Gdelta[0, m]               # dc:158 gamrnd(ad,1/bd)
        tauh[...] = matlab_cumprod_delta(delta)                    # dc:158 (Q5)
        for h in range(1, K):                                      # dc:160
            bd = hyper.bd2 + (0.5 * (1.0 / delta[h, 0, 0])) * np.sum(   # dc:161 delta(h) (Q4)
                tauh[h:, 0, m] * colsum[h:])
            delta[h, 0, m] = (1.0 / bd) * d.Gdelta[h, m]           # dc:163
            tauh[:, :, m] = np.cumprod(delta[:, :, m], axis=0)     # dc:163


def update_ps(st: SamplerState, Yd, hyper: Hyper, d: IterDraws):
    """dc:167-172: residual precision; Omega becomes diag(1./ps) (Q1)."""
    n, P, g = Yd.shape
    for m in range(g):
        Ytil = Yd[:, :, m] - st.eta[:, :, m] @ st.Lambda[:, :, m].T     # dc:169
        scale = 1.0 / (hyper.bs + 0.5 * np.sum(Ytil ** 2, axis=0))     # dc:170
        st.ps[:, 0, m] = scale * d.Gps[:, m]
        st.omega[:, m] = 1.0 / st.ps[:, 0, m]                      # dc:171


def update_Plam(st: SamplerState):
    """dc:174-177."""
    g = st.psi.shape[2]
    for m in range(g):
        st.Plam[:, :, m] = st.psi[:, :, m] * st.tauh[:, 0, m][None, :]


def gibbs_iteration(st: SamplerState, Yd, rho, hyper: Hyper, d: IterDraws,
                    snapshots: dict | None = None):
    """One pass of dc:93-177.  Optionally records a copy after every update."""
    steps = (
        ("Z", lambda: update_Z(st, Yd, rho, d)),
        ("X", lambda: update_X(st, Yd, rho, d)),
        ("eta", lambda: update_eta(st, rho)),
        ("Lambda", lambda: update_Lambda(st, Yd, d)),
        ("psi", lambda: update_psi(st, hyper, d)),
        ("delta", lambda: update_delta_tau(st, hyper, d)),
        ("ps", lambda: update_ps(st, Yd, hyper, d)),
        ("Plam", lambda: update_Plam(st)),
    )
    for name, fn in steps:
        fn()
        if snapshots is not None:
            snapshots[name] = st.copy()
    return st


def assemble_sample(st: SamplerState, rho) -> np.ndarray:
    """dc:182-192: Sigma blocks  Lambda_r Lambda_r' + Omega_r  /  rho Lambda_r Lambda_c'."""
    P, K, g = st.Lambda.shape
    p = P * g
    Sigma = np.zeros((p, p))
    for rind in range(g):
        for cind in range(g):
            rs = slice(rind * P, (rind + 1) * P)
            cs = slice(cind * P, (cind + 1) * P)
            if rind == cind:
                Sigma[rs, cs] = st.Lambda[:, :, rind] @ st.Lambda[:, :, rind].T + np.diag(st.omega[:, rind])
            else:
                Sigma[rs, cs] = (rho * st.Lambda[:, :, rind]) @ st.Lambda[:, :, cind].T
    return Sigma


def run_chain(Yd, st: SamplerState, rho, hyper: Hyper, draws, first_iter: int, n_iter: int,
              burnin: int, mcmc: int, thin: int, Sigmaout=None, record=None):
    """dc:90-197 for iterations first_iter .. first_iter+n_iter-1 (1-based).

    ``draws`` is a callable it -> IterDraws.  ``record`` (list) receives a copy
    of the state after each iteration.  Returns Sigmaout.
    """
    n, P, g = Yd.shape
    effsamp = (burnin + mcmc - burnin) / thin                      # dc:45 (Q8)
    if Sigmaout is None:
        Sigmaout = np.zeros((P * g, P * g))                        # dc:42
    for it in range(first_iter, first_iter + n_iter):              # dc:90
        gibbs_iteration(st, Yd, rho, hyper, draws(it))
        if it % thin == 0 and it > burnin:                         # dc:180
            Sigma = assemble_sample(st, rho)
            Sigmaout = Sigmaout + Sigma / effsamp                  # dc:194
            Sigmaout = (Sigmaout + Sigmaout.T) / 2                 # dc:195 (Q9)
        if record is not None:
            record.append(st.copy())
    return Sigmaout


def divideconquer(Y, g, k, BURNIN, MCMC, thin, rho, seed=0, hyper: Hyper = Hyper(),
                  return_all=False):
    """Whole reference function (dc:1-201) with a seeded injected draw source."""
    Y, n, p, P, K, keep = preprocess(Y, g, k)
    src = DrawSource(seed, n, p, g, K, hyper)
    init = src.init()
    Yd = standardize(partition(Y, g, init.varind))
    st = initialise(n, P, K, g, rho, hyper, init)
    Sigmaout = run_chain(Yd, st, rho, hyper, src.iteration, 1, BURNIN + MCMC, BURNIN, MCMC, thin)
    if return_all:
        return Sigmaout, dict(Yd=Yd, state=st, varind=init.varind, keep=keep, n=n, p=p, P=P, K=K)
    return Sigmaout
