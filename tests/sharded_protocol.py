"""Per-rank restatement of libdcfm's multi-GPU exchange protocol (TEST INFRASTRUCTURE).

libdcfm (csrc/dcfm.hip, dcfm_run) splits the g shards of one chain over
nranks GPUs and exchanges, per iteration (the fused K <= 32 chain):
  1. all-gather of sum_{local m} (W_m - sqrt(1-rho) Z_m A_m') (n x K), summed in rank
     order -> replicated X draw  (dc:112-128)
  2. ONE all-gather of [per-shard column sums of psi o Lambda^2 (K per shard) ;
     sum_{local m} A_m of the NEXT iteration (from the new Lambda, omega; K x K)]
     -> replicated delta/tau chain over ALL shards (quirks Q4/Q5, dc:155-165) and the
     next iteration's Xprec (dc:117); before the first iteration the A sums alone
and per assembly flush an all-gather of the saved Lambda rows and omega, after
which each rank accumulates its round-robin share of lower-triangle tiles;
dcfm_get_sigma sums the per-rank accumulators (all-reduce) and mirrors.

This module runs the same decomposition with NumPy on CPU ranks connected by
torch.distributed (gloo), so tests can check that the decomposition reproduces
the single-process oracle.  It is a checker, never the product.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from oracle.dc_oracle import matlab_cumprod_delta


def all_gather_np(x: np.ndarray):
    t = torch.from_numpy(np.ascontiguousarray(x))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.numpy() for o in out]


def chol_upper(A):
    S = np.triu(A) + np.swapaxes(np.triu(A, 1), -1, -2)
    return np.swapaxes(np.linalg.cholesky(S), -1, -2)


class RankChain:
    """One rank's shards [s0, s0+G) of the chain; X, delta, tauh replicated."""

    def __init__(self, Yd_local, state_local: dict, g, rho, hyper):
        self.Ys = np.ascontiguousarray(np.moveaxis(Yd_local, 2, 0))      # G x n x P
        self.yy = np.einsum("mij,mij->mj", self.Ys, self.Ys)
        self.G, self.n, self.P = self.Ys.shape
        self.g, self.rho, self.hyper = g, rho, hyper
        self.s0 = dist.get_rank() * self.G
        self.st = {k: np.array(v, dtype=float, copy=True) for k, v in state_local.items()}
        self.K = self.st["Lambda"].shape[1]

    def iteration(self, d):
        st, rho, hyper, K, G, s0 = self.st, self.rho, self.hyper, self.K, self.G, self.s0
        loc = slice(s0, s0 + G)
        Lg = np.ascontiguousarray(np.moveaxis(st["Lambda"], 2, 0))
        Lw = Lg * st["omega"].T[:, :, None]
        A = np.swapaxes(Lw, 1, 2) @ Lg
        W = self.Ys @ Lw
        R = chol_upper(np.eye(K)[None] + (1 - rho) * A)
        bz = np.sqrt(1 - rho) * (W - np.sqrt(rho) * (st["X"][None] @ np.swapaxes(A, 1, 2)))
        v = np.linalg.solve(R, np.swapaxes(bz, 1, 2))
        eps = np.moveaxis(d.NZ[:, :, loc], 2, 0)
        Zk = np.linalg.solve(np.swapaxes(R, 1, 2), v + eps)                # G x K x n
        st["Z"] = np.moveaxis(np.swapaxes(Zk, 1, 2), 0, 2)
        Zg = np.swapaxes(Zk, 1, 2)
        Sr = (W - np.sqrt(1 - rho) * (Zg @ np.swapaxes(A, 1, 2))).sum(axis=0)
        if not hasattr(self, "Asums"):                                   # before the first iteration
            self.Asums = all_gather_np(A.sum(axis=0))
        parts = all_gather_np(Sr)                                        # exchange 1
        S = parts[0]
        for p_ in parts[1:]:
            S = S + p_
        Asum = self.Asums[0]
        for p_ in self.Asums[1:]:
            Asum = Asum + p_
        Rx = chol_upper(self.g * np.eye(K) + rho * Asum)
        vx = np.linalg.solve(Rx, (np.sqrt(rho) * S).T)
        st["X"] = np.linalg.solve(Rx.T, vx + d.NX).T
        st["eta"] = np.sqrt(rho) * st["X"][:, :, None] + np.sqrt(1 - rho) * st["Z"]
        # loadings
        eta = np.ascontiguousarray(np.moveaxis(st["eta"], 2, 0))
        E = np.swapaxes(eta, 1, 2) @ eta
        C = np.swapaxes(self.Ys, 1, 2) @ eta
        ps = st["ps"][:, 0, :].T
        Q = ps[:, :, None, None] * E[:, None, :, :]
        idx = np.arange(K)
        Q[:, :, idx, idx] += np.moveaxis(st["Plam"], 2, 0)
        L = np.linalg.cholesky(Q)
        z = np.moveaxis(d.NL[:, :, loc], (0, 1, 2), (2, 1, 0))
        vv = np.linalg.solve(L, (ps[:, :, None] * C)[..., None])[..., 0]
        lam = np.linalg.solve(np.swapaxes(L, -1, -2), (vv + z)[..., None])[..., 0]
        st["Lambda"] = np.moveaxis(lam, 0, 2)
        tau_loc = st["tauh"][:, 0, loc][None]
        st["psi"] = (1.0 / (hyper.df / 2 + 0.5 * (st["Lambda"] ** 2 * tau_loc))) * d.Gpsi[:, :, loc]
        colsum = (st["psi"] * st["Lambda"] ** 2).sum(axis=0)            # K x G
        SS = self.yy - 2.0 * np.einsum("mjk,mjk->mj", lam, C) + np.einsum("mjk,mkl,mjl->mj", lam, E, lam)
        st["ps"][:, 0, :] = ((1.0 / (hyper.bs + 0.5 * SS)) * d.Gps[:, loc].T).T
        st["omega"] = 1.0 / st["ps"][:, 0, :]
        Ln = np.ascontiguousarray(np.moveaxis(st["Lambda"], 2, 0))
        An = np.swapaxes(Ln * st["omega"].T[:, :, None], 1, 2) @ Ln     # next iteration's A_m
        msgs = all_gather_np(np.concatenate([colsum.T.reshape(-1), An.sum(axis=0).reshape(-1)]))   # exchange 2
        colsum_all = np.concatenate([m_[:G * K].reshape(G, K) for m_ in msgs], axis=0).T   # K x g
        self.Asums = [m_[G * K:].reshape(K, K) for m_ in msgs]
        self._delta_tau(colsum_all, d.Gdelta)
        st["Plam"] = st["psi"] * st["tauh"][:, 0, loc][None]

    def _delta_tau(self, colsum_all, Gdelta):
        """dc:155-165 over ALL shards on every rank (replicated)."""
        hyper, K = self.hyper, self.K
        delta, tauh = self.st["delta"], self.st["tauh"]
        for m in range(self.g):
            cs = colsum_all[:, m]
            bd = hyper.bd1 + (0.5 * (1.0 / delta[0, 0, m])) * np.sum(tauh[:, 0, m] * cs)
            delta[0, 0, m] = (1.0 / bd) * Gdelta[0, m]
            tauh[...] = matlab_cumprod_delta(delta)
            for h in range(1, K):
                bd = hyper.bd2 + (0.5 * (1.0 / delta[h, 0, 0])) * np.sum(tauh[h:, 0, m] * cs[h:])
                delta[h, 0, m] = (1.0 / bd) * Gdelta[h, m]
                tauh[:, :, m] = np.cumprod(delta[:, :, m], axis=0)

    def save_and_assemble(self, SigLower, effsamp, tile=8):
        """Flush of one saved sample: all-gather Lambda/omega, this rank's tiles (round-robin)."""
        st = self.st
        Lloc = np.moveaxis(st["Lambda"], 2, 0).reshape(self.G * self.P, self.K)
        L = np.concatenate(all_gather_np(Lloc), axis=0)                  # exchange 3
        w = np.concatenate(all_gather_np(st["omega"].T.reshape(-1)))
        p = L.shape[0]
        nt = -(-p // tile)
        idx = 0
        rank, world = dist.get_rank(), dist.get_world_size()
        for ti in range(nt):
            for tj in range(ti + 1):
                if idx % world == rank:
                    a = slice(ti * tile, min(p, (ti + 1) * tile))
                    b = slice(tj * tile, min(p, (tj + 1) * tile))
                    blk = L[a] @ L[b].T
                    ra = np.arange(a.start, a.stop)[:, None] // self.P
                    rb = np.arange(b.start, b.stop)[None, :] // self.P
                    blk = np.where(ra == rb, 1.0, self.rho) * blk / effsamp
                    if ti == tj:
                        blk = np.tril(blk) + np.diag(w[a] / effsamp)
                    SigLower[a, b] += blk
                idx += 1
        return SigLower
