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
which each rank accumulates its block of Sigmaout: the contiguous tile rows
[Tb[r], Tb[r+1]) of the lower triangle (``sigma_split``, balanced by tile count).
dcfm_get_sigma gathers to rank 0: each rank packs, per column of the stripe, the
rows it owns (``win_lo`` / ``win_off``), sends them point to point, and rank 0
unpacks — every element moves once, nothing is all-reduced.

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


def tri(t):
    return t * (t + 1) // 2


def sigma_split(nt, nranks):
    """Tile-row boundaries Tb[0..nranks] of the block-sharded Sigmaout (dcfm.hip sigma_split)."""
    Tb = [0] + [nt] * nranks
    total = float(tri(nt))
    for k in range(1, nranks):
        target = total * k / nranks
        t = Tb[k - 1]
        while t < nt and tri(t) < target:
            t += 1
        if t > Tb[k - 1] and target - tri(t - 1) < tri(t) - target:
            t -= 1
        Tb[k] = t
    return Tb


def win_lo(c, R0, R1):
    """First owned row of column c for a rank owning rows [R0, R1) (dcfm_internal.h)."""
    return 0 if R0 <= c < R1 else (R0 if c < R0 else R1)


def win_off(c, c0, R0, R1):
    na = max(min(c, R0) - c0, 0)
    nb = max(min(c, R1) - max(c0, R0), 0)
    return na * (R1 - R0) + nb * R1


def pack_stripe(SigLower, R0, R1, c0, c1):
    """This rank's packed windows of the columns [c0, c1) of Sigmaout (k_sigma_pack)."""
    out = np.zeros(win_off(c1, c0, R0, R1))
    for c in range(c0, c1):
        lo = win_lo(c, R0, R1)
        for r in range(lo, R1):
            out[win_off(c, c0, R0, R1) + r - lo] = SigLower[r, c] if r >= c else SigLower[c, r]
    return out


def unpack_stripe(parts, Tb, tile, p, c0, c1):
    """Rank 0: the dense p x (c1 - c0) stripe from every rank's packed windows (k_sigma_unpack)."""
    out = np.zeros((p, c1 - c0))
    for c in range(c0, c1):
        for r in range(p):
            t = max(r, c) // tile
            k = max(i for i in range(len(Tb) - 1) if Tb[i] <= t)
            R0, R1 = min(p, Tb[k] * tile), min(p, Tb[k + 1] * tile)
            out[r, c - c0] = parts[k][win_off(c, c0, R0, R1) + r - win_lo(c, R0, R1)]
    return out


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
        """Flush of one saved sample: all-gather Lambda/omega, this rank's block of tile rows."""
        st = self.st
        Lloc = np.moveaxis(st["Lambda"], 2, 0).reshape(self.G * self.P, self.K)
        L = np.concatenate(all_gather_np(Lloc), axis=0)                  # exchange 3
        w = np.concatenate(all_gather_np(st["omega"].T.reshape(-1)))
        p = L.shape[0]
        nt = -(-p // tile)
        rank, world = dist.get_rank(), dist.get_world_size()
        Tb = sigma_split(nt, world)
        for ti in range(Tb[rank], Tb[rank + 1]):
            for tj in range(ti + 1):
                if True:
                    a = slice(ti * tile, min(p, (ti + 1) * tile))
                    b = slice(tj * tile, min(p, (tj + 1) * tile))
                    blk = L[a] @ L[b].T
                    ra = np.arange(a.start, a.stop)[:, None] // self.P
                    rb = np.arange(b.start, b.stop)[None, :] // self.P
                    blk = np.where(ra == rb, 1.0, self.rho) * blk / effsamp
                    if ti == tj:
                        blk = np.tril(blk) + np.diag(w[a] / effsamp)
                    SigLower[a, b] += blk
        return SigLower

    @staticmethod
    def gather_sigma(SigLower, tile=8, stripe=16):
        """dcfm_get_sigma: stripes of packed windows, point to point to rank 0 (gloo gather)."""
        p = SigLower.shape[0]
        rank, world = dist.get_rank(), dist.get_world_size()
        Tb = sigma_split(-(-p // tile), world)
        R0, R1 = min(p, Tb[rank] * tile), min(p, Tb[rank + 1] * tile)
        full = np.zeros((p, p)) if rank == 0 else None
        for c0 in range(0, p, stripe):
            c1 = min(p, c0 + stripe)
            mine = torch.from_numpy(pack_stripe(SigLower, R0, R1, c0, c1))
            cnts = [win_off(c1, c0, min(p, Tb[k] * tile), min(p, Tb[k + 1] * tile)) for k in range(world)]
            if rank == 0:
                bufs = [torch.empty(n_, dtype=torch.float64) for n_ in cnts]
                bufs[0] = mine
                for k in range(1, world):
                    if cnts[k]:
                        dist.recv(bufs[k], src=k)
                full[:, c0:c1] = unpack_stripe([b_.numpy() for b_ in bufs], Tb, tile, p, c0, c1)
            elif cnts[rank]:
                dist.send(mine, dst=0)
        return full
