"""Handle wrapper around the C ABI: the hot loop of divideconquer.m (dc:90-197).

Arrays cross the boundary in the reference's MATLAB shapes and column-major
order (``Lambda`` P x K x g_local, ``Yd`` n x P x g_local, ``delta`` K x 1 x g,
...), exactly as a MEX gateway would pass them.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi

STATE_FIELDS = ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "eta", "delta", "tauh")


@dataclass(frozen=True)
class Hyper:
    """dc:62-65 (hard-coded in the reference)."""
    as_: float = 1.0
    bs: float = 0.3
    df: float = 3.0
    ad1: float = 2.0
    bd1: float = 1.0
    ad2: float = 2.0
    bd2: float = 1.0


def _f64F(a) -> np.ndarray:
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Sampler:
    """One rank's handle: shards [rank*g_local, (rank+1)*g_local) of a chain."""

    def __init__(self, n, P, g, K, rho, burnin, mcmc, thin, *, hyper: Hyper = Hyper(), seed=0,
                 nranks=1, rank=0, device=0, inject_draws=False, asm_batch=0, flags=0):
        self.lib = _abi.load_library()
        cfg = _abi.DcfmConfig()
        cfg.n, cfg.P, cfg.g, cfg.K = int(n), int(P), int(g), int(K)
        cfg.rho = float(rho)
        cfg.burnin, cfg.mcmc, cfg.thin = int(burnin), int(mcmc), int(thin)
        cfg.as_, cfg.bs, cfg.df = hyper.as_, hyper.bs, hyper.df
        cfg.ad1, cfg.bd1, cfg.ad2, cfg.bd2 = hyper.ad1, hyper.bd1, hyper.ad2, hyper.bd2
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.nranks, cfg.rank, cfg.device = int(nranks), int(rank), int(device)
        cfg.flags = (_abi.DCFM_FLAG_INJECT_DRAWS if inject_draws else 0) | int(flags)
        cfg.asm_batch = int(asm_batch)
        self.cfg = cfg
        h = C.c_void_p()
        rc = self.lib.dcfm_create(C.byref(cfg), C.byref(h))
        _abi.check(self.lib, None, rc)
        self.h = h
        self.n, self.P, self.g, self.K = cfg.n, cfg.P, cfg.g, cfg.K
        self.nranks, self.rank = cfg.nranks, cfg.rank
        self.g_local = self.g // self.nranks
        self.shard0 = self.rank * self.g_local

    # -- lifecycle -------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.dcfm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        _abi.check(self.lib, self.h, rc)

    # -- multi-rank -------------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        lib = _abi.load_library()
        buf = (C.c_uint8 * 128)()
        _abi.check(lib, None, lib.dcfm_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.dcfm_comm_init(self.h, buf))

    # -- inputs ----------------------------------------------------------------
    @staticmethod
    def comm_loopback(samplers):
        """In-process loopback communicator over ``samplers`` (ranks 0..n-1 of one chain
        on one device): each sampler must then be driven from its own thread."""
        n = len(samplers)
        arr = (C.c_void_p * n)(*[s_.h.value for s_ in samplers])
        lib = samplers[0].lib
        _abi.check(lib, None, lib.dcfm_comm_init_loopback(arr, n))

    def set_data(self, Yd_local):
        Y = _f64F(Yd_local)
        if Y.shape != (self.n, self.P, self.g_local):
            raise ValueError(f"Yd_local must be n x P x g_local = {(self.n, self.P, self.g_local)}, got {Y.shape}")
        self._check(self.lib.dcfm_set_data(self.h, _ptr(Y)))

    def set_data_raw(self, Y, cols):
        """On-device ingest (dc:48-59, dcfm_set_data_raw): Y is the raw n x p_in data,
        ``cols`` the 0-based input column of every (local shard, position) pair, length
        P * g_local (``shard_columns``).  Returns (sd, kernel_ms): the P x g_local sample
        standard deviations and the standardise kernel's device time."""
        Y = _f64F(Y)
        if Y.ndim != 2 or Y.shape[0] != self.n:
            raise ValueError(f"Y must be n x p_in with n = {self.n}, got {Y.shape}")
        c = np.ascontiguousarray(np.asarray(cols, dtype=np.int64).reshape(-1))
        if c.size != self.P * self.g_local:
            raise ValueError(f"cols must hold P * g_local = {self.P * self.g_local} indices, got {c.size}")
        sd = np.zeros((self.P, self.g_local), dtype=np.float64, order="F")
        ms = C.c_double(0.0)
        self._check(self.lib.dcfm_set_data_raw(self.h, _ptr(Y), Y.shape[1],
                                               c.ctypes.data_as(C.POINTER(C.c_int64)), _ptr(sd), C.byref(ms)))
        return sd, ms.value

    def get_data(self) -> np.ndarray:
        """Yd as the sweep holds it (n x P x g_local)."""
        out = np.zeros((self.n, self.P, self.g_local), dtype=np.float64, order="F")
        self._check(self.lib.dcfm_get_data(self.h, _ptr(out)))
        return out

    def _shapes(self):
        n, P, K, gl, g = self.n, self.P, self.K, self.g_local, self.g
        return {"Lambda": (P, K, gl), "ps": (P, 1, gl), "omega": (P, gl), "psi": (P, K, gl),
                "Plam": (P, K, gl), "X": (n, K), "Z": (n, K, gl), "eta": (n, K, gl),
                "delta": (K, 1, g), "tauh": (K, 1, g)}

    def set_state(self, state: dict):
        """state: MATLAB-shaped arrays; local shards for per-shard fields, all g for delta/tauh."""
        shapes = self._shapes()
        keep = []
        view = _abi.DcfmStateView()
        for f in STATE_FIELDS:
            if f == "eta":
                continue
            a = _f64F(state[f])
            if a.size != int(np.prod(shapes[f])):
                raise ValueError(f"{f}: expected shape {shapes[f]}, got {a.shape}")
            keep.append(a)
            setattr(view, f, _ptr(a))
        self._check(self.lib.dcfm_set_state(self.h, C.byref(view)))

    def init_state(self):
        """dc:68-87 on the device from the Philox stream (dcfm_init_state), instead of set_state."""
        self._check(self.lib.dcfm_init_state(self.h))

    def set_draws(self, draws: dict, first_iter: int, n_iter: int):
        """draws: full-g arrays NZ (K,n,g,T), NX (K,n,T), NL (K,P,g,T), Gpsi (P,K,g,T),
        Gdelta (K,g,T), Gps (P,g,T) — the layout of oracle.IterDraws.stacked()."""
        view = _abi.DcfmDrawsView()
        keep = []
        for f in ("NZ", "NX", "NL", "Gpsi", "Gdelta", "Gps"):
            a = _f64F(draws[f])
            keep.append(a)
            setattr(view, f, _ptr(a))
        self._check(self.lib.dcfm_set_draws(self.h, C.byref(view), int(first_iter), int(n_iter)))

    # -- hot loop ----------------------------------------------------------------
    def run(self, first_iter: int, n_iter: int):
        self._check(self.lib.dcfm_run(self.h, int(first_iter), int(n_iter)))

    def synchronize(self):
        self._check(self.lib.dcfm_synchronize(self.h))

    # -- outputs -------------------------------------------------------------------
    def get_state(self, fields=STATE_FIELDS, raw=False) -> dict:
        """The state in MATLAB shapes.  ``raw``: skip the non-finite check (dcfm_get_state_raw), to
        read the state after a run that ended in DCFM_ERR_NUMERIC."""
        shapes = self._shapes()
        out = {f: np.zeros(shapes[f], dtype=np.float64, order="F") for f in fields}
        view = _abi.DcfmStateView()
        for f, a in out.items():
            setattr(view, f, _ptr(a))
        fn = self.lib.dcfm_get_state_raw if raw else self.lib.dcfm_get_state
        self._check(fn(self.h, C.byref(view)))
        return out

    def get_sigma(self):
        """Sigmaout (p x p, Fortran order).  Collective when nranks > 1: every rank calls it,
        rank 0 receives the matrix and the other ranks get None (Sigmaout is block-sharded
        over the ranks, dcfm_sigma_block; each element moves once, owner -> rank 0)."""
        p = self.P * self.g
        if self.rank != 0:
            self._check(self.lib.dcfm_get_sigma(self.h, None))
            return None
        S = np.zeros((p, p), dtype=np.float64, order="F")
        self._check(self.lib.dcfm_get_sigma(self.h, _ptr(S)))
        return S

    def get_sigma_cols(self, col0: int, ncols: int):
        """Sigmaout(:, col0 : col0+ncols) as a p x ncols Fortran array (collective if nranks > 1;
        rank 0 receives it, other ranks get None)."""
        p = self.P * self.g
        if self.rank != 0:
            self._check(self.lib.dcfm_get_sigma_cols(self.h, int(col0), int(ncols), None))
            return None
        S = np.zeros((p, int(ncols)), dtype=np.float64, order="F")
        self._check(self.lib.dcfm_get_sigma_cols(self.h, int(col0), int(ncols), _ptr(S)))
        return S

    def sigma_block(self) -> dict:
        """This rank's block of Sigmaout: rows [row0, row1) of the lower triangle and its bytes."""
        out = (C.c_int64 * 3)()
        self._check(self.lib.dcfm_sigma_block(self.h, out))
        return {"row0": int(out[0]), "row1": int(out[1]), "bytes": int(out[2])}

    def sigma_error(self, U, s, iters: int = 60, seed: int = 1) -> dict:
        """Frobenius / operator-norm error of Sigmaout against U U' + diag(s), on the device
        (dcfm_sigma_error).  U: p x r truth factors in output coordinates, s: p."""
        p = self.P * self.g
        U = _f64F(np.asarray(U, dtype=np.float64).reshape(p, -1))
        s = _f64F(np.asarray(s, dtype=np.float64).reshape(p))
        out = np.zeros(3)
        self._check(self.lib.dcfm_sigma_error(self.h, _ptr(U), U.shape[1], _ptr(s), int(iters),
                                              int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(out)))
        fro, tru, op = (float(x) for x in out)
        return {"fro": fro, "op": op, "fro_rel": fro / tru if tru > 0 else float("nan"), "truth_fro": tru}

    def saved_samples(self) -> int:
        return int(self.lib.dcfm_saved_samples(self.h))

    # -- chain trace (diagnostics across chains) -----------------------------------
    TRACE_FIELDS = ("lambda_fro2", "tr_omega", "sum_log_ps", "sum_log_tau")

    def set_trace(self, capacity: int):
        """Record one row of TRACE_FIELDS per iteration of later runs (0 = off)."""
        self._check(self.lib.dcfm_set_trace(self.h, int(capacity)))
        self._trace_cap = int(capacity)

    def get_trace(self) -> np.ndarray:
        """(iterations recorded) x 4 array of this rank's local-shard sums."""
        cnt = C.c_int64(0)
        cap = getattr(self, "_trace_cap", 0)
        out = np.zeros((max(cap, 1), 4), dtype=np.float64)
        self._check(self.lib.dcfm_get_trace(self.h, _ptr(out), C.byref(cnt)))
        return out[:cnt.value].copy()

    # -- measurement -----------------------------------------------------------------
    def set_profiling(self, on: bool):
        self._check(self.lib.dcfm_set_profiling(self.h, 1 if on else 0))

    def set_profiling_kernels(self, names, stride: int = 1):
        """Time only these kernels (names of _abi.KERNEL_IDS); empty = off.  stride > 1 times
        one in `stride` launches of each (the event records cost device time per launch)."""
        mask = 0
        for nm in names:
            mask |= 1 << _abi.KERNEL_IDS[nm]
        self._check(self.lib.dcfm_set_profiling_mask(self.h, mask))
        if stride != 1:
            self._check(self.lib.dcfm_set_profiling_stride(self.h, int(stride)))

    def kernel_stats(self) -> dict:
        ms = (C.c_double * _abi.K_COUNT)()
        cnt = (C.c_int64 * _abi.K_COUNT)()
        self._check(self.lib.dcfm_get_kernel_stats(self.h, ms, cnt))
        return {name: (ms[i], cnt[i]) for name, i in _abi.KERNEL_IDS.items()}


def count_nonzero_columns(Y, device=0, return_ms=False):
    """dc:31-34 on the device: nnz of every column of the n x p matrix Y (int32)."""
    lib = _abi.load_library()
    Y = _f64F(Y)
    if Y.ndim != 2:
        raise ValueError("Y must be n x p")
    out = np.zeros(Y.shape[1], dtype=np.int32)
    ms = C.c_double(0.0)
    rc = lib.dcfm_count_nonzero_columns(int(device), _ptr(Y), Y.shape[0], Y.shape[1],
                                        out.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(ms))
    _abi.check(lib, None, rc)
    return (out, ms.value) if return_ms else out


def rng_fill(kind: str, count: int, *, seed=0, shape=1.0, site=15, shard=0, iteration=0, device=0, width=32):
    """On-device Philox variates exactly as the sweep draws them (diagnostic): variate e at the
    counter (site, shard, row = e // width, index = e % width, iteration)."""
    lib = _abi.load_library()
    out = np.zeros(int(count), dtype=np.float64)
    k = {"normal": 0, "gamma": 1}[kind]
    if width == 32:
        rc = lib.dcfm_rng_fill(int(device), int(seed), k, float(shape), int(site), int(shard),
                               int(iteration), int(count), _ptr(out))
    else:
        rows = (int(count) + int(width) - 1) // int(width)
        rc = lib.dcfm_rng_fill_rows(int(device), int(seed), k, float(shape), int(site), int(shard),
                                    int(iteration), rows, int(width), int(count), _ptr(out))
    _abi.check(lib, None, rc)
    return out
