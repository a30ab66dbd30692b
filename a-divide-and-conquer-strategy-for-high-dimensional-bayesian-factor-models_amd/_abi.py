"""ctypes binding of the C ABI in include/dcfm.h (libdcfm.so, built for gfx950).

This is the binding a Python caller uses; a MATLAB caller would use the MEX
gateway sketched in INTEGRATION.md.  There is no fallback: if libdcfm.so is
missing or cannot be loaded, importing the sampler raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("DCFM_LIB", PKG_DIR / "libdcfm.so"))

DCFM_OK = 0
DCFM_ERR_INVALID = 1
DCFM_ERR_UNSUPPORTED = 2
DCFM_ERR_HIP = 3
DCFM_ERR_RCCL = 4
DCFM_ERR_NUMERIC = 5
DCFM_ERR_ALLOC = 6
DCFM_FLAG_INJECT_DRAWS = 0x1
DCFM_FLAG_UNFUSED = 0x2        # K <= 32 through the side-stream layout (same results)
DCFM_FLAG_ONE_STREAM = 0x4     # every launch on one stream
DCFM_FLAG_FLAT_PRIORITY = 0x8  # default priority for every stream
DCFM_FLAG_COMM_SELF = 0x20   # one rank on the collective path with a real 1-rank RCCL communicator
DCFM_FLAG_EXACT_RESIDUAL = 0x10  # ps / omega from the direct residual (dc:169), one more Y pass
DCFM_FLAG_GUARD_ALL = 0x40       # the SS-identity guard rejects every row (its residual fallback, tests)

KERNEL_IDS = {
    "k_prep": 0, "k_wpass": 1, "k_zdraw": 2, "k_xred": 3, "k_xdraw": 4, "k_cpass": 5,
    "k_lambda": 6, "k_colsum": 7, "k_delta": 8, "k_save": 9, "k_assemble": 10, "rccl": 11,
    "k_xchol": 12, "k_draws": 13, "k_resid": 14,
}
K_COUNT = 15

# every symbol include/dcfm.h declares
EXPORTS = (
    "dcfm_create", "dcfm_destroy", "dcfm_last_error", "dcfm_abi_version",
    "dcfm_comm_unique_id", "dcfm_comm_init", "dcfm_comm_init_loopback", "dcfm_set_data", "dcfm_set_state",
    "dcfm_set_draws", "dcfm_run", "dcfm_synchronize", "dcfm_get_state", "dcfm_get_state_raw", "dcfm_get_sigma",
    "dcfm_get_sigma_cols", "dcfm_sigma_block",
    "dcfm_saved_samples", "dcfm_sigma_error", "dcfm_set_profiling", "dcfm_set_profiling_mask", "dcfm_set_profiling_stride", "dcfm_get_kernel_stats",
    "dcfm_kernel_name",
    "dcfm_rng_fill", "dcfm_rng_fill_rows", "dcfm_set_data_raw", "dcfm_get_data", "dcfm_count_nonzero_columns",
    "dcfm_set_trace", "dcfm_get_trace", "dcfm_init_state",
)


class DcfmConfig(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("P", C.c_int32), ("g", C.c_int32), ("K", C.c_int32),
        ("rho", C.c_double),
        ("burnin", C.c_int64), ("mcmc", C.c_int64), ("thin", C.c_int64),
        ("as_", C.c_double), ("bs", C.c_double), ("df", C.c_double), ("ad1", C.c_double),
        ("bd1", C.c_double), ("ad2", C.c_double), ("bd2", C.c_double),
        ("seed", C.c_uint64),
        ("nranks", C.c_int32), ("rank", C.c_int32), ("device", C.c_int32),
        ("flags", C.c_uint32), ("asm_batch", C.c_int32), ("reserved", C.c_int32 * 7),
    ]


_DP = C.POINTER(C.c_double)


class DcfmStateView(C.Structure):
    _fields_ = [(f, _DP) for f in ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "eta", "delta", "tauh")]


class DcfmDrawsView(C.Structure):
    _fields_ = [(f, _DP) for f in ("NZ", "NX", "NL", "Gpsi", "Gdelta", "Gps")]


class DcfmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"dcfm error {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: Path | None = None):
    """Load libdcfm.so once; raises (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise ImportError(
            f"libdcfm.so not found at {p}: build it first (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C <pkg>/csrc). There is no CPU fallback.")
    lib = C.CDLL(str(p))
    vp = C.c_void_p
    sig = {
        "dcfm_create": (C.c_int, [C.POINTER(DcfmConfig), C.POINTER(vp)]),
        "dcfm_destroy": (None, [vp]),
        "dcfm_last_error": (C.c_char_p, [vp]),
        "dcfm_abi_version": (C.c_int, []),
        "dcfm_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "dcfm_comm_init": (C.c_int, [vp, C.POINTER(C.c_uint8)]),
        "dcfm_comm_init_loopback": (C.c_int, [C.POINTER(vp), C.c_int32]),
        "dcfm_set_data": (C.c_int, [vp, _DP]),
        "dcfm_set_state": (C.c_int, [vp, C.POINTER(DcfmStateView)]),
        "dcfm_set_draws": (C.c_int, [vp, C.POINTER(DcfmDrawsView), C.c_int64, C.c_int64]),
        "dcfm_run": (C.c_int, [vp, C.c_int64, C.c_int64]),
        "dcfm_synchronize": (C.c_int, [vp]),
        "dcfm_get_state": (C.c_int, [vp, C.POINTER(DcfmStateView)]),
        "dcfm_get_state_raw": (C.c_int, [vp, C.POINTER(DcfmStateView)]),
        "dcfm_get_sigma": (C.c_int, [vp, _DP]),
        "dcfm_get_sigma_cols": (C.c_int, [vp, C.c_int64, C.c_int64, _DP]),
        "dcfm_sigma_block": (C.c_int, [vp, C.POINTER(C.c_int64)]),
        "dcfm_saved_samples": (C.c_int64, [vp]),
        "dcfm_sigma_error": (C.c_int, [vp, _DP, C.c_int32, _DP, C.c_int32, C.c_uint64, _DP]),
        "dcfm_set_profiling": (C.c_int, [vp, C.c_int]),
        "dcfm_set_profiling_mask": (C.c_int, [vp, C.c_uint32]),
        "dcfm_set_profiling_stride": (C.c_int, [vp, C.c_int32]),
        "dcfm_get_kernel_stats": (C.c_int, [vp, _DP, C.POINTER(C.c_int64)]),
        "dcfm_kernel_name": (C.c_char_p, [C.c_int]),
        "dcfm_rng_fill": (C.c_int, [C.c_int, C.c_uint64, C.c_int, C.c_double, C.c_int32, C.c_int32,
                                    C.c_int64, C.c_int64, _DP]),
        "dcfm_rng_fill_rows": (C.c_int, [C.c_int, C.c_uint64, C.c_int, C.c_double, C.c_int32, C.c_int32,
                                         C.c_int64, C.c_int64, C.c_int32, C.c_int64, _DP]),
        "dcfm_set_data_raw": (C.c_int, [vp, _DP, C.c_int64, C.POINTER(C.c_int64), _DP, _DP]),
        "dcfm_get_data": (C.c_int, [vp, _DP]),
        "dcfm_set_trace": (C.c_int, [vp, C.c_int64]),
        "dcfm_init_state": (C.c_int, [vp]),
        "dcfm_get_trace": (C.c_int, [vp, _DP, C.POINTER(C.c_int64)]),
        "dcfm_count_nonzero_columns": (C.c_int, [C.c_int, _DP, C.c_int32, C.c_int64, C.POINTER(C.c_int32),
                                                 _DP]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(lib, handle, code: int):
    if code != DCFM_OK:
        msg = lib.dcfm_last_error(handle)
        raise DcfmError(code, msg.decode() if msg else "")
