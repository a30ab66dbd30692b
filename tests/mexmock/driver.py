"""ctypes driver for the MEX gateway compiled against the mock runtime (test infrastructure).

build(out_dir) compiles matlab/dcfm_mex.c + tests/mexmock/mexmock.c with gcc into a shared
library linked to libdcfm.so; Mex(lib).call("cmd", args...) plays MATLAB's part: numpy
arrays go in as mxArrays (column-major, class from the dtype), outputs come back as numpy
arrays, and a mexErrMsgIdAndTxt surfaces as MexError(id, message).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd"
MX_DOUBLE, MX_INT64 = 6, 14
FLAGS = ["-std=c11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror", f"-I{ROOT / 'tests' / 'mexmock'}",
         f"-I{ROOT / 'include'}"]


def syntax_check():
    subprocess.run(["gcc", "-fsyntax-only", *FLAGS, str(ROOT / "matlab" / "dcfm_mex.c")], check=True,
                   capture_output=True, text=True)


def build(out_dir: Path) -> Path:
    out = Path(out_dir) / "libdcfm_mex_mock.so"
    cmd = ["gcc", "-shared", "-fPIC", "-O1", *FLAGS, str(ROOT / "matlab" / "dcfm_mex.c"),
           str(ROOT / "tests" / "mexmock" / "mexmock.c"), f"-L{PKG}", "-ldcfm", f"-Wl,-rpath,{PKG}", "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr)
    return out


class MexError(Exception):
    def __init__(self, ident, msg):
        super().__init__(f"{ident}: {msg}")
        self.id, self.msg = ident, msg


class Mex:
    def __init__(self, path):
        L = C.CDLL(str(path))
        vp = C.c_void_p
        L.mm_numeric.restype = vp
        L.mm_numeric.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int64), vp, C.c_int]
        L.mm_string.restype = vp
        L.mm_string.argtypes = [C.c_char_p]
        L.mm_struct.restype = vp
        L.mm_struct.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(vp)]
        L.mm_data.restype = vp
        L.mm_data.argtypes = [vp]
        L.mm_numel.restype = C.c_int64
        L.mm_numel.argtypes = [vp]
        L.mm_ndim.argtypes = [vp]
        L.mm_dim.restype = C.c_int64
        L.mm_dim.argtypes = [vp, C.c_int]
        L.mm_free.argtypes = [vp]
        L.mm_call.argtypes = [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp)]
        L.mm_error_id.restype = C.c_char_p
        L.mm_error_msg.restype = C.c_char_p
        self.L = L

    def arr(self, x, cplx=False):
        if isinstance(x, str):
            return self.L.mm_string(x.encode())
        if isinstance(x, dict):
            names = (C.c_char_p * len(x))(*[k.encode() for k in x])
            vals = (C.c_void_p * len(x))(*[self.arr(v) for v in x.values()])
            return self.L.mm_struct(len(x), names, vals)
        a = np.asarray(x)
        if a.dtype == np.int64:
            cls = MX_INT64
        else:
            a = a.astype(np.float64)
            cls = MX_DOUBLE
        a = np.asfortranarray(a)
        shape = a.shape if a.ndim >= 2 else ((1, 1) if a.ndim == 0 else (a.shape[0], 1))
        dims = (C.c_int64 * len(shape))(*shape)
        return self.L.mm_numeric(cls, len(shape), dims, a.ctypes.data_as(C.c_void_p), 1 if cplx else 0)

    def out(self, p):
        nd = self.L.mm_ndim(p)
        shape = tuple(self.L.mm_dim(p, d) for d in range(nd))
        n = self.L.mm_numel(p)
        buf = (C.c_double * max(n, 1)).from_address(self.L.mm_data(p))
        a = np.frombuffer(buf, dtype=np.float64, count=n).copy().reshape(shape, order="F")
        self.L.mm_free(p)
        return a

    def call(self, cmd, *args, nlhs=1, raw=()):
        """raw: indices of args already converted (mxArray pointers)."""
        ins = [self.L.mm_string(cmd.encode()) if isinstance(cmd, str) else self.arr(cmd)]
        ins += [a if i in raw else self.arr(a) for i, a in enumerate(args)]
        prhs = (C.c_void_p * len(ins))(*ins)
        plhs = (C.c_void_p * max(nlhs, 1))()
        rc = self.L.mm_call(nlhs, plhs, len(ins), prhs)
        for p in ins:
            self.L.mm_free(p)
        if rc:
            raise MexError(self.L.mm_error_id().decode(), self.L.mm_error_msg().decode())
        outs = [self.out(plhs[i]) for i in range(max(nlhs, 1)) if plhs[i]]
        return outs[0] if nlhs == 1 and outs else outs

    def locks(self):
        return self.L.mm_locks()
