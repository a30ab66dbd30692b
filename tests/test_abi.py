"""CPU tests of the C ABI boundary: the library loads, exports exactly what
include/dcfm.h declares, the ctypes structs match the C layout, argument
validation works without a GPU, and the product fails loudly without its .so."""
import ctypes as C
import os
import re
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "dcfm.h"


def header_functions():
    txt = HEADER.read_text()
    return set(re.findall(r"^\s*(?:int|void|const char|int64_t)\s*\*?\s*(dcfm_\w+)\s*\(", txt, re.M))


def test_library_exports_every_declared_symbol(dcfm):
    lib = dcfm.load_library()
    declared = header_functions()
    assert declared == set(dcfm.EXPORTS), declared ^ set(dcfm.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.dcfm_abi_version() == 2


def test_struct_layout_matches_c(dcfm, tmp_path):
    from dcfm_amd import _abi
    fields = [f for f, _ in _abi.DcfmConfig._fields_]
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "dcfm.h"', "int main(void){"]
    src.append('printf("config %zu\\n", sizeof(dcfm_config));')
    for f in fields:
        src.append(f'printf("%s %zu\\n", "{f}", offsetof(dcfm_config, {f}));')
    src.append('printf("state %zu\\n", sizeof(dcfm_state_view));')
    src.append('printf("draws %zu\\n", sizeof(dcfm_draws_view));')
    src.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", str(ROOT / "include"), str(c), "-o", str(exe)], check=True)
    out = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.splitlines())
    assert int(out["config"]) == C.sizeof(_abi.DcfmConfig)
    for f in fields:
        assert int(out[f]) == getattr(_abi.DcfmConfig, f).offset, f
    assert int(out["state"]) == C.sizeof(_abi.DcfmStateView)
    assert int(out["draws"]) == C.sizeof(_abi.DcfmDrawsView)


def _create(dcfm, **kw):
    from dcfm_amd import _abi
    lib = dcfm.load_library()
    cfg = _abi.DcfmConfig()
    base = dict(n=10, P=4, g=2, K=2, rho=0.5, burnin=0, mcmc=2, thin=1, nranks=1, rank=0, device=0,
                as_=1.0, bs=0.3, df=3.0, ad1=2.0, bd1=1.0, ad2=2.0, bd2=1.0)
    base.update(kw)
    for k, v in base.items():
        setattr(cfg, k, v)
    h = C.c_void_p()
    rc = lib.dcfm_create(C.byref(cfg), C.byref(h))
    msg = lib.dcfm_last_error(None).decode()
    if rc == 0:
        lib.dcfm_destroy(h)
    return rc, msg


def test_create_validates_before_touching_a_device(dcfm):
    from dcfm_amd import _abi
    assert _create(dcfm, K=129)[0] == _abi.DCFM_ERR_UNSUPPORTED
    assert _create(dcfm, g=3, nranks=2)[0] == _abi.DCFM_ERR_UNSUPPORTED
    assert _create(dcfm, rho=1.5)[0] == _abi.DCFM_ERR_INVALID
    assert _create(dcfm, thin=0)[0] == _abi.DCFM_ERR_INVALID
    assert _create(dcfm, n=0)[0] == _abi.DCFM_ERR_INVALID
    assert _create(dcfm, bs=0.0)[0] == _abi.DCFM_ERR_INVALID
    # every positive hyper-parameter the reference accepts (dc:62-65) is drawn on the device
    # (gamma shapes below 1 by the boost): past validation, to the device lookup
    for kw in (dict(df=1.5), dict(as_=0.5), dict(ad2=0.9), dict(ad1=0.5, flags=_abi.DCFM_FLAG_INJECT_DRAWS)):
        assert _create(dcfm, **kw)[0] not in (_abi.DCFM_ERR_UNSUPPORTED, _abi.DCFM_ERR_INVALID), kw
    assert _create(dcfm, as_=0.0)[0] == _abi.DCFM_ERR_INVALID
    assert _create(dcfm, ad2=-1.0)[0] == _abi.DCFM_ERR_INVALID
    # the register tree of the fused K <= 32 chain caps g; the side-stream layout does not
    assert _create(dcfm, g=1024, P=2)[0] == _abi.DCFM_ERR_UNSUPPORTED
    assert _create(dcfm, g=1024, P=2, flags=_abi.DCFM_FLAG_UNFUSED)[0] not in (_abi.DCFM_ERR_UNSUPPORTED,
                                                                             _abi.DCFM_ERR_INVALID)


def test_create_without_gpu_reports_hip_error(dcfm, gpu_available):
    if gpu_available:
        pytest.skip("GPU present")
    from dcfm_amd import _abi
    rc, msg = _create(dcfm)
    assert rc == _abi.DCFM_ERR_HIP and "device" in msg


def test_product_fails_loudly_without_library(tmp_path):
    code = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {str(ROOT)!r})
        import __graft_entry__ as ge
        pkg = ge.load_package()
        try:
            pkg.Sampler(10, 4, 2, 2, 0.5, 0, 2, 1)
        except ImportError as e:
            print("IMPORTERROR", e)
    """)
    env = dict(os.environ, DCFM_LIB=str(tmp_path / "missing.so"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env)
    assert "IMPORTERROR" in out.stdout and "no CPU fallback" in out.stdout, out.stdout + out.stderr


def test_driver_preprocess_matches_oracle(dcfm):
    """The product's host driver (dc:29-87) agrees with the oracle's restatement."""
    import numpy as np
    import oracle
    from oracle import dc_oracle as F
    Y, _ = oracle.synth.make_data(20, 26, k0=3, zero_cols=2)
    a = dcfm.preprocess(Y, 4, 8)
    b = F.preprocess(Y, 4, 8)
    assert np.array_equal(a[0], b[0]) and a[1:5] == b[1:5] and np.array_equal(a[5], b[5])
    src = oracle.DrawSource(3, a[1], a[2], 4, 2, F.Hyper())
    init = src.init()
    Yd1 = dcfm.partition_standardize(a[0], 4, init.varind)
    Yd2 = F.standardize(F.partition(b[0], 4, init.varind))
    assert np.array_equal(Yd1, Yd2)
    s1 = dcfm.initial_state(a[1], a[3], 2, 4, 0.5, dcfm.Hyper(), init)
    s2 = F.initialise(a[1], a[3], 2, 4, 0.5, F.Hyper(), init)
    for f, v in s1.items():
        assert np.allclose(v, getattr(s2, f), rtol=1e-15, atol=0), f
