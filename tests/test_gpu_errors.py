"""Failure detection through the C ABI: the NaN / Inf sentinel of dcfm_run
returns DCFM_ERR_NUMERIC at the next synchronising call, and a set_state clears it."""
import numpy as np
import pytest

from helpers import make_case, stacked_draws, state_dict

pytestmark = pytest.mark.gpu


def test_non_finite_state_is_reported(dcfm):
    from dcfm_amd import _abi
    c = make_case(30, 40, 4, 3, seed=5)
    smp = dcfm.Sampler(c["n"], c["P"], 4, 3, c["rho"], 0, 3, 1, inject_draws=True)
    try:
        smp.set_data(c["Yd"])
        st = {f: v for f, v in state_dict(c["st"]).items() if f != "eta"}
        smp.set_state(st)
        smp.set_draws(stacked_draws(c["src"], 1, 3), 1, 3)
        smp.run(1, 1)
        smp.synchronize()                                   # clean chain: no error
        bad = {f: np.array(v, copy=True) for f, v in st.items()}
        bad["ps"][3, 0, 1] = np.nan                         # residual precision of one row
        smp.set_state(bad)
        smp.run(2, 1)
        with pytest.raises(_abi.DcfmError) as ei:
            smp.get_state()
        assert ei.value.code == _abi.DCFM_ERR_NUMERIC
        with pytest.raises(_abi.DcfmError):
            smp.synchronize()
        smp.set_state(st)                                   # restart clears the sentinel
        smp.run(2, 1)
        smp.get_state()
    finally:
        smp.close()
