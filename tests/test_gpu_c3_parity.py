"""north_star check (2) at the north-star config c3 (p 19,968, n 1,000, g 64, K 30; BURNIN 500,
MCMC 1,500, thin 5): the GPU chain's posterior-mean Sigmaout has the oracle chain's Frobenius AND
operator-norm error against the synthetic truth, within Monte Carlo error (dc:180-196).

Oracle leg: tests/golden/make_c3_parity.py -> tests/golden/c3_parity.json, 6 replicates of the
vectorised oracle chain with dc:169's direct residual (~50 min each on 2 host threads; Frobenius
norm from the lower triangle, operator norm by ARPACK).  GPU leg: the same data and initial state,
16 chains per case with independent Philox draws, errors from dcfm_sigma_error (Sigmaout never leaves
the device; operator norm by 120 Lanczos steps).  Bar: tests/stat_parity.py (the oracle chains' errors
against the GPU chains' distribution per case, two-sided 1 %); every chain's numbers go to
gpurun_out/c3_parity_gpu.json."""
from pathlib import Path

import pytest

from stat_parity import run_paired

pytestmark = pytest.mark.gpu
FIX = Path(__file__).resolve().parent / "golden" / "c3_parity.json"


def test_c3_posterior_error_matches_oracle(dcfm, record_property):
    s = run_paired(dcfm, FIX, "c3", seed0=7000, dense_truth=False, record_property=record_property)
    assert s["R"] >= 6 and s["oracle_direct_residual"]
