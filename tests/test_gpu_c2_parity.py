"""north_star check (2) at BASELINE config c2 (p 5,000, n 500, g 8, K 20; BURNIN 500, MCMC 2,000,
thin 5): the GPU chain's posterior-mean Sigmaout has the oracle chain's Frobenius AND
operator-norm error against the synthetic truth, within Monte Carlo error (dc:180-196).

Oracle leg: tests/golden/make_c2_parity.py -> tests/golden/c2_parity.json, 8 replicates of the
vectorised oracle chain with dc:169's direct residual (exact eigvalsh operator norm).  GPU leg: the
same data and initial state, 16 chains per case with independent Philox draws, errors from
dcfm_sigma_error.  Bar: tests/stat_parity.py (the oracle chains' errors against the GPU chains'
distribution per case, two-sided 1 %); every chain's numbers go to gpurun_out/c2_parity_gpu.json."""
from pathlib import Path

import pytest

from stat_parity import run_paired

pytestmark = pytest.mark.gpu
FIX = Path(__file__).resolve().parent / "golden" / "c2_parity.json"


def test_c2_posterior_error_matches_oracle(dcfm, record_property):
    s = run_paired(dcfm, FIX, "c2", seed0=5000, dense_truth=True, record_property=record_property)
    assert s["R"] >= 8 and s["oracle_direct_residual"]
