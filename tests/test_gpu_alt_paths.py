"""Parity of the alternate launch layouts selected by dcfm_config.flags:
  DCFM_FLAG_UNFUSED      K <= 32 through the side-stream layout (k_prep / k_asum /
                         k_xchol / k_wpass / k_zdraw / k_colsum / k_delta with events)
  DCFM_FLAG_ONE_STREAM   every launch on one stream
Each case runs (in a child process, as the driver's GPU runs do) the injected-draw chain of a
tests/test_gpu_parity.py case and checks every state field after every iteration against the
oracle at the same 1e-10 bar."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import __graft_entry__ as ge
from helpers import make_case, state_dict, stacked_draws, rel_err, STATE_CMP
from oracle import dc_oracle as F
import test_gpu_parity as T
dcfm = ge.load_package()
n, p, g, K, burnin, mcmc, thin = T.CASES[sys.argv[1]]
c = make_case(n, p, g, K)
N = burnin + mcmc
smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True, flags=int(sys.argv[2]))
smp.set_data(c["Yd"]); smp.set_state(state_dict(c["st"])); smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
ref = c["st"].copy(); Sref = None
worst = 0.0
for it in range(1, N + 1):
    smp.run(it, 1)
    Sref = F.run_chain(c["Yd"], ref, c["rho"], c["hyper"], c["src"].iteration, it, 1, burnin, mcmc, thin, Sigmaout=Sref)
    got = smp.get_state()
    for f in STATE_CMP:
        worst = max(worst, rel_err(got[f], getattr(ref, f)))
worst = max(worst, rel_err(smp.get_sigma(), Sref))
print("WORST", worst)
"""


UNFUSED, ONE_STREAM = 0x2, 0x4


@pytest.mark.parametrize("flags,case", [(UNFUSED, "basic"), (UNFUSED, "K30"), (ONE_STREAM, "K30"),
                                        (UNFUSED | ONE_STREAM, "basic"),
                                        (UNFUSED, "g5_odd_chunk"), (UNFUSED, "g10_odd_chunk")])
def test_alternate_path_parity(flags, case):
    import test_gpu_parity as T
    if case not in T.CASES:
        pytest.skip(f"no case {case}")
    r = subprocess.run([sys.executable, "-c", CHILD, case, str(flags)], cwd=ROOT, env=dict(os.environ),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    worst = float([ln for ln in r.stdout.splitlines() if ln.startswith("WORST")][-1].split()[1])
    assert worst < 1e-10, f"flags {flags:#x} {case}: worst rel err {worst:.3e}"
