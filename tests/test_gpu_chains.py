"""Parallel chains (config c4's 8 chains; bench.py --chains): one independent chain per
rank, seed 1 + rank, no collectives.

A chain is defined by its seed alone: rank r's chain must be bitwise the chain a single
process runs with seed 1 + r, whether it runs alone, concurrently with other chains on the
same device (independent handles, host threads), or as a rank of `bench.py --chains`
under torch.distributed.run.  Different seeds must give different chains.
"""
import json
import os
import socket
import subprocess
import sys
import threading
from pathlib import Path

import numpy as np
import pytest

from helpers import make_case

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

SHAPE = dict(n=60, P=40, g=4, K=6, burnin=2, mcmc=6, thin=2)


def _chain(dcfm, Yd, seed):
    s = SHAPE
    smp = dcfm.Sampler(s["n"], s["P"], s["g"], s["K"], 0.5, s["burnin"], s["mcmc"], s["thin"], seed=seed)
    return smp


def _finish(smp):
    N = SHAPE["burnin"] + SHAPE["mcmc"]
    smp.run(1, N)
    st = smp.get_state()
    st["Sig"] = smp.get_sigma()
    smp.close()
    return st


def _alone(dcfm, Yd, seed):
    smp = _chain(dcfm, Yd, seed)
    smp.set_data(Yd)
    smp.init_state()
    return _finish(smp)


def test_concurrent_chains_equal_single_runs(dcfm):
    c = make_case(SHAPE["n"], SHAPE["P"] * SHAPE["g"], SHAPE["g"], SHAPE["K"], seed=5)
    Yd = c["Yd"]
    nch = 4
    alone = [_alone(dcfm, Yd, 1 + r) for r in range(nch)]
    smps = [_chain(dcfm, Yd, 1 + r) for r in range(nch)]
    for smp in smps:
        smp.set_data(Yd)
        smp.init_state()
    out, errs = [None] * nch, []

    def body(r):
        try:
            out[r] = _finish(smps[r])
        except Exception as e:
            errs.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(nch)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    for r in range(nch):
        for f, a in alone[r].items():
            assert np.array_equal(out[r][f], a), f"chain {r}: {f} differs from its single run"
    for r in range(1, nch):
        assert not np.array_equal(out[r]["Lambda"], out[0]["Lambda"]), "seeds 1 and 1 + r gave the same chain"
        assert not np.array_equal(out[r]["Sig"], out[0]["Sig"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_chains_two_ranks(tmp_path):
    """bench.py --chains as the driver would launch it (torch.distributed.run, 2 ranks on
    this box's device(s)): one JSON line, weak scaling, iterations of both chains counted,
    the diagnostics pooled over 2 chains."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--chains", "--steps", "10", "--warmup", "4", "--g", "8", "--P", "50",
           "--nobs", "200", "--K", "10", "--no-cpu-baseline", "--err-iters", "0", "--asm-batch", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["value"] > 0 and out["steps"] == 10
    assert out["diagnostics"]["chains"] == 2
    assert "chains2" in out["config"]["parallelism"]
