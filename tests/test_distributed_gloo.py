"""world_size-2 gloo test of the multi-GPU decomposition (CPU): two ranks, each
owning half the shards, exchanging exactly what libdcfm exchanges over RCCL,
reproduce the single-process oracle chain and Sigmaout."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


CASE = dict(n=24, p=36, g=4, K=3, burnin=1, mcmc=4, thin=2, seed=21)


def _setup():
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    from helpers import make_case
    c = make_case(CASE["n"], CASE["p"], CASE["g"], CASE["K"], seed=CASE["seed"])
    return c


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = _setup()
        from sharded_protocol import RankChain
        g, G = c["g"], c["g"] // world
        s0 = rank * G
        loc = {}
        for f in ("Lambda", "ps", "omega", "psi", "Plam", "Z", "eta"):
            loc[f] = getattr(c["st"], f)[..., s0:s0 + G]
        for f in ("X", "delta", "tauh"):
            loc[f] = getattr(c["st"], f)
        rc = RankChain(c["Yd"][:, :, s0:s0 + G], loc, g, c["rho"], c["hyper"])
        p = c["P"] * g
        Sig = np.zeros((p, p))
        N = CASE["burnin"] + CASE["mcmc"]
        effsamp = CASE["mcmc"] / CASE["thin"]
        for it in range(1, N + 1):
            rc.iteration(c["src"].iteration(it))
            if it % CASE["thin"] == 0 and it > CASE["burnin"]:
                rc.save_and_assemble(Sig, effsamp)
        full = RankChain.gather_sigma(Sig)                  # rank 0 only (block-sharded output)
        extra = {"Sig": full} if rank == 0 else {}
        np.savez(Path(outdir) / f"rank{rank}.npz", X=rc.st["X"], delta=rc.st["delta"],
                 tauh=rc.st["tauh"], Lambda=rc.st["Lambda"], ps=rc.st["ps"], Sig_local=Sig, **extra)
    finally:
        dist.destroy_process_group()


def test_two_rank_protocol_matches_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    c = _setup()
    from oracle import vectorised as V
    st = c["st"].copy()
    N = CASE["burnin"] + CASE["mcmc"]
    S_ref = V.full(V.run_chain(c["Yd"], st, c["rho"], c["hyper"], c["src"].iteration, 1, N,
                               CASE["burnin"], CASE["mcmc"], CASE["thin"]))
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    rel = lambda a, b: np.max(np.abs(a - b)) / np.max(np.abs(b))
    # replicated quantities identical on both ranks, bit for bit
    for f in ("X", "delta", "tauh"):
        assert np.array_equal(r0[f], r1[f]), f
    # each rank holds only its block of tile rows; the blocks are disjoint and cover Sigmaout
    from sharded_protocol import sigma_split
    p = S_ref.shape[0]
    Tb = sigma_split(-(-p // 8), world)
    for k, r in enumerate((r0, r1)):
        rows = np.zeros(p, bool)
        rows[min(p, Tb[k] * 8):min(p, Tb[k + 1] * 8)] = True
        assert not np.any(r["Sig_local"][~rows]), f"rank {k} wrote rows it does not own"
    assert "Sig" not in r1.files
    assert rel(r0["Sig"], S_ref) < 1e-12
    assert rel(r0["X"], st.X) < 1e-12
    assert rel(r0["delta"], st.delta) < 1e-12
    G = c["g"] // world
    assert rel(np.concatenate([r0["Lambda"], r1["Lambda"]], axis=2), st.Lambda) < 1e-12
    assert rel(np.concatenate([r0["ps"], r1["ps"]], axis=2), st.ps) < 1e-12
