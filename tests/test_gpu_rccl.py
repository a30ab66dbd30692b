"""The real multi-rank path of libdcfm (RCCL all-gathers inside dcfm_run, the RCCL
send/recv gather of the block-sharded Sigmaout in dcfm_get_sigma) with one process per
GPU, up to 8 ranks.

Needs >= 2 devices (RCCL refuses two ranks on one device): it is skipped only then.  On
a multi-GPU node any communicator or collective failure FAILS the test.  With injected
draws the multi-rank chain must reproduce the single-process oracle to the same 1e-10
bar as tests/test_gpu_parity.py, the replicated quantities (X, delta, tau) must be
bitwise identical on all ranks, and rank 0 alone receives Sigmaout.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
CASE = dict(n=40, p=2048, g=8, K=5, burnin=1, mcmc=4, thin=2, seed=13)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _case():
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    from helpers import make_case, stacked_draws
    c = make_case(CASE["n"], CASE["p"], CASE["g"], CASE["K"], seed=CASE["seed"])
    N = CASE["burnin"] + CASE["mcmc"]
    return c, stacked_draws(c["src"], 1, N), N


def _worker(rank, world, port, outdir, ndev):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)   # rendezvous only
    try:
        import __graft_entry__ as ge
        from helpers import state_dict
        dcfm = ge.load_package()
        c, draws, N = _case()
        g, G = CASE["g"], CASE["g"] // world
        s0 = rank * G
        smp = dcfm.Sampler(c["n"], c["P"], g, CASE["K"], c["rho"], CASE["burnin"], CASE["mcmc"], CASE["thin"],
                           inject_draws=True, nranks=world, rank=rank, device=rank % ndev)
        obj = [dcfm.Sampler.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        smp.comm_init(obj[0])                  # a failure here fails the test (raised in the worker)
        smp.set_data(c["Yd"][:, :, s0:s0 + G])
        st = state_dict(c["st"], s0, G)
        smp.set_state({f: st[f] for f in st if f != "eta"})
        smp.set_draws(draws, 1, N)
        smp.run(1, N)
        got = smp.get_state()
        S = smp.get_sigma()                    # collective; rank 0 receives
        blk = smp.sigma_block()
        smp.close()
        extra = {"Sig": S} if rank == 0 else {}
        np.savez(Path(outdir) / f"rank{rank}.npz", row0=blk["row0"], row1=blk["row1"], **extra, **got)
    finally:
        dist.destroy_process_group()


def test_ranks_match_oracle(tmp_path, gpu_available):
    if not gpu_available:
        pytest.skip("no GPU")
    import torch
    ndev = torch.cuda.device_count()
    if ndev < 2:
        pytest.skip(f"RCCL needs one device per rank; {ndev} device(s) here")
    world = max(w for w in (2, 4, 8) if w <= ndev)   # divides g = 8
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), ndev), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / f"rank{k}.npz") for k in range(world)]
    c, draws, N = _case()
    from oracle import dc_oracle as F
    from helpers import rel_err
    ref = c["st"].copy()
    S_ref = F.run_chain(c["Yd"], ref, c["rho"], c["hyper"], c["src"].iteration, 1, N, CASE["burnin"],
                        CASE["mcmc"], CASE["thin"])
    for k in range(1, world):
        for f in ("X", "delta", "tauh"):
            assert np.array_equal(r[0][f], r[k][f]), f"{f} differs between ranks 0 and {k}"
        assert "Sig" not in r[k].files
        assert int(r[k]["row0"]) == int(r[k - 1]["row1"])
    assert int(r[0]["row0"]) == 0 and int(r[-1]["row1"]) == c["p"]
    assert rel_err(r[0]["Sig"], S_ref) < 1e-10
    for f in ("X", "delta", "tauh"):
        assert rel_err(r[0][f], getattr(ref, f)) < 1e-10, f
    for f in ("Lambda", "ps", "omega", "psi", "Plam", "Z", "eta"):
        both = np.concatenate([r[k][f] for k in range(world)], axis=-1)
        assert rel_err(both, getattr(ref, f)) < 1e-10, f


COMM_SELF = 0x20   # DCFM_FLAG_COMM_SELF


@pytest.mark.parametrize("K,flags", [(5, 0), (30, 0), (40, 0), (5, 0x2)])   # fused, fused c3 width, wide, unfused
def test_one_rank_rccl_communicator(dcfm, K, flags):
    """RCCL on a ONE-GPU box: a one-rank chain with DCFM_FLAG_COMM_SELF takes the collective data
    path (packed all-gather per iteration, side / assembly all-gathers, agree()'s all-reduce in
    get_sigma and the Lanczos all-reduces of sigma_error) through a real one-rank RCCL
    communicator (ncclGetUniqueId, ncclCommInitRank, ncclCommSplit x 2, ncclAllGather,
    ncclAllReduce).  Its results must be bitwise those of the plain one-rank chain, which skips
    every collective; the 'rccl' kernel-stat counter proves the calls ran."""
    from helpers import make_case, stacked_draws, state_dict
    n, p, g, burnin, mcmc, thin = 40, 256, 4, 1, 4, 2
    c = make_case(n, p, g, K, seed=21)
    N = burnin + mcmc
    draws = stacked_draws(c["src"], 1, N)
    _, _, L0, s2 = __import__("oracle").synth.make_data(n, p, k0=4, factors=True)
    U, s = dcfm.truth_factors(L0, s2, c["Y"], c["keep"], c["init"].varind)
    out = []
    for f in (flags, flags | COMM_SELF):
        smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True, flags=f)
        try:
            if f & COMM_SELF:
                smp.comm_init(dcfm.Sampler.unique_id())
            smp.set_data(c["Yd"])
            smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
            smp.set_draws(draws, 1, N)
            smp.set_profiling_kernels(["rccl"])
            smp.run(1, N)
            comm = smp.kernel_stats()["rccl"][1]
            got = smp.get_state()
            got["Sig"] = smp.get_sigma()
            got["err"] = np.array([v for v in smp.sigma_error(U, s, iters=20).values()])
            out.append((got, comm))
        finally:
            smp.close()
    (plain, c0), (rccl, c1) = out
    assert c0 == 0 and c1 >= N, (c0, c1)
    for f in plain:
        assert np.array_equal(plain[f], rccl[f]), f"{f} differs with the one-rank RCCL communicator"
