"""Dev probe (GPU): which Philox seeds make the reference sampler's X excursions at a config's shape.

Runs generated-draw chains from the case's initial state and prints max|X| and min ps every
`--step` iterations (a NaN surfaces as DCFM_ERR_NUMERIC from dcfm_run).  Used to pick the seed of
tests/test_gpu_excursion.py::test_c4_generated_chain_through_excursions.

  python tools/dev/excursion_probe.py --shape c4 --seeds 1-12 --iters 1000
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as ge  # noqa: E402
from helpers import make_case, state_dict  # noqa: E402

SHAPES = {"c2": (500, 5000, 8, 20), "c4": (2000, 10000, 8, 100), "c3": (1000, 19968, 64, 30)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c4")
    ap.add_argument("--seeds", default="1-8")
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--step", type=int, default=100)
    a = ap.parse_args()
    lo, hi = (int(x) for x in a.seeds.split("-"))
    n, p, g, K = SHAPES[a.shape]
    dcfm = ge.load_package()
    c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
    for seed in range(lo, hi + 1):
        smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 10 ** 6, 0, 1, seed=seed)
        xs, ok = [], True
        t0 = time.time()
        try:
            smp.set_data(c["Yd"])
            smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
            for it in range(1, a.iters + 1, a.step):
                try:
                    smp.run(it, a.step)
                    st = smp.get_state(("X", "ps"))
                except Exception as e:  # noqa: BLE001
                    print(f"seed {seed}: iteration {it}..{it + a.step - 1}: {e}", flush=True)
                    ok = False
                    break
                xs.append(float(np.abs(st["X"]).max()))
        finally:
            smp.close()
        print(f"{a.shape} seed {seed}: ok={ok} {time.time() - t0:.1f}s max|X| per {a.step}: "
              + " ".join(f"{v:.3g}" for v in xs), flush=True)


if __name__ == "__main__":
    main()
