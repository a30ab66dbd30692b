"""Dev probe (GPU): the first iteration at which a generated-draw chain turns non-finite.

Runs the chain in chunks, then steps the failing chunk one iteration at a time from the last
finite state, and saves that state plus the iteration's variates (dcfm_rng_fill at the sweep's
counters, K <= 32 only) to gpurun_out/nan_hunt_<shape>_<seed>.npz, so the oracle can replay the
same iteration on the CPU (which stage goes non-finite, and whether the reference's algebra
does too).

  python tools/dev/nan_hunt.py --shape c2 --seed 11
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as ge  # noqa: E402
from helpers import make_case, state_dict  # noqa: E402
from test_gpu_generated_draws import _draws  # noqa: E402

SHAPES = {"c2": (500, 5000, 8, 20), "c4": (2000, 10000, 8, 100)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c2")
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=20)
    ap.add_argument("--flags", type=int, default=0)
    a = ap.parse_args()
    n, p, g, K = SHAPES[a.shape]
    dcfm = ge.load_package()
    c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
    st = {f: v for f, v in state_dict(c["st"]).items() if f != "eta"}

    def chain(state, first, count, step):
        smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 10 ** 6, 0, 1, seed=a.seed, flags=a.flags)
        good, it = state, first
        try:
            smp.set_data(c["Yd"])
            smp.set_state(state)
            while it < first + count:
                try:
                    smp.run(it, step)
                    s = smp.get_state()
                except Exception as e:  # noqa: BLE001
                    return good, it, str(e)
                good = {f: v for f, v in s.items() if f != "eta"}
                it += step
        finally:
            smp.close()
        return good, it, None

    good, it, err = chain(st, 1, a.iters, a.chunk)
    if err is None:
        print(f"{a.shape} seed {a.seed} flags {a.flags}: finite through {a.iters} iterations")
        return
    print(f"chunk failure at [{it}, {it + a.chunk}): {err}")
    good, it, err = chain(good, it, a.chunk, 1)
    assert err is not None
    x = np.abs(good["X"]).max()
    print(f"first non-finite iteration {it}; before it max|X| {x:.3g} min ps {good['ps'].min():.3g} "
          f"max ps {good['ps'].max():.3g} max|Lambda| {np.abs(good['Lambda']).max():.3g} "
          f"max tau {good['tauh'].max():.3g} min tau {good['tauh'].min():.3g}")
    out = {f"st_{f}": v for f, v in good.items()}
    if K <= 32:
        dr = _draws(dcfm, a.seed, c["n"], c["P"], g, K, it, 1, dcfm.Hyper())
        out.update({f"dr_{k}": v for k, v in dr.items()})
    Path("gpurun_out").mkdir(exist_ok=True)
    np.savez(f"gpurun_out/nan_hunt_{a.shape}_{a.seed}.npz", iteration=it, **out)
    # the same iteration with the reference's residual for every row (DCFM_FLAG_EXACT_RESIDUAL)
    if a.flags == 0:
        smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 10 ** 6, 0, 1, seed=a.seed, flags=0x10)
        try:
            smp.set_data(c["Yd"])
            smp.set_state(good)
            smp.run(it, 1)
            s = smp.get_state()
            print(f"exact-residual mode at iteration {it}: finite, max|X| {np.abs(s['X']).max():.3g}")
        except Exception as e:  # noqa: BLE001
            print(f"exact-residual mode at iteration {it}: {e}")
        finally:
            smp.close()


if __name__ == "__main__":
    main()
