"""Dev (CPU): replay the iteration tools/dev/nan_hunt.py found non-finite on the GPU, through the
faithful per-row oracle (oracle/dc_oracle.py, dc:97-177 stage by stage) from the GPU's last finite
state with the same variates, and report which stage first goes non-finite (or fails, as MATLAB's
chol would) and the conditioning it meets there.

  python tools/dev/nan_replay.py gpurun_out/nan_hunt_c2_11.npz
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from helpers import make_case  # noqa: E402
from oracle import IterDraws, SamplerState  # noqa: E402
from oracle import dc_oracle as F  # noqa: E402

SHAPES = {"c2": (500, 5000, 8, 20), "c4": (2000, 10000, 8, 100)}


def finite(st):
    return {f: bool(np.all(np.isfinite(v))) for f, v in st.as_dict().items()}


def main(path):
    z = np.load(path)
    shape = Path(path).stem.split("_")[2]
    n, p, g, K = SHAPES[shape]
    c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
    fields = ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "delta", "tauh")
    st = SamplerState(**{f: np.array(z[f"st_{f}"], dtype=np.float64, order="F") for f in fields},
                      eta=np.zeros((c["n"], K, g), order="F"))
    F.update_eta(st, c["rho"])
    d = IterDraws(**{k: np.asarray(z[f"dr_{k}"])[..., 0] for k in ("NZ", "NX", "NL", "Gpsi", "Gdelta", "Gps")})
    it = int(z["iteration"])
    print(f"iteration {it}: start max|X| {np.abs(st.X).max():.3g}, min ps {st.ps.min():.3g}, "
          f"max tau {st.tauh.max():.3g}, max |Lambda| {np.abs(st.Lambda).max():.3g}")
    hyper = c["hyper"]
    np.seterr(all="warn")
    for name, fn in (("Z dc:97-108", lambda: F.update_Z(st, c["Yd"], c["rho"], d)),
                     ("X dc:112-129", lambda: F.update_X(st, c["Yd"], c["rho"], d)),
                     ("eta dc:132-134", lambda: F.update_eta(st, c["rho"])),
                     ("Lambda dc:137-145", lambda: F.update_Lambda(st, c["Yd"], d)),
                     ("psi dc:149-152", lambda: F.update_psi(st, hyper, d)),
                     ("delta/tau dc:155-165", lambda: F.update_delta_tau(st, hyper, d)),
                     ("ps dc:168-172", lambda: F.update_ps(st, c["Yd"], hyper, d)),
                     ("Plam dc:175-177", lambda: F.update_Plam(st))):
        try:
            fn()
        except Exception as e:  # noqa: BLE001
            print(f"{name}: raised {type(e).__name__}: {e}")
            return
        bad = [f for f, ok in finite(st).items() if not ok]
        eta = st.eta
        E = np.einsum("ikm,ilm->mkl", eta, eta)
        print(f"{name}: non-finite {bad or 'none'}; max|X| {np.abs(st.X).max():.3g} max|Z| {np.abs(st.Z).max():.3g} "
              f"cond(E_m) max {max(np.linalg.cond(E[m]) for m in range(g)):.3g} min ps {st.ps.min():.3g} "
              f"max tau {st.tauh.max():.3g}")
        if bad:
            return


if __name__ == "__main__":
    main(sys.argv[1])
