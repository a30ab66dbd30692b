"""Dev aid: run a generated-draw chain at a config's shape and save its state (compare two library builds
bit for bit: DCFM_LIB=<build A> python tools/dev/bitcmp.py c4 a.npz; DCFM_LIB=<build B> ... b.npz;
python tools/dev/bitcmp.py --cmp a.npz b.npz)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
SHAPES = {"c2": (500, 5000, 8, 20), "c4": (2000, 10000, 8, 100), "c3": (1000, 19968, 64, 30), "w40": (400, 2000, 4, 40)}

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print("bitwise equal" if not bad else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)
import __graft_entry__ as ge  # noqa: E402
from helpers import make_case, state_dict  # noqa: E402
n, p, g, K = SHAPES[sys.argv[1]]
dcfm = ge.load_package()
c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 2, 8, 2, seed=5)
smp.set_data(c["Yd"])
smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
smp.run(1, 10)
st = smp.get_state()
st["Sigma_cols"] = smp.get_sigma_cols(0, 256)
np.savez(sys.argv[2], **st)
print("saved", sys.argv[2])
