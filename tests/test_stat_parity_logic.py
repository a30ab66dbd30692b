"""CPU checks of the statistical-parity machinery (tests/stat_parity.py) on synthetic chain errors:
the mode clustering finds well-separated modes and ignores a few outlying chains, and the
mode-conditional z statistic accepts oracle values drawn from the GPU chains' own distribution and
rejects a shift of a fraction of a percent."""
import numpy as np

import stat_parity as sp


def _rows(rng, R=6, M=16, shift=0.0, modes=(0.486, 0.517), sd=0.001, outliers=1):
    rows = []
    for r in range(R):
        pick = rng.random(M) < 0.5
        g = np.where(pick, modes[1], modes[0]) + sd * rng.standard_normal(M)
        if r < outliers:
            g[0] = 0.57                                    # a chain that spent time in an excursion
        o = (modes[1] if rng.random() < 0.5 else modes[0]) + sd * rng.standard_normal() + shift
        rows.append({"gpu_fro_rel": g.tolist(), "oracle_fro_rel": float(o)})
    return rows


def test_clusters_find_the_modes():
    rng = np.random.default_rng(1)
    rows = _rows(rng)
    g = np.concatenate([r["gpu_fro_rel"] for r in rows])
    parts, _ = sp._clusters(g)
    major = [p for p in parts if len(p[2]) >= 0.1 * len(g)]
    assert len(major) == 2
    assert abs(np.median(major[0][2]) - 0.486) < 1e-3 and abs(np.median(major[1][2]) - 0.517) < 1e-3


def test_mode_conditional_accepts_parity_and_rejects_a_shift():
    rng = np.random.default_rng(2)
    zs = [sp._mode_conditional(_rows(rng), "fro_rel")["z"] for _ in range(200)]
    assert np.mean(np.abs(zs) < sp.Z99) > 0.95                 # ~1 % false alarms under parity
    shifted = [sp._mode_conditional(_rows(rng, shift=0.003), "fro_rel")["z"] for _ in range(50)]
    assert np.mean(np.abs(shifted) > sp.Z99) > 0.9             # a 0.6 % shift is caught


def test_unimodal_errors_have_no_modes():
    rng = np.random.default_rng(3)
    rows = [{"gpu_fro_rel": (0.5 + 0.01 * rng.standard_normal(16)).tolist(), "oracle_fro_rel": 0.5}
            for _ in range(6)]
    assert sp._mode_conditional(rows, "fro_rel") is None
