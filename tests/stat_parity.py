"""north_star check (2), shared by tests/test_gpu_c{2,3}_parity.py: the GPU chain's posterior-mean
Sigmaout has the oracle chain's Frobenius and operator-norm error against the synthetic truth,
within Monte Carlo error (divideconquer.m:180-196).

Paired design: replicate r fixes the data set and the driver's init / partition draws
(oracle.DrawSource(case_seed_r)); the oracle leg (NumPy draws, dc:169's direct residual) ran in
the build container (tests/golden/make_c{2,3}_parity.py), the GPU leg runs from the same data and
initial state with independent on-device Philox draws.  d_r = err_gpu,r - err_oracle,r are then
independent across r with mean 0 under parity, and mean(d) / (sd(d) / sqrt(R)) is Student-t with
R - 1 degrees of freedom.  The test passes when
    |mean d| < t_{R-1, 0.995} sd(d) / sqrt(R)     (two-sided 99 %: fails 1 time in 100 under parity)
and |mean d| < CAP of the error (a fixed cap, so a noisy replicate set cannot widen the bar: 1 % for the
Frobenius error; 5 % for the operator norm, whose Monte Carlo spread is ~8x larger -- at c3 the oracle's
own replicates span 0.535-0.550).
Every replicate's GPU and oracle errors, the bars and the t statistics are written to
gpurun_out/<name>_parity_gpu.json (committed under profiles/ with the round's evidence)."""
from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np
from scipy import stats

import oracle
from helpers import make_case, state_dict

CAP = {"fro_rel": 0.01, "op_rel": 0.05}
ALPHA = 0.01


def run_paired(dcfm, fixture: Path, name: str, seed0: int, dense_truth: bool, record_property=None):
    doc = json.loads(fixture.read_text())
    prm, reps = doc["params"], doc["replicates"]
    n, p, g, K, rho = prm["n"], prm["p"], prm["g"], prm["K"], prm["rho"]
    burnin, mcmc, thin = prm["burnin"], prm["mcmc"], prm["thin"]
    Y, _, L0, sig2 = oracle.synth.make_data(n, p, k0=prm["k0"], factors=True, dense_truth=dense_truth)
    rows = []
    for rec in reps:
        c = make_case(n, p, g, K, seed=rec["case_seed"], k0=prm["k0"], rho=rho, dense_truth=dense_truth)
        assert np.array_equal(c["Y"], Y)
        U, s = dcfm.truth_factors(L0, sig2, Y, c["keep"], c["init"].varind)
        smp = dcfm.Sampler(c["n"], c["P"], g, K, rho, burnin, mcmc, thin, seed=seed0 + rec["rep"])
        try:
            smp.set_data(c["Yd"])
            smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
            smp.run(1, burnin + mcmc)
            e = smp.sigma_error(U, s, iters=120)
        finally:
            smp.close()
        assert abs(e["truth_fro"] / rec["truth_fro"] - 1) < 1e-9      # same truth, same coordinates
        rows.append({"rep": rec["rep"], "case_seed": rec["case_seed"], "gpu_seed": seed0 + rec["rep"],
                     "gpu_fro_rel": e["fro"] / rec["truth_fro"], "oracle_fro_rel": rec["fro_rel"],
                     "gpu_op_rel": e["op"] / rec["truth_op"], "oracle_op_rel": rec["op_rel"]})
    R = len(rows)
    tcrit = float(stats.t.ppf(1 - ALPHA / 2, R - 1))
    summary = {"config": name, "params": prm, "replicates": rows, "R": R, "t_crit": tcrit, "cap": CAP,
               "oracle_direct_residual": bool(doc.get("direct", False))}
    verdicts = {}
    for key in ("fro_rel", "op_rel"):
        d = np.array([r[f"gpu_{key}"] - r[f"oracle_{key}"] for r in rows])
        base = float(np.mean([r[f"oracle_{key}"] for r in rows]))
        se = float(np.std(d, ddof=1)) / np.sqrt(R)
        bar = tcrit * se
        summary[key] = {"mean_diff": float(np.mean(d)), "se": se, "t": float(np.mean(d)) / se if se > 0 else 0.0,
                        "bar": bar, "bar_rel": bar / base, "cap": CAP[key] * base, "mean_oracle": base,
                        "oracle_sd": float(np.std([r[f"oracle_{key}"] for r in rows], ddof=1)),
                        "gpu_sd": float(np.std([r[f"gpu_{key}"] for r in rows], ddof=1))}
        verdicts[key] = abs(float(np.mean(d))) < min(bar, CAP[key] * base)
    out = Path(os.environ.get("DCFM_PARITY_OUT", "gpurun_out"))
    out.mkdir(parents=True, exist_ok=True)
    (out / f"{name}_parity_gpu.json").write_text(json.dumps(summary, indent=1) + "\n")
    if record_property is not None:
        for key in ("fro_rel", "op_rel"):
            for f in ("mean_diff", "bar", "bar_rel", "t"):
                record_property(f"{key}_{f}", summary[key][f])
    print(f"{name.upper()}_PARITY", json.dumps({k: summary[k] for k in ("fro_rel", "op_rel")}))
    for key, ok in verdicts.items():
        assert ok, (key, summary[key], [(r[f"gpu_{key}"], r[f"oracle_{key}"]) for r in rows])
    return summary
