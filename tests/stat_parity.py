"""north_star check (2), shared by tests/test_gpu_c{2,3}_parity.py: the GPU chain's posterior-mean
Sigmaout has the oracle chain's Frobenius and operator-norm error against the synthetic truth,
within Monte Carlo error (divideconquer.m:180-196).

Design.  Case r fixes the data set and the driver's init / partition draws
(oracle.DrawSource(case_seed_r)).  The oracle leg is ONE chain per case (NumPy draws, dc:169's
direct residual; tests/golden/make_c{2,3}_parity.py, ~72 min per case at c3).  The GPU leg runs M
chains per case from the same data and initial state with independent on-device Philox draws, which
measures the chain-to-chain spread of the error on the GPU side, where chains are cheap.  The spread
is large and not Gaussian: at c3 (MCMC 1,500) single-chain errors cluster near 0.486 and 0.516 with
rare larger ones (a chain that spent time in an X excursion), so the oracle's few replicates cannot
estimate it themselves.  A GPU chain whose excursion escalates to the reference's own breakdown
(DCFM_ERR_NUMERIC where dc:142's chol fails; tests/test_gpu_excursion.py) has no posterior mean: it is
counted, left out of the error statistics, and the oracle's R completed chains are checked against the
GPU chains' breakdown rate (P(no breakdown in R) > 1 %).

Under parity the oracle chain's error o_r is one more draw from the GPU chains' distribution for
case r, so d_r = o_r - mean_r(gpu) has mean 0 and variance s_r^2 (1 + 1/M), s_r the GPU chains' sd.
The test passes when
    |z| < 2.576,   z = sum_r d_r / sqrt(sum_r s_r^2 (1 + 1/M))     (two-sided 1 %)
for both norms.  The bar in error units, 2.576 sqrt(sum_r s_r^2 (1 + 1/M)) / R, is what R oracle
replicates can resolve; it is reported with each oracle value's percentile among its case's GPU
chains (a Kolmogorov-Smirnov test of those percentiles against Uniform(0, 1) at 1 %).  Where the
chains' errors fall into well-separated modes (c2, c3), the same comparison also runs within the modes
(each oracle value against the GPU chains of the major mode it falls in) -- a bar of a fraction of a
percent where the unconditional one is a few percent; an oracle value outside every major mode counts
against the check (_mode_conditional).  Everything
goes to gpurun_out/<name>_parity_gpu.json (kept under profiles/ per round)."""
from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np
from scipy import stats

import oracle
from helpers import make_case, state_dict

Z99 = 2.5758293035489004       # two-sided 1 % normal quantile
DCFM_ERR_NUMERIC = 5           # include/dcfm.h
M_CHAINS = 16


def _clusters(x, gap_factor=20.0):
    """Modes of the GPU chains' errors: the sorted values split wherever consecutive values lie more than
    gap_factor times the median consecutive spacing apart.  Returns [(lo, hi, values)]."""
    v = np.sort(np.asarray(x))
    gaps = np.diff(v)
    thr = gap_factor * max(float(np.median(gaps)), 1e-12)
    cuts = np.nonzero(gaps > thr)[0]
    parts = np.split(v, cuts + 1)
    return [(float(p_[0]), float(p_[-1]), p_) for p_ in parts], thr


MODE_WINDOW = 10.0             # a value belongs to a major mode within this many of the mode's sds


def _mode_conditional(rows, key):
    """Where the GPU chains' errors fall into well-separated modes (c2, c3: a few posterior modes that a
    chain settles in), the sharper check: each oracle value against the GPU chains of the major mode
    (>= 10 % of the chains; outlying chains fall in modes of their own) nearest to it, if it lies within
    MODE_WINDOW of that mode's sds -- z as in the unconditional test, with the mode's MEAN and SD (under
    parity o - mean has expectation 0 whatever the mode's shape; o - median does not when the mode is
    skewed, and the GPU modes are: skewness ~2 at c2 / c3).

    An oracle value outside every major mode is not dropped silently: such values are counted, and
    under parity they occur at the rate q at which the GPU chains themselves fall outside every major
    mode (same window; q = (outside + 1) / (M + 2)), so their count must not be improbably high:
    P(Binomial(R, q) >= count) > 1 %.  Fewer than 3 oracle values inside the modes fails the check.
    None when the errors have fewer than two major modes."""
    g = np.concatenate([np.asarray(r[f"gpu_{key}"]) for r in rows])
    parts, thr = _clusters(g)
    major = [v for lo, hi, v in parts if len(v) >= 0.1 * len(g) and len(v) >= 5]
    if len(major) < 2:
        return None
    mus = np.array([float(np.mean(v)) for v in major])
    sds = np.array([float(np.std(v, ddof=1)) for v in major])
    # the gap split only seeds the modes: it cuts a skewed mode's tail into minor clusters, which would
    # bias the mode's mean toward its median and shrink its sd.  Membership is the rule the oracle values
    # get -- the nearest mode, within MODE_WINDOW of its sds -- applied to every GPU chain, to a fixed point.
    for _ in range(20):
        k = np.argmin(np.abs(g[:, None] - mus[None, :]), axis=1)
        member = np.abs(g - mus[k]) <= MODE_WINDOW * sds[k]
        groups = [g[member & (k == i)] for i in range(len(mus))]
        if min(len(v) for v in groups) < 5:
            break
        new_mus = np.array([float(np.mean(v)) for v in groups])
        new_sds = np.array([float(np.std(v, ddof=1)) for v in groups])
        done = np.array_equal(new_mus, mus) and np.array_equal(new_sds, sds)
        mus, sds = new_mus, new_sds
        if done:
            break
    k = np.argmin(np.abs(g[:, None] - mus[None, :]), axis=1)
    member = np.abs(g - mus[k]) <= MODE_WINDOW * sds[k]
    ns = np.array([int(np.sum(member & (k == i))) for i in range(len(mus))])
    gpu_outside = int(np.sum(~member))
    q = (gpu_outside + 1.0) / (len(g) + 2.0)
    o = np.array([r[f"oracle_{key}"] for r in rows])
    d, var, which = [], [], []
    for ov in o:
        k = int(np.argmin(np.abs(ov - mus)))
        if abs(ov - mus[k]) > MODE_WINDOW * sds[k]:
            which.append(None)
            continue
        which.append(k)
        d.append(ov - mus[k])
        var.append(sds[k] ** 2 * (1.0 + 1.0 / ns[k]))
    n_out = len(o) - len(d)
    p_out = float(stats.binom.sf(n_out - 1, len(o), q)) if n_out else 1.0
    res = {"modes": [{"mean": float(m), "sd": float(sd), "count": int(n)} for m, sd, n in zip(mus, sds, ns)],
           "minor_chains": int(len(g) - ns.sum()), "oracle_mode": which, "n_used": len(d),
           "oracle_outside": n_out, "oracle_outside_values": [float(v) for v, w in zip(o, which) if w is None],
           "gpu_outside": gpu_outside, "gpu_chains": int(len(g)), "q_outside": q, "p_outside": p_out}
    if len(d) < 3:
        return {**res, "z": float("nan"), "mean_diff": float("nan"), "bar": float("nan"), "bar_rel": float("nan"),
                "ok": False}
    scale = float(np.sqrt(np.sum(var)))
    z = float(np.sum(d) / scale)
    return {**res, "z": z, "mean_diff": float(np.mean(d)), "bar": Z99 * scale / len(d),
            "bar_rel": Z99 * scale / len(d) / float(np.mean(o)), "ok": abs(z) < Z99 and p_out > 0.01}


def run_paired(dcfm, fixture: Path, name: str, seed0: int, dense_truth: bool, record_property=None,
               m_chains: int = M_CHAINS):
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
        fro, op, broke = [], [], []
        for k in range(m_chains):
            smp = dcfm.Sampler(c["n"], c["P"], g, K, rho, burnin, mcmc, thin, seed=seed0 + 100 * rec["rep"] + k)
            try:
                smp.set_data(c["Yd"])
                smp.set_state({kk: v for kk, v in state_dict(c["st"]).items() if kk != "eta"})
                try:
                    smp.run(1, burnin + mcmc)
                    e = smp.sigma_error(U, s, iters=120)
                except dcfm.DcfmError as err:       # the reference's own breakdown (chol of dc:142 fails)
                    assert err.code == DCFM_ERR_NUMERIC, err
                    broke.append(seed0 + 100 * rec["rep"] + k)
                    continue
            finally:
                smp.close()
            assert abs(e["truth_fro"] / rec["truth_fro"] - 1) < 1e-9      # same truth, same coordinates
            fro.append(e["fro"] / rec["truth_fro"])
            op.append(e["op"] / rec["truth_op"])
        assert len(fro) >= m_chains // 2, f"case {rec['rep']}: {len(broke)} of {m_chains} chains broke down"
        rows.append({"rep": rec["rep"], "case_seed": rec["case_seed"], "gpu_seeds": [seed0 + 100 * rec["rep"], m_chains],
                     "gpu_broke_down": broke, "gpu_fro_rel": fro, "oracle_fro_rel": rec["fro_rel"], "gpu_op_rel": op,
                     "oracle_op_rel": rec["op_rel"]})
    R = len(rows)
    n_broke = sum(len(r["gpu_broke_down"]) for r in rows)
    summary = {"config": name, "params": prm, "R": R, "m_chains": m_chains, "z_crit": Z99,
               "oracle_direct_residual": bool(doc.get("direct", False)),
               "gpu_chains_broke_down": n_broke, "gpu_chains": R * m_chains,
               # the oracle's R chains all completed: how likely is that at the GPU chains' breakdown rate
               "p_oracle_none_broke": float((1.0 - n_broke / (R * m_chains)) ** R), "replicates": rows}
    verdicts = {}
    for key in ("fro_rel", "op_rel"):
        mu = np.array([np.mean(r[f"gpu_{key}"]) for r in rows])
        sd = np.array([np.std(r[f"gpu_{key}"], ddof=1) for r in rows])
        nk = np.array([len(r[f"gpu_{key}"]) for r in rows])
        o = np.array([r[f"oracle_{key}"] for r in rows])
        d = o - mu
        scale = float(np.sqrt(np.sum(sd ** 2 * (1.0 + 1.0 / nk))))
        z = float(np.sum(d) / scale)
        base = float(np.mean(o))
        pct = [float(np.mean(np.asarray(r[f"gpu_{key}"]) < r[f"oracle_{key}"])) for r in rows]
        summary[key] = {"z": z, "mean_diff": float(np.mean(d)), "bar": Z99 * scale / R, "bar_rel": Z99 * scale / R / base,
                        "mean_oracle": base, "mean_gpu": float(np.mean(mu)), "gpu_sd_per_case": sd.tolist(),
                        "oracle_percentile_among_gpu_chains": pct}
        verdicts[key] = abs(z) < Z99
        # the oracle values' percentiles among their cases' GPU chains are Uniform(0, 1) under parity
        summary[key]["ks_p"] = float(stats.kstest(pct, "uniform").pvalue)
        verdicts[key] = verdicts[key] and summary[key]["ks_p"] > 0.01
        modal = _mode_conditional(rows, key)
        if modal is not None:
            summary[key]["modes"] = modal
            verdicts[key] = verdicts[key] and modal["ok"]
    out = Path(os.environ.get("DCFM_PARITY_OUT", "gpurun_out"))
    out.mkdir(parents=True, exist_ok=True)
    (out / f"{name}_parity_gpu.json").write_text(json.dumps(summary, indent=1) + "\n")
    if record_property is not None:
        for key in ("fro_rel", "op_rel"):
            for f in ("z", "mean_diff", "bar", "bar_rel"):
                record_property(f"{key}_{f}", summary[key][f])
    print(f"{name.upper()}_PARITY", json.dumps({k: {**{kk: summary[k][kk] for kk in ("z", "mean_diff", "bar_rel")},
                                                     "ks_p": summary[k]["ks_p"],
                                                     **({"modes": {kk: summary[k]["modes"][kk] for kk in
                                                                   ("z", "bar_rel", "n_used", "oracle_outside",
                                                                    "p_outside")}}
                                                        if "modes" in summary[k] else {})}
                                                 for k in ("fro_rel", "op_rel")}))
    assert summary["p_oracle_none_broke"] > 0.01, ("breakdown rate", n_broke, R * m_chains)
    for key, ok in verdicts.items():
        assert ok, (key, summary[key])
    return summary
