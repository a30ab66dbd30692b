"""Summarise rocprofv3 PMC passes per kernel (tools/profile_round.sh output).

HBM bytes per dispatch: FETCH_SIZE (KiB) x 1024 x 2 — the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts exactly
half of the bytes of a wide (16 B/lane) coalesced read — and WRITE_SIZE (KiB) x
1024 as is.  Calibrated here for the widths these kernels use (tools/calib/
calib_fetch.hip, 2 GiB streamed, profiles/r01_fetch_calibration.txt): 8 B/lane and
16 B/lane coalesced reads both report 0.500 of their bytes, 8 B/lane and 16 B/lane
stores 1.000 — so the x2 / x1 corrections hold for every kernel in this library.  Both include Infinity-Cache hits (memory-side requests), so on a
working set that stays MALL-resident they are an upper bound on HBM traffic.
fp64 MFMA flops: SQ_INSTS_VALU_MFMA_MOPS_F64 x 512.  MFMA busy share:
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) — GRBM_GUI_ACTIVE is summed
over the 8 XCDs (MI355X guide), so it is divided back to per-XCD cycles.  Per-dispatch
lists (dispatch order) let bench.py take the timed region's launches; the summary carries
the profiled bench's build id and config key (from its JSON line), and bench.py only uses
a summary whose build and config equal its own.
Usage: python tools/pmc_summary.py gpurun_out/prof_TAG > profiles/..._pmc.json
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def load(dirpat):
    rows = []
    for f in glob.glob(f"{dirpat}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def per_kernel(rows, counter):
    """kernel -> (mean over dispatches, dispatch count, per-dispatch values in dispatch order);
    a counter's instances (per XCD / per SE) are summed within a dispatch."""
    acc = defaultdict(lambda: defaultdict(float))
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = short(r["Kernel_Name"])
        acc[k][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for k, v in acc.items():
        each = [v[i] for i in sorted(v)]
        out[k] = (sum(each) / len(each), len(each), each)
    return out


def bench_meta(base):
    """build id and config key of the profiled bench command (its JSON line in the pass log)."""
    for suffix in ("_fetch.log", "_write.log", ".log"):
        try:
            for ln in open(base + suffix):
                ln = ln.strip()
                if ln.startswith("{") and '"metric"' in ln:
                    d = json.loads(ln)
                    return d.get("build"), d.get("config_key")
        except OSError:
            continue
    return None, None


NXCD = 8          # GRBM_GUI_ACTIVE is reported summed over the 8 XCDs (MI355X guide, DVFS note)
NSIMD = 256 * 4   # SQ_VALU_MFMA_BUSY_CYCLES: summed over every SIMD of the chip

base = sys.argv[1]
fetch = per_kernel(load(base + "_fetch"), "FETCH_SIZE")
write = per_kernel(load(base + "_write"), "WRITE_SIZE")
mrows = load(base + "_mfma")
mops = per_kernel(mrows, "SQ_INSTS_VALU_MFMA_MOPS_F64")
busy = per_kernel(mrows, "SQ_VALU_MFMA_BUSY_CYCLES")
gui = per_kernel(mrows, "GRBM_GUI_ACTIVE")
out = {}
for k in sorted(set(fetch) | set(write) | set(mops)):
    e = {}
    if k in fetch:
        e["fetch_bytes_per_dispatch"] = fetch[k][0] * 1024 * 2
        e["dispatches"] = fetch[k][1]
        e["fetch_bytes_each"] = [v * 1024 * 2 for v in fetch[k][2]]
    if k in write:
        e["write_bytes_per_dispatch"] = write[k][0] * 1024
        e["write_bytes_each"] = [v * 1024 for v in write[k][2]]
    if "fetch_bytes_per_dispatch" in e and "write_bytes_per_dispatch" in e:
        e["hbm_bytes_per_dispatch"] = e["fetch_bytes_per_dispatch"] + e["write_bytes_per_dispatch"]
    if k in mops:
        e["mfma_f64_flops_per_dispatch"] = mops[k][0] * 512
        e["mfma_f64_flops_each"] = [v * 512 for v in mops[k][2]]
    if k in busy and k in gui and gui[k][0] > 0:
        # MFMA pipe busy share: busy cycles summed over the chip's SIMDs / (the dispatch's
        # active cycles per XCD x SIMDs); GRBM_GUI_ACTIVE is the sum over the 8 XCD instances
        e["mfma_busy_frac"] = busy[k][0] / (gui[k][0] / NXCD * NSIMD)
        e["mfma_busy_frac_each"] = [b / (c / NXCD * NSIMD) if c > 0 else None
                                    for b, c in zip(busy[k][2], gui[k][2])]
        e["gui_cycles_per_xcd"] = gui[k][0] / NXCD
    out[k] = e
# wave-state pass (quad-cycle units): active / issue-stalled / parked shares of wave time
wrows = load(base + "_waves")
if wrows:
    wc = {c: per_kernel(wrows, c) for c in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                            "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU",
                                            "SQ_INSTS_LDS")}
    for k, (cyc, _, _) in wc["SQ_WAVE_CYCLES"].items():
        if cyc <= 0 or k not in out:
            continue
        e = out[k]
        e["waves_per_dispatch"] = wc["SQ_WAVES"].get(k, (0, 0))[0]
        e["valu_insts_per_wave"] = wc["SQ_INSTS_VALU"].get(k, (0, 0))[0] / max(1.0, e["waves_per_dispatch"])
        e["lds_insts_per_wave"] = wc["SQ_INSTS_LDS"].get(k, (0, 0))[0] / max(1.0, e["waves_per_dispatch"])
        for c, name in (("SQ_ACTIVE_INST_ANY", "active_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                        ("SQ_WAIT_ANY", "parked_frac"), ("SQ_ACTIVE_INST_VALU", "valu_active_frac")):
            e[name] = wc[c].get(k, (0, 0))[0] / cyc
build, config = bench_meta(base)
json.dump({"source": base, "build": build, "config": config, "kernels": out}, sys.stdout, indent=1)
print()
