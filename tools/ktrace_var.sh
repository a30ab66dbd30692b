#!/bin/bash
# Per-kernel trace averages (rocprofv3 --kernel-trace --stats, no counters) of one bench
# configuration for several library builds (dev aid, run on the GPU box): "main" = in-tree,
# NAME = build/libdcfm_NAME.so.  Usage: BENCH_ARGS="..." bash tools/ktrace_var.sh TAG NAME...
set -o pipefail
TAG=$1; shift
ARGS=${BENCH_ARGS:---gpus 1 --steps 40 --warmup 5}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
for V in "$@"; do
  LIB=$GRAFT_REPO_ROOT/a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/libdcfm.so
  [ "$V" != main ] && LIB=$GRAFT_REPO_ROOT/build/libdcfm_$V.so
  ( cd /tmp && DCFM_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kv_${TAG}_$V -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-profile --converged-mcmc 0 --err-iters 0 $ARGS > $OUT/kv_${TAG}_$V.log 2>&1 ) \
    || { echo "trace $V failed"; tail -5 $OUT/kv_${TAG}_$V.log; exit 1; }
  find $OUT/kv_${TAG}_$V -name "*kernel_trace.csv" -exec gzip -9 {} \;
  python3 - "$OUT/kv_${TAG}_$V" "$V" <<'PY'
import csv, glob, re, sys, json
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
out = []
for r in rows:
    m = re.search(r"(k_\w+)", r["Name"])
    if m and not m.group(1).startswith(("k_sigma_err", "k_rng", "k_nnz", "k_colstats", "k_stdize", "k_init")):
        out.append((m.group(1), int(r["Calls"]), float(r["AverageNs"]) / 1e3))
out.sort(key=lambda x: -x[1] * x[2])
print(f"{sys.argv[2]:10s} " + "  ".join(f"{k}={a:.1f}x{c}" for k, c, a in out))
PY
  tail -1 $OUT/kv_${TAG}_$V.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('           value', d['value'], 'it/s', d['ms_per_step'], 'ms/step')" || true
done
