#!/bin/bash
# dev: bench line + per-kernel trace stats for one bench configuration (run on the GPU box).
# Usage: bash tools/ktrace.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/ks_${TAG}.log 2>&1 || { echo "trace failed"; tail $OUT/ks_${TAG}.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - $OUT/ks_${TAG} <<'PY'
import csv, glob, sys, re
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:16]:
        n = re.search(r"(k_\w+|\w+Kernel\w*)", r["Name"])
        print(f"  {n.group(1) if n else r['Name'][:40]:28s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs'])/1000:8.1f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
grep -h '"metric"' $OUT/ks_${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('  bench', d['value'], d['unit'], 'ms/step', d['ms_per_step'])"
