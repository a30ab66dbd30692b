#!/bin/bash
# rocprofv3 kernel trace of the c4-shape bench (dev aid): per-kernel average durations
TAG=${1:-c4}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-profile --g 8 --P 1250 --n 2000 --K 100 --steps 30 --warmup 5 > $OUT/kt_${TAG}.log 2>&1 || { echo "trace failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - "$OUT/kt_${TAG}" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    nm = row['Name'].split('(')[0].replace('void ', '')
    print(f"{nm[:44]:44s} calls={row['Calls']:>4s} avg_us={float(row['AverageNs'])/1000:9.2f}")
PY
