#!/bin/bash
# L2 / memory-pipeline counters of the driver's bench command, one pass per counter group
# (within the per-block limits: <= 4 TCC, <= 4 TCP, <= 2 TA, <= 8 SQ).  Usage: bash tools/diag_l2.sh TAG
TAG=${1:-l2}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
BENCH="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --converged-mcmc 0 --no-profile --err-iters 0 --gpus 1 --steps 20 --warmup 5"
cd /tmp
i=0
for P in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr TA_BUSY_max" "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/diag_${TAG}_$i -o run -- $BENCH > $OUT/diag_${TAG}_$i.log 2>&1 || echo "pass $i ($P) failed: $(tail -2 $OUT/diag_${TAG}_$i.log)"
done
cd $GRAFT_REPO_ROOT
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/diag_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dcfm::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ("k_wcol", "k_cpass<32, false>", "k_cpass", "k_lambda<30>", "k_xdraw", "k_assemble"):
    if k in agg:
        print(k, {c: round(sum(v) / len(v)) for c, v in sorted(agg[k].items())})
PY
find gpurun_out -path "*diag_${TAG}*" -name "*.csv" -size +512k -exec gzip -9 {} \;
echo diag done
