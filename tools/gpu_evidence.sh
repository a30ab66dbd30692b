#!/bin/bash
# Round evidence on the box for the current build: every GPU test + smoke, then per workload the
# rocprofv3 kernel trace + PMC passes FIRST (tools/profile_round.sh; the summary is copied into
# the box's profiles/ so the bench line that follows takes roofline.traffic from it), then the
# bench line.  Workloads: the driver's c3 command, c4, the g = 8 share (bench only), c5.
# Stops at the first failing step.  Usage: bash tools/gpu_evidence.sh TAG c3|rest
# (c3: GPU tests, smoke, the driver's c3 command; rest: c4, the g = 8 share, c5)
TAG=$1; PHASE=${2:-c3}
mkdir -p gpurun_out
if [ "$PHASE" = "c3" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread --junitxml=gpurun_out/t_$TAG.xml > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
  grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
fi
C3="--gpus 1 --steps 20 --warmup 5"
C4="--g 8 --P 1250 --n 2000 --K 100 --steps 100 --warmup 10"
C5="--g 256 --P 391 --n 2000 --K 30 --steps 30 --warmup 5"
run() {   # name, bench args, extra bench args (not part of the profiled command)
  local N=$1 A=$2 X=$3
  bash tools/profile_round.sh $N $A || exit 1
  cp gpurun_out/prof_${N}_pmc.json profiles/${N}_pmc.json
  timeout -k 10 400 python3 -u bench.py $A $X > gpurun_out/bench_$N.json 2> gpurun_out/bench_$N.err || { echo "bench $N failed"; tail gpurun_out/bench_$N.err; exit 1; }
}
if [ "$PHASE" = "c3" ]; then
  run ${TAG} "$C3"
  python3 tools/show_bench.py gpurun_out/bench_${TAG}.json
  run ${TAG}_exact "$C3 --exact-residual" "--no-cpu-baseline --converged-mcmc 0"
  python3 tools/show_bench.py gpurun_out/bench_${TAG}_exact.json
  exit 0
fi
run ${TAG}_c4 "$C4" "--no-cpu-baseline"
timeout -k 10 300 python3 -u bench.py --g 8 --thin 100000 --steps 2000 --warmup 100 --no-cpu-baseline --no-profile --converged-mcmc 0 > gpurun_out/bench_${TAG}_g8.json 2> gpurun_out/bench_${TAG}_g8.err || { echo "g8 bench failed"; exit 1; }
run ${TAG}_c5 "$C5" "--no-cpu-baseline --converged-mcmc 0"
python3 tools/show_bench.py gpurun_out/bench_${TAG}_c4.json gpurun_out/bench_${TAG}_g8.json gpurun_out/bench_${TAG}_c5.json
