#!/bin/bash
# Round evidence on the box for the current build: GPU tests, smoke, the driver's bench + its
# rocprofv3 trace and PMC passes (gpu_full.sh), then the c4 shape (bench + trace + PMC) and the
# g = 8 share bench.  Stops at the first failing step.  Usage: bash tools/gpu_evidence.sh TAG
TAG=$1
bash tools/gpu_full.sh $TAG || exit 1
C4="--g 8 --P 1250 --n 2000 --K 100 --steps 100 --warmup 10"
C5="--g 256 --P 391 --n 2000 --K 30 --steps 30 --warmup 5"
timeout -k 10 300 python3 -u bench.py $C4 > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err || { echo "c4 bench failed"; exit 1; }
bash tools/profile_round.sh ${TAG}_c4 $C4 || exit 1
timeout -k 10 300 python3 -u bench.py --g 8 --thin 100000 --steps 2000 --warmup 100 --no-cpu-baseline --no-profile --converged-mcmc 0 > gpurun_out/bench_${TAG}_g8.json 2> gpurun_out/bench_${TAG}_g8.err || { echo "g8 bench failed"; exit 1; }
timeout -k 10 400 python3 -u bench.py $C5 --no-cpu-baseline --converged-mcmc 0 > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo "c5 bench failed"; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_${TAG}.json gpurun_out/bench_${TAG}_c4.json gpurun_out/bench_${TAG}_g8.json gpurun_out/bench_${TAG}_c5.json
