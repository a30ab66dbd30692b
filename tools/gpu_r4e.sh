#!/bin/bash
# round 4: GPU tests on the in-tree build; exact-residual bench; A/B of build variants (args)
TAG=${1:-r4e}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
B="python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0"
timeout -k 10 200 $B --exact-residual > gpurun_out/b_${TAG}_ex.json 2> gpurun_out/b_${TAG}_ex.err || { echo "bench ex failed"; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('exact', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})" gpurun_out/b_${TAG}_ex.json
[ $# -gt 0 ] && bash tools/gpu_ab.sh $TAG 3 "$@"
echo all done
