#!/bin/bash
# round 4: GPU tests on the in-tree build; driver bench default / exact / asm_tail off / asm-batch 1, 2;
# then the A/B of build variants (args)
TAG=${1:-r4c}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
B="python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0"
for V in "def:" "ex:--exact-residual" "notail:--asm-tail -1" "ab1:--asm-batch 1" "ab2:--asm-batch 2" "def2:"; do
  N=${V%%:*}; A=${V#*:}
  timeout -k 10 200 $B $A > gpurun_out/b_${TAG}_$N.json 2> gpurun_out/b_${TAG}_$N.err || { echo "bench $N failed"; tail -5 gpurun_out/b_${TAG}_$N.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})" gpurun_out/b_${TAG}_$N.json $N
done
[ $# -gt 0 ] && bash tools/gpu_ab.sh $TAG 2 "$@"
echo all done
bash tools/diag_l2.sh r4c
