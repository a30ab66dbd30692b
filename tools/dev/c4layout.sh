# c4: the default side-stream layout vs every launch on one stream (DCFM_FLAG_ONE_STREAM) vs flat priorities
set -e
mkdir -p gpurun_out
C4="--g 8 --P 1250 --n 2000 --K 100 --steps 100 --warmup 10 --no-cpu-baseline --converged-mcmc 0"
for r in 1 2; do
  for F in 0 0x4 0x8; do
    timeout -k 10 300 python3 -u bench.py $C4 --layout-flags $F > gpurun_out/b_c4l_${F}_$r.json 2> gpurun_out/b_c4l.err
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'])" gpurun_out/b_c4l_${F}_$r.json $F
  done
done
