for v in NOUPDATE NOFACTOR; do
DCFM_LIB=build/libdcfm_$v.so timeout -k 10 200 python -u bench.py --g 8 --P 1250 --n 2000 --K 100 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4_$v.json 2>/dev/null || exit 1
done
