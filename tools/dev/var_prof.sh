#!/bin/bash
# Serialized kernel trace of a bench run per library variant (dev aid).
# Usage (on the GPU box): BENCH_ARGS="--g 8 ..." bash tools/var_prof.sh v1 v2:ENV=VAL ...
#   v = build/libdcfm_<v>.so, "main" = in-tree; ":ENV=VAL" adds one environment setting
cd /tmp && export TMPDIR=/tmp && export DCFM_SERIALIZE=1
ARGS=${BENCH_ARGS:---steps 40 --warmup 5 --thin 1000}
for spec in "$@"; do
  v=${spec%%:*}; extra=""; [ "$spec" != "$v" ] && extra=${spec#*:}
  tag=$(echo "$spec" | tr ':=' '__')
  if [ "$v" = main ]; then unset DCFM_LIB; else export DCFM_LIB=$GRAFT_REPO_ROOT/build/libdcfm_$v.so; fi
  env $extra timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/vp_$tag -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-profile $ARGS > /dev/null 2>&1 || exit 1
done
