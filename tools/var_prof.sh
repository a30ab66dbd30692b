#!/bin/bash
# Serialized kernel trace of a c3 bench per library variant (dev aid).
# Usage (on the GPU box): bash tools/var_prof.sh name1 name2 ...   (build/libdcfm_<name>.so; "main" = in-tree)
cd /tmp && export TMPDIR=/tmp && export DCFM_SERIALIZE=1
for v in "$@"; do
  if [ "$v" = main ]; then unset DCFM_LIB; else export DCFM_LIB=$GRAFT_REPO_ROOT/build/libdcfm_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/vp_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-profile --steps 40 --warmup 5 --thin 1000 > /dev/null 2>&1 || exit 1
done
