#!/bin/bash
# Build the current library sources with extra compile flags into build/ab/libdcfm_NAME.so (A/B
# variants for tools/gpu_ab.sh).  Usage: bash tools/build_variant.sh NAME "-DFOO=1 ..."
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
mkdir -p $W/pkg $ROOT/build/ab
cp -r $ROOT/a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/csrc $W/pkg/csrc
cp -r $ROOT/include $W/include
rm -f $W/pkg/csrc/*.o
make -C $W/pkg/csrc -j8 OUT=$ROOT/build/ab/libdcfm_$NAME.so \
  CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function -I/opt/rocm/include -I$W/include $EXTRA" \
  > $W/build.log 2>&1 || { tail -20 $W/build.log; exit 1; }
rm -rf $W
ls -la $ROOT/build/ab/libdcfm_$NAME.so
