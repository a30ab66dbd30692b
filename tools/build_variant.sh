#!/bin/bash
# Build a development variant of libdcfm into build/libdcfm_<NAME>.so with extra
# compiler flags, e.g.  bash tools/build_variant.sh phase -DDCFM_PHASE_TIMING
set -e
NAME=$1; shift
SRC=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/csrc
OBJ=build/obj_$NAME
mkdir -p $OBJ
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I/opt/rocm/include -Iinclude $*"
for f in kernels kernels_wide sigma_err ingest trace init dcfm; do
  hipcc $FLAGS -c $SRC/$f.hip -o $OBJ/$f.o &
done
wait
hipcc $FLAGS $OBJ/*.o -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o build/libdcfm_$NAME.so
echo build/libdcfm_$NAME.so
