#!/bin/bash
# Build the loading-row dev harness against the in-tree libdcfm.so (run from the repo root).
set -e
PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I $PKG/csrc -I tools/lambench \
  tools/lambench/lambench.hip -L $PKG -ldcfm -Wl,-rpath,'$ORIGIN/../../'$PKG -o tools/lambench/lambench "$@"
