#!/bin/bash
# Development A/B builds (never shipped): copy csrc to build/src_NAME, apply a Python patch
# script to the copy (it receives the directory as argv[1]), build build/libdcfm_NAME.so.
# Run a bench against it with DCFM_LIB=build/libdcfm_NAME.so.
# Usage: bash tools/variant.sh NAME PATCH.py (a dev patch script kept outside the tree)
set -e
NAME=$1; PATCH=$2
SRC=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/csrc
DST=build/src_$NAME
rm -rf $DST; mkdir -p $DST; cp $SRC/*.hip $SRC/*.h $SRC/Makefile $DST/
[ -n "$PATCH" ] && python3 $PATCH $DST
make -C $DST -j8 OUT=$PWD/build/libdcfm_$NAME.so > /dev/null
echo build/libdcfm_$NAME.so
