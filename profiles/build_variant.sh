#!/bin/bash
# build/variants/<name>.so (VDIR=... elsewhere; build/variants is not pushed to gpurun boxes) = libkrrn_hip.so with one source replaced: <file>.hip recompiled under extra
# flags, or (with SRC=path) another version of that file, e.g. the committed one for an A/B:
#   git show HEAD:pose_estimation_amd/csrc/winograd.hip > /tmp/w_old.hip
#   SRC=/tmp/w_old.hip profiles/build_variant.sh wino_old winograd ""
# usage: profiles/build_variant.sh name file "flags"
set -e
cd "$(dirname "$0")/../pose_estimation_amd/csrc"
make -s
VDIR=${VDIR:-../../build/variants}
mkdir -p $VDIR
objs=$(ls ../../build/csrc/*.o | grep -v "/$2.o")
src=${SRC:-$2.hip}
# the Makefile's flags (no packed FP32; per-file extras)
extra=""
[ "$2" = winograd ] && extra="-fno-slp-vectorize"
[ "$2" = winograd4 ] && extra="-fno-slp-vectorize"
[ "$2" = pnp ] && extra="-ffp-contract=off"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast-honor-pragmas \
  -Xclang -target-feature -Xclang -packed-fp32-ops -I. $extra $3 -c $src -o $VDIR/$1_$2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $VDIR/$1.so $objs $VDIR/$1_$2.o -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
echo built $VDIR/$1.so
