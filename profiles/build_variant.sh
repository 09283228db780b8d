#!/bin/bash
# build/variants/<name>.so = libkrrn_hip.so with <file>.hip recompiled under extra flags
# usage: profiles/build_variant.sh name file "flags"
set -e
cd "$(dirname "$0")/../pose_estimation_amd/csrc"
make -s
mkdir -p ../../build/variants
objs=$(ls ../../build/csrc/*.o | grep -v "/$2.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast-honor-pragmas $3 -c $2.hip -o ../../build/variants/$1_$2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build/variants/$1.so $objs ../../build/variants/$1_$2.o -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
echo built build/variants/$1.so
