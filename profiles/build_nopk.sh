#!/bin/bash
# build/variants/nopk.so = libkrrn_hip.so with every source compiled without packed-FP32 VALU ops
# (v_pk_mul/fma/add_f32): the A/B for DESIGN.md section 5's cross-kernel mismatch
set -e
cd "$(dirname "$0")/../pose_estimation_amd/csrc"
out=../../build/variants/nopk
mkdir -p $out
for f in *.hip; do
  b=${f%.hip}; extra=""
  [ $b = pnp ] && extra="-ffp-contract=off"
  [ $b = winograd ] && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast-honor-pragmas $extra \
    -Xclang -target-feature -Xclang -packed-fp32-ops -c $f -o $out/$b.o 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../build/variants/nopk.so $out/*.o -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
echo built build/variants/nopk.so
