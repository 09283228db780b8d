#!/bin/bash
# PnP timing variants (CPU build, GPU run with profiles/bench_pnp.py and KRRN_HIP_LIB): the library
# with pnp.hip recompiled from a macro-instrumented copy ($1) under each -D set below.
set -e
SRC=$1
cd "$(dirname "$0")/.."
make -s -C pose_estimation_amd/csrc
mkdir -p build/variants
objs=$(ls build/csrc/*.o | grep -v "/pnp.o")
build() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Xclang -target-feature -Xclang -packed-fp32-ops \
    -Ipose_estimation_amd/csrc $2 -c $SRC -o build/variants/pnp_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/pnp_$1.so $objs build/variants/pnp_$1.o -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
}
build base "" &
build w2 "-DPNP_WAVES=2" &
build noeig12 "-DPNP_NOEIG12" &
build a1 "-DPNP_APPROX_MAX=1" &
wait
build nogn "-DPNP_NOGN" &
build a1nogn "-DPNP_APPROX_MAX=1 -DPNP_NOGN" &
build a1nognnoeig "-DPNP_APPROX_MAX=1 -DPNP_NOGN -DPNP_NOEIG12" &
wait
ls build/variants/pnp_*.so
