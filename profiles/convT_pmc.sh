#!/bin/bash
# Per-conv HBM traffic of krrn_convT_s2_x3_f32 (profiles/bench_convT.py, s2 only): FETCH_SIZE and
# WRITE_SIZE in separate passes for the deconv (CASE=0) and XYZNet's convT (CASE=1); summarise with
#   python profiles/pmc_traffic.py gpurun_out/ctpmc_f0/*/*counter_collection.csv gpurun_out/ctpmc_w0/...
set -e
export TMPDIR=/tmp TILES=
mkdir -p gpurun_out
for c in 0 1; do
  CASE=$c timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ctpmc_f$c -o run -- \
    python3 profiles/bench_convT.py > gpurun_out/ctpmc_f$c.log 2>&1
  CASE=$c timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ctpmc_w$c -o run -- \
    python3 profiles/bench_convT.py > gpurun_out/ctpmc_w$c.log 2>&1
done
CASE= timeout -k 10 120 python3 profiles/bench_convT.py > gpurun_out/ctpmc_time.log 2>&1
