#!/bin/bash
# Round profile collection on the GPU box (run from the repo root through gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench (graph-replayed steps + the serial
#      per-op profile pass bench.py uses for its roofline) -> gpurun_out/prof_$R/
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE: they cannot share a pass) of a short bench
# then summarise into profiles/ with kernel_trace_summary.py / pmc_traffic.py (on the CPU side).
set -e
R=${1:-r2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --breakdown gpurun_out/breakdown_$R.json \
  > gpurun_out/bench_prof_$R.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$R -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmcf_$R.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$R -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmcw_$R.log 2>&1
