#!/bin/bash
# round-4 GPU pass: Winograd variants (tests + timing), panel GEMM tests, bench A/B, write audit,
# F0 shadow diagnostic, Winograd PMC. Stops at the first step that faults / aborts / times out.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step NAME CMD...: run, report, stop the script on a fault, abort or time limit
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc $rc"
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
  return 0
}
step wino_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -k "winograd or wino_up2 or kchunk or convT or group" --timeout 120 --timeout-method thread -o log_cli=false > gpurun_out/r4_wtest.log 2>&1
tail -2 gpurun_out/r4_wtest.log
for v in 0 1; do step wbench_$v env KRRN_WINO_X3W=$v timeout -k 10 120 python -u profiles/bench_wino_x3.py > gpurun_out/r4_wbench_$v.log 2>&1; done
step gemm_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gemmtest.log 2>&1
tail -2 gpurun_out/r4_gemmtest.log
for v in "0 0 0" "1 0 0" "1 1 0" "1 1 16"; do
  set -- $v
  step bench_x3w_$1_up2_$2_kc$3 env KRRN_WINO_X3W=$1 KRRN_UP2_FUSE=$2 KRRN_CONVT_KCHUNK=$3 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --breakdown gpurun_out/r4_bd_$1$2_$3.json > gpurun_out/r4_bench_$1$2_$3.log 2>&1
  tail -1 gpurun_out/r4_bench_$1$2_$3.log | cut -c1-220
done
step eval_epoch timeout -k 10 400 python3 -u profiles/eval_epoch.py --out gpurun_out/r4_eval_epoch.json > gpurun_out/r4_eval.log 2>&1
tail -1 gpurun_out/r4_eval.log | cut -c1-300
step audit timeout -k 10 400 python -u -m pytest tests/test_gpu_write_audit.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r4_audit.log 2>&1
step shadow timeout -k 10 300 python -u profiles/f0_shadow.py 5 --history > gpurun_out/r4_shadow.log 2>&1
step pmc timeout -k 10 200 bash profiles/r4_wino_pmc.sh base > gpurun_out/r4_wpmc.log 2>&1
