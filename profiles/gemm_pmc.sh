#!/bin/bash
# SQ counters of krrn_gemm_x3_f32 (profiles/bench_gemm_x3.py), one rocprofv3 --pmc pass per set
# usage: bash profiles/gemm_pmc.sh out_dir [M K N]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS \
  SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $R/gpurun_out/$1/a -o pmc --output-format csv \
  -- python3 $R/profiles/bench_gemm_x3.py $2 $3 $4
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY \
  SQ_INSTS_VALU GRBM_COUNT -d $R/gpurun_out/$1/b -o pmc --output-format csv \
  -- python3 $R/profiles/bench_gemm_x3.py $2 $3 $4
