#!/bin/bash
# SQ counters of the fused BasicBlock kernel vs conv_small (profiles/bench_bb.py, branch-0 shape, T=4)
# usage: bash profiles/bb_pmc.sh out_tag
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export SHAPES_IDX=${SHAPES_IDX:-0} TS=${TS:-4}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU -d $R/gpurun_out/$1_a -o pmc --output-format csv \
  -- python3 $R/profiles/bench_bb.py > $R/gpurun_out/$1_a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM \
  SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/$1_b -o pmc --output-format csv \
  -- python3 $R/profiles/bench_bb.py > $R/gpurun_out/$1_b.log 2>&1
