#!/bin/bash
# SQ counters of the branch-conv kernels (profiles/bench_branch_conv.py), one rocprofv3 --pmc pass
# usage: bash profiles/branch_pmc.sh SHAPES_IDX TILES SPLITS SMALL_NW out_dir
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export NOMIO=1 SHAPES_IDX=$1 TILES=$2 SPLITS=$3 SMALL_NW=$4
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $R/gpurun_out/$5 -o pmc --output-format csv \
  -- python3 $R/profiles/bench_branch_conv.py
