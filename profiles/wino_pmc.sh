#!/bin/bash
# SQ / TA counters of the Winograd variants on one shape (profiles/bench_wino.py), one rocprofv3
# --pmc pass per variant: bash profiles/wino_pmc.sh "0 3 5" [SHAPES]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export NOMIO=1 SHAPES=${2:-64,128,128,120,120} KRRN_WINO_PIPE=1
for v in $1; do
  KRRN_WINO_V=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE TA_TA_BUSY_sum \
    -d $R/gpurun_out/wpmc_v$v -o pmc --output-format csv -- python3 $R/profiles/bench_wino.py
done
