#!/bin/bash
# SQ / TA counters of the split-bf16 Winograd kernel on the step's 120-px shape (B = 64,
# 128 -> 128), one rocprofv3 --pmc pass per counter set (a pass holds at most 8 SQ_ counters):
#   bash profiles/r4_wino_pmc.sh [TAG]      (GPU box, repo root)
# then: python profiles/pmc_kernel_summary.py gpurun_out/wpmc_TAG_*/pmc_counter_collection.csv
set -e
TAG=${1:-r4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
export SHAPES=${SHAPES:-64,128,128,120,120} NOREF=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM TA_BUSY_avr"
P3="SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_DATA_FIFO_FULL"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/wpmc_${TAG}_$i -o pmc --output-format csv \
    -- python3 $R/profiles/bench_wino_x3.py
done
