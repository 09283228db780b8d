#!/bin/bash
# SQ / TA counters of the f32 and split-bf16 Winograd kernels (profiles/bench_wino_x3.py; both
# kernels in one run, rocprofv3 reports per dispatch), three --pmc passes per split-kernel variant:
#   bash profiles/wino_x3_pmc.sh "1 0" [SHAPES]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export SHAPES=${2:-64,128,128,120,120} NOREF=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM TA_BUSY_avr"
P3="SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_DATA_FIFO_FULL"
for v in $1; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    KRRN_WINO_X3V=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $R/gpurun_out/wx3pmc_v${v}_$i -o pmc --output-format csv \
      -- python3 $R/profiles/bench_wino_x3.py
  done
done
