#!/bin/bash
# What-if timing (GPU box): the default bench step with whole kernel families left out of the
# plans (runtime KRRN_DIAG_DROP; results are meaningless, only ms_per_step is read). Shows how
# much of each family's serial time is on the step's critical path under graph concurrency.
#   bash profiles/whatif.sh [tag]
T=${1:-r3}
mkdir -p gpurun_out
run() {
  local name=$1; shift
  KRRN_DIAG_DROP=$1 timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-profile \
    > gpurun_out/whatif_${T}_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/whatif_${T}_$name.log; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/whatif_${T}_$name.log').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'])"
}
run base "" &&
run no_small krrn_conv_small_f32 &&
run no_wino krrn_conv3x3_wino_x3_f32 &&
run no_gcn krrn_gcn_conv_f32 &&
run no_gemm krrn_gemm_x3_f32,krrn_gemm_panel_x3_f32,krrn_blas_gemm_run &&
run no_pnp krrn_pnp_ransac_f32 &&
run no_group krrn_conv2d_group_x3_f32,krrn_conv2d_x3_f32,krrn_conv2d_f32 &&
run no_resize krrn_resize_bilinear_f32 &&
run no_nchw krrn_conv1x1_nchw_f32
