#!/bin/bash
# A/B of the runtime's tuning knobs on the default bench step (GPU box), one process per setting,
# ms_per_step only (no profile / CPU leg). usage: bash profiles/knob_sweep.sh [tag]
T=${1:-sweep}
mkdir -p gpurun_out
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu --no-profile > gpurun_out/${T}_$name.log 2>&1 || { echo "FAIL $name"; return 0; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_$name.log').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d['value'])"
}
run base KRRN_X=0
run hr_group KRRN_HR_GROUP=1
run pose_heads KRRN_POSE_AT=heads
run pose_level2 KRRN_POSE_AT=level2
run tbase_late KRRN_TBASE_EARLY=0
run no_plan_streams KRRN_PLAN_STREAMS=0
run splitk0 KRRN_SPLITK=0
run base2 KRRN_X=0
