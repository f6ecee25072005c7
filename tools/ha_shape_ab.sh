#!/bin/bash
# Hybrid A* launch-shape A/B: tail threshold and the middle shape (env overrides of mp_ha_plan).
set -o pipefail
O=gpurun_out/${1:-ha_shape_ab}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python3 tools/ha_plan_time.py > $O/$n.log 2>&1 || exit $?
  echo "$n $(tail -3 $O/$n.log | sed -E 's/.*library call ([0-9.]+) ms.*/\1/' | tr '\n' ' ')"
}
run base MPGPU_HA_MID_BLOCKS=0
run mid640 MPGPU_HA_MID_BLOCKS=640
run mid1280 MPGPU_HA_MID_BLOCKS=1280
run tail544 MPGPU_HA_TAIL_BLOCKS=544
run base2 MPGPU_HA_MID_BLOCKS=0
run mid320 MPGPU_HA_MID_BLOCKS=320
