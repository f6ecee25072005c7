#!/bin/bash
# Hybrid A* A/B: the fused ha_step_kernel (default) vs the split iter + book launches (MPGPU_HA_SPLIT=1),
# alternating, each a fresh process of tools/ha_plan_time.py (256 scenarios, 5 plans).
set -o pipefail
O=gpurun_out/${1:-ha_fuse_ab}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python3 tools/ha_plan_time.py > $O/fused_$r.log 2>&1 || exit $?
  MPGPU_HA_SPLIT=1 timeout -k 10 120 python3 tools/ha_plan_time.py > $O/split_$r.log 2>&1 || exit $?
done
for f in $O/*.log; do echo "== $f"; cat $f; done
