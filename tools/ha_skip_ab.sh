#!/bin/bash
# Hybrid A* A/B: the Dict pre-check that lets neighbour groups skip rs_heuristic (default) vs every group
# evaluating it (MPGPU_HA_NOSKIP=1), alternating fresh processes of tools/ha_plan_time.py.
set -o pipefail
O=gpurun_out/${1:-ha_skip_ab}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python3 tools/ha_plan_time.py > $O/skip_$r.log 2>&1 || exit $?
  MPGPU_HA_NOSKIP=1 timeout -k 10 120 python3 tools/ha_plan_time.py > $O/noskip_$r.log 2>&1 || exit $?
done
for f in $O/*.log; do echo "== $f"; cat $f; done
