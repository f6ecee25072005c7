#!/bin/bash
# Hybrid A* A/B of env knobs: default vs each "NAME=VALUE" argument, alternating fresh processes of
# tools/ha_plan_time.py; prints the library-call ms of plans 3-5 per run.
# usage: bash tools/ha_env_ab.sh OUTTAG MPGPU_HA_TAIL_BLOCKS=256 "MPGPU_LIB=$PWD/variant.so" [...]
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python3 tools/ha_plan_time.py > $O/base_$r.log 2>&1 || exit $?
  echo "base $(tail -3 $O/base_$r.log | sed -E 's/.*library call ([0-9.]+) ms.*/\1/' | tr '\n' ' ')"
  i=0
  for kv in "$@"; do
    i=$((i + 1))
    env $kv timeout -k 10 120 python3 tools/ha_plan_time.py > $O/v${i}_$r.log 2>&1 || exit $?
    echo "$(echo $kv | sed -E 's#=/[^ ]*/#=#g') $(tail -3 $O/v${i}_$r.log | sed -E 's/.*library call ([0-9.]+) ms.*/\1/' | tr '\n' ' ')"
  done
done
