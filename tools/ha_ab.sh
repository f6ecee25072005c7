#!/bin/bash
# A/B of Hybrid A* builds: configs[3] plan time (tools/ha_plan_time.py) per libmpgpu variant.
# usage: bash tools/ha_ab.sh TAG lib-suffix...   ("" = libmpgpu.so)
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
for v in "$@"; do
  echo "== lib$v" >> $D/ha.log
  MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so timeout -k 10 120 python3 tools/ha_plan_time.py >> $D/ha.log 2>&1 || exit 1
done
cat $D/ha.log
