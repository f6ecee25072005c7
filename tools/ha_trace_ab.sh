#!/bin/bash
# Kernel traces of the configs[3] plan (tools/ha_plan_time.py) per libmpgpu variant, with the
# per-iteration split of the last plan (tools/ha_iters.py).
# usage: bash tools/ha_trace_ab.sh TAG lib-suffix...   ("" = libmpgpu.so)
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
export TMPDIR=/tmp
for v in "$@"; do
  n=${v:-default}
  MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d $D/tr_$n -o run --output-format csv -- python3 tools/ha_plan_time.py > $D/tr_$n.log 2>&1 || exit 1
  echo "== lib$v" >> $D/iters.log
  python3 tools/ha_iters.py $D/tr_$n/run_kernel_trace.csv >> $D/iters.log || exit 1
done
cat $D/iters.log
