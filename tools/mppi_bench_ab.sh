#!/bin/bash
# Headline-only bench A/B (bench.py --no-extras --no-cpu --no-single) alternating libmpgpu variants.
# usage: bash tools/mppi_bench_ab.sh TAG STEPS lib-suffix...   ("" = libmpgpu.so)
set -o pipefail
TAG=$1; STEPS=$2; shift 2
D=gpurun_out/$TAG; mkdir -p $D
for v in "$@"; do
  n=${v:-default}
  MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so timeout -k 10 120 python3 bench.py --steps $STEPS --warmup 10 --no-cpu --no-extras --no-single > $D/b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('$D/b.log').read().strip().splitlines()[-1]); print('%-10s value %.4g ms/step %.4f kernel %.4f' % ('$n', d['value'], d['ms_per_step'], d['roofline']['kernel_ms']))" >> $D/ab.log
done
cat $D/ab.log
