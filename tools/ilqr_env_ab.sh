#!/bin/bash
# iLQR A/B of env knobs / variant libraries: default vs each "NAME=VALUE ..." argument, alternating
# fresh processes of tools/ilqr_time.py; prints the backward-pass kernel ms and the solve ms per run.
# usage: bash tools/ilqr_env_ab.sh OUTTAG MPGPU_ILQR_FUSED=0 "MPGPU_LIB=$PWD/variant.so" [...]
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
show() { echo "$1 backward $(grep -o 'backward: .* ms kernel' $2 | awk '{print $5}') solve $(grep -o 'solve: [0-9.]* ms' $2 | awk '{print $2}')"; }
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/ilqr_time.py > $O/base_$r.log 2>&1 || exit $?
  show base $O/base_$r.log
  i=0
  for kv in "$@"; do
    i=$((i + 1))
    env $kv timeout -k 10 120 python3 tools/ilqr_time.py > $O/v${i}_$r.log 2>&1 || exit $?
    show "$(echo $kv | sed -E 's#=/[^ ]*/#=#g')" $O/v${i}_$r.log
  done
done
