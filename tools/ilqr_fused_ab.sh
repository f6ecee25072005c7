#!/bin/bash
# iLQR A/B of the backward pass: fused above kDeriv4Max active instances (default, MPGPU_ILQR_FUSED=1),
# always fused (=2), never (=0, the two-kernel path); alternating fresh processes of tools/ilqr_time.py.
set -o pipefail
O=gpurun_out/${1:-ilqr_fused_ab}
mkdir -p $O
for r in 1 2 3; do
  for m in 1 2 0; do
    MPGPU_ILQR_FUSED=$m timeout -k 10 120 python3 tools/ilqr_time.py > $O/mode${m}_$r.log 2>&1 || exit $?
  done
done
for f in $O/*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
