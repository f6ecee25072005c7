# the node hand-off: tagged granules (MPGPU_HA_NGR=1) vs node buffers + drained flag (0), same box
set -o pipefail
O=gpurun_out/r05zl; mkdir -p $O
export TMPDIR=/tmp
MPGPU_HA_NGR=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest0.log 2>&1; rc=$?; tail -2 $O/pytest0.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_NGR=1" "MPGPU_HA_NGR=0" "MPGPU_HA_NGR=1" "MPGPU_HA_NGR=0"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && grep -v amdgpu.ids $O/lone.log || exit 1
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha.log 2>&1 && grep "plan 256" $O/ha.log | tail -2 || exit 1
done
