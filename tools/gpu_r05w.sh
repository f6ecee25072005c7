# the 6-wave middle shape (ha_step_kernel<6,16>, MPGPU_HA_MID_BLOCKS): bit-exactness with it on, then timing
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
MPGPU_HA_MID_BLOCKS=1024 timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread -k "batch or driver" > $O/pytest_mid.log 2>&1; rc=$?; tail -3 $O/pytest_mid.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_MID_BLOCKS=0" "MPGPU_HA_MID_BLOCKS=512" "MPGPU_HA_MID_BLOCKS=768" "MPGPU_HA_MID_BLOCKS=1024" "MPGPU_HA_MID_BLOCKS=1536" "MPGPU_HA_MID_BLOCKS=0" "MPGPU_HA_MID_BLOCKS=768" "MPGPU_HA_MID_BLOCKS=1024"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
