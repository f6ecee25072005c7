# near-threshold live-count polling (MPGPU_HA_NEAR_CH=4 vs 0): HA tests, then plan / shards timing
set -o pipefail
O=gpurun_out/r05zn; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_NEAR_CH=4" "MPGPU_HA_NEAR_CH=0" "MPGPU_HA_NEAR_CH=4" "MPGPU_HA_NEAR_CH=0" "MPGPU_HA_NEAR_CH=2"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha.log 2>&1 && grep "plan 256" $O/ha.log | tail -3 | awk '{print $7}' | tr '\n' ' ' && echo || exit 1
done
