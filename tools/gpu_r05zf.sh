# step launches: the groups' Dict records (MPGPU_HA_DREC) -- tests, then A/B
set -o pipefail
O=gpurun_out/r05zf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_DREC=1" "MPGPU_HA_DREC=0" "MPGPU_HA_DREC=1" "MPGPU_HA_DREC=0"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
