# the persistent tail on 4-wave blocks (three per CU, up to 42 scenes) vs 6 -- tests, A/B
set -o pipefail
O=gpurun_out/r05zh; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
MPGPU_HA_PERSIST_HW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest6.log 2>&1; rc=$?; tail -3 $O/pytest6.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_PERSIST_HW=6" "MPGPU_HA_PERSIST_HW=4" "MPGPU_HA_PERSIST_HW=6" "MPGPU_HA_PERSIST_HW=4"; do
  echo "== $env"
  env $env MPGPU_HA_VERBOSE=1 timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && grep -v amdgpu.ids $O/lone.log | sort -u | tail -3 || exit 1
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -3 || exit 1
done
