# ha_persist_kernel (cooperative persistent tail): bit-exactness (HA, fuzz, track, distributed GPU tests) and
# timing against MPGPU_HA_PERSIST=0 (one ha_pipe_kernel launch per iteration)
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
export TMPDIR=/tmp
MPGPU_HA_VERBOSE=1 timeout -k 10 120 python3 tools/ha_lone.py 1 > $O/lone0.log 2>&1; rc=$?; tail -5 $O/lone0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_PERSIST=1" "MPGPU_HA_PERSIST=0" "MPGPU_HA_PERSIST=1" "MPGPU_HA_PERSIST=0"; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha.log 2>&1 && tail -2 $O/ha.log || exit 1
  env $env timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && tail -3 $O/lone.log || exit 1
done
