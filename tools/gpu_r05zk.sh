# the node hand-off as tagged granules (ha_publish_node / ha_consume_node): HA GPU tests (both persistent block
# sizes, and the non-persistent pipe), then lone / plan / shards timing
set -o pipefail
O=gpurun_out/r05zk; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
MPGPU_HA_PERSIST=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pipe.log 2>&1; rc=$?; tail -2 $O/pytest_pipe.log; [ $rc -ne 0 ] && exit $rc
MPGPU_HA_PERSIST_HW=12 timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest_12.log 2>&1; rc=$?; tail -2 $O/pytest_12.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && grep -v amdgpu.ids $O/lone.log || exit 1
  timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -3 || exit 1
done
