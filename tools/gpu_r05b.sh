set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_distributed.py tests/test_gpu_track.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -3 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha_new.log 2>&1 && cat $O/ha_new.log &&
MPGPU_HA_RS_FULL=1 timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha_full.log 2>&1 && cat $O/ha_full.log
