# primitive-table memo (mp_ha_neighbor_origin): HA GPU tests, then the plan's wall vs library time
set -o pipefail
O=gpurun_out/r05za; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha.log 2>&1 && cat $O/ha.log
