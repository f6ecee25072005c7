set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -3 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && cat $O/lone.log &&
MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu_noovl.so timeout -k 10 200 python3 tools/ha_lone.py > $O/lone_noovl.log 2>&1 && cat $O/lone_noovl.log &&
timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && cat $O/ha.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_hastar.py -x -v --timeout 120 --timeout-method thread -k translated > $O/pytest_translated.log 2>&1; rc=$?; tail -3 $O/pytest_translated.log; exit $rc
