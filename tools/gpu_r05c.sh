set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -3 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha_tab.log 2>&1 && cat $O/ha_tab.log &&
MPGPU_HA_NOTAB=1 timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha_notab.log 2>&1 && cat $O/ha_notab.log &&
timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && cat $O/lone.log &&
MPGPU_HA_RS_FULL=1 MPGPU_HA_NOTAB=1 timeout -k 10 200 python3 tools/ha_lone.py > $O/lone_old.log 2>&1 && cat $O/lone_old.log &&
MPGPU_HA_SPLIT=1 timeout -k 10 200 python3 tools/ha_lone.py > $O/lone_split.log 2>&1 && cat $O/lone_split.log &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_lone -o run --output-format csv -- python3 tools/ha_lone.py 3 --lone-only > $O/prof_lone.log 2>&1 &&
MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/lone_stamps.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/lone_stamp.log 2>&1 && python3 tools/ha_stamps.py $O/lone_stamps.bin > $O/lone_stamps.txt 2>&1; rc=$?
find $O -name 'run_kernel_trace.csv' | xargs -r gzip -f
exit $rc
