set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -3 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rest.log 2>&1; rc=$?; tail -2 $O/pytest_rest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_PIPE=0" ""; do
  echo "== $env"
  env $env timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && cat $O/lone.log | grep -v amdgpu.ids || exit 1
  env $env timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && tail -4 $O/ha.log || exit 1
done
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st.log 2>&1 &&
python3 tools/ha_stamps_blocks.py $O/st.bin 5 > $O/st.txt
