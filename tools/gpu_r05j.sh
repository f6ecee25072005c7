set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result tools/ubench/task_counter.hip -o $O/task_counter && timeout -k 10 120 $O/task_counter > $O/task_counter.txt 2>&1; rc=$?; cat $O/task_counter.txt; [ $rc -ne 0 ] && exit $rc
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st.log 2>&1 &&
python3 tools/ha_stamps_blocks.py $O/st.bin 6 > $O/st.txt &&
MPGPU_LIB=$L/libmpgpu_stamp.so MPGPU_HA_PRESCAN=0 MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=$O/st0.bin timeout -k 10 200 python3 tools/ha_lone.py 1 --lone-only > $O/st0.log 2>&1 &&
python3 tools/ha_stamps_blocks.py $O/st0.bin 6 > $O/st0.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -2 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
for v in "" _wpe3; do
  for env in "MPGPU_HA_PRESCAN=0" ""; do
    echo "== lib$v $env"
    env $env MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && cat $O/lone.log | grep -v amdgpu.ids || exit 1
    env $env MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha.log 2>&1 && tail -2 $O/ha.log || exit 1
  done
done
