# ha_persist_kernel: the bookkeeping's wait for the expansion after its open-list loads (HA_PREWAIT) -- tests, A/B
set -o pipefail
O=gpurun_out/r05ze; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py tests/test_gpu_track.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "" _nopre "" _nopre; do
  echo "== libmpgpu$v"
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && grep -v amdgpu.ids $O/lone.log || exit 1
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -3 || exit 1
done
