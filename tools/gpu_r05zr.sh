# persistent tail: issue priority by role (book 2, groups 1, RS 0) vs none -- tests, then lone / plan / shards
set -o pipefail
O=gpurun_out/r05zr; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "" _noprio "" _noprio; do
  echo "== libmpgpu$v"
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_lone.py > $O/lone.log 2>&1 && grep -v amdgpu.ids $O/lone.log || exit 1
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -3 || exit 1
done
