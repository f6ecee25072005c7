# the 6-wave middle shape at 3 waves per SIMD (139 VGPRs, no spills; still two blocks per CU) vs 4 (128 + spills)
set -o pipefail
O=gpurun_out/r05zp; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "" _mid4 "" _mid4; do
  echo "== libmpgpu$v"
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
