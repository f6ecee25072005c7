# the full-width / middle groups' sweep probing each neighbour's last pose first (HA_SWEEP_PROBE) vs not
set -o pipefail
O=gpurun_out/r05zt; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/motionplanning_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "" _noprobe "" _noprobe; do
  echo "== libmpgpu$v"
  MPGPU_LIB=$L/libmpgpu$v.so timeout -k 10 200 python3 tools/ha_plan_time.py --shards > $O/ha.log 2>&1 && grep -v "scenes still" $O/ha.log | tail -4 || exit 1
done
