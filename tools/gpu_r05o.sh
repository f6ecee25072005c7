set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ha.log 2>&1; rc=$?; tail -2 $O/pytest_ha.log; [ $rc -ne 0 ] && exit $rc
MPGPU_HA_RS_LAST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_hastar.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ha2.log 2>&1; rc=$?; tail -2 $O/pytest_ha2.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_HA_RS_LAST=0" "MPGPU_HA_RS_LAST=1" "MPGPU_HA_RS_LAST=0" "MPGPU_HA_RS_LAST=1"; do
  echo "== $env"; env $env timeout -k 10 200 python3 tools/ha_plan_time.py > $O/ha.log 2>&1 && tail -2 $O/ha.log || exit 1
done
