# iLQR: the count mirror (MPGPU_ILQR_MIRROR=1) vs the stream copy + event poll; memset A/B beside; tests first
set -o pipefail
O=gpurun_out/r05zd; mkdir -p $O
export TMPDIR=/tmp
MPGPU_ILQR_MIRROR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ilqr.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for env in "MPGPU_ILQR_MIRROR=0" "MPGPU_ILQR_MIRROR=1" "MPGPU_ILQR_MEMSET=1" "MPGPU_ILQR_MIRROR=0" "MPGPU_ILQR_MIRROR=1" "MPGPU_ILQR_MEMSET=1"; do
  echo "== $env"; env $env timeout -k 10 300 python3 tools/ilqr_time.py --solve-only --solve-reps 6 > $O/ilqr.log 2>&1 && grep solve $O/ilqr.log | tail -5 | awk '{print $2}' | tr '\n' ' ' && echo || exit 1
done
