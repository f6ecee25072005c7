# iLQR: the finish kernel's zeroing vs a memset launch per solve iteration (MPGPU_ILQR_MEMSET=1)
set -o pipefail
O=gpurun_out/r05zc; mkdir -p $O
export TMPDIR=/tmp
for env in "MPGPU_ILQR_MEMSET=0" "MPGPU_ILQR_MEMSET=1" "MPGPU_ILQR_MEMSET=0" "MPGPU_ILQR_MEMSET=1"; do
  echo "== $env"; env $env timeout -k 10 300 python3 tools/ilqr_time.py --solve-only --solve-reps > $O/ilqr.log 2>&1 && grep solve $O/ilqr.log || exit 1
done
