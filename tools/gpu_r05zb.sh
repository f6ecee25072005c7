# iLQR: list-buffer parity (no memset launch per solve iteration): iLQR GPU tests, then solve timing
set -o pipefail
O=gpurun_out/r05zb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilqr.py tests/test_gpu_pipeline.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ilqr_time.py --solve-only > $O/ilqr.log 2>&1 && tail -4 $O/ilqr.log
