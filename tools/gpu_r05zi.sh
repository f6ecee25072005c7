# the primitive-table memo test + the HA GPU tests on the final tree
set -o pipefail
O=gpurun_out/r05zi; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hastar.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; exit $rc
