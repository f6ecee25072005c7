#!/bin/bash
# One GPU pass on the gpurun box, by steps (each under its own time limit, chained: the first failure ends
# the pass).  Replaces round 5's one-off tools/gpu_r05*.sh scripts.
# usage: bash tools/gpu_run.sh TAG STEP [STEP ...]
#   tests[:PYTEST-ARGS]  the GPU suite (pytest -m gpu), e.g. tests or "tests:tests/test_gpu_ilqr.py -k solve"
#   smoke                __graft_entry__.smoke()
#   bench[:ARGS]         python bench.py ARGS (default: the driver's --steps 20 --warmup 5)
#   prof                 rocprofv3 kernel-trace stats of a short bench run
#   pass                 tools/gpu_pass4.sh's PMC / roofline / bench chain (its own output dir)
#   cmd:COMMAND          any other command (its output to TAG/cmdN.log)
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  case $name in
    tests)
      timeout -k 10 1500 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        > $O/pytest_gpu_$n.log 2>&1
      rc=$?; tail -4 $O/pytest_gpu_$n.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; tail -3 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${arg:---steps 20 --warmup 5} > $O/bench_$n.log 2>&1
      rc=$?; tail -c 2500 $O/bench_$n.log ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
        python3 bench.py --steps 30 --warmup 3 --no-cpu > $O/prof.log 2>&1
      rc=$?; find $O -name 'run_kernel_trace.csv' | xargs -r gzip -f ;;
    pass)
      bash tools/gpu_pass4.sh ${TAG}_pass_notest
      rc=$? ;;
    cmd)
      timeout -k 10 900 bash -c "$arg" > $O/cmd$n.log 2>&1
      rc=$?; tail -c 2500 $O/cmd$n.log ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
  echo "step $n ($name) exit $rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
