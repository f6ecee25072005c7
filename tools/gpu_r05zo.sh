# the driver's own bench invocation (defaults) on the final tree
set -o pipefail
O=gpurun_out/r05zo; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err; rc=$?; tail -c 600 $O/bench.log; exit $rc
