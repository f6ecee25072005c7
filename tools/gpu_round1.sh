#!/bin/bash
# First GPU pass: parity tests, bench, rocprof kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" | tee -a gpurun_out/pytest_gpu.log
tail -30 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/prof.log 2>&1
echo "prof exit $?"
find gpurun_out/prof -name "*stats*" | head
