#!/bin/bash
# GPU pass: parity tests, bench, kernel-trace stats, then PMC passes (each its own run).
# usage: bash tools/gpu_pass.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q "$@" > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; tail -15 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-single --no-extras"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$TAG/pmc2 -o run --output-format csv -- $B > gpurun_out/$TAG/pmc2.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$TAG/pmc3 -o run --output-format csv -- $B > gpurun_out/$TAG/pmc3.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/$TAG/pmc1 -o run --output-format csv -- $B > gpurun_out/$TAG/pmc1.log 2>&1 &&
python3 tools/pmc_traffic.py gpurun_out/$TAG 8 8192 50 > gpurun_out/$TAG/traffic.json && cat gpurun_out/$TAG/traffic.json &&
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 --traffic gpurun_out/$TAG/traffic.json > gpurun_out/$TAG/bench.log 2>&1 && tail -1 gpurun_out/$TAG/bench.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/$TAG/prof.log 2>&1
echo "prof chain exit $?"
