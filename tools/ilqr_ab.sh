#!/bin/bash
# A/B of iLQR builds: wall/kernel times (tools/ilqr_time.py) and a kernel-trace split per build.
# usage: bash tools/ilqr_ab.sh TAG lib-suffix...   ("" = libmpgpu.so)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for v in "$@"; do
  n=${v:-default}
  echo "== lib$v" >> gpurun_out/$TAG/ilqr.log
  MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$n -o run --output-format csv -- python3 tools/ilqr_time.py >> gpurun_out/$TAG/ilqr.log 2>&1 || exit 1
  python3 - gpurun_out/$TAG/prof_$n/run_kernel_stats.csv >> gpurun_out/$TAG/ilqr.log <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'ilqr' in r['Name']:
        print("  %-28s %6s calls %10.1f us avg" % (r['Name'].split('::')[1].split('(')[0], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
cat gpurun_out/$TAG/ilqr.log
