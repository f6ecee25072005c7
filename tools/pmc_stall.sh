#!/bin/bash
# Stall breakdown of mppi_plan_kernel (two PMC passes of <= 8 SQ counters each) for lane layouts.
# usage: bash tools/pmc_stall.sh TAG "S LPR" ["S LPR" ...]
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
PB="SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC"
for cfg in "$@"; do
  set -- $cfg
  n=s$1_l$2
  i=0
  for P in "$PA" "$PB"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $D/${n}_$i -o run --output-format csv -- python3 tools/plan_time.py --scenes $1 --lpr $2 --reps 4 > $D/${n}_$i.log 2>&1 || exit 1
  done
  python3 - $D $n >> $D/stall.log <<'PY'
import csv, sys, glob, collections
d, n = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(f"{d}/{n}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mppi_plan_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"== {n}")
for k, v in sorted(acc.items()):
    print(f"  {k:26s} {sum(v)/len(v):18.0f}")
PY
done
cat $D/stall.log
