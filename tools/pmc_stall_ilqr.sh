#!/bin/bash
# Stall breakdown of the iLQR kernels (tools/ilqr_time.py: backward, forward, solve) from two PMC
# passes of <= 8 SQ counters each; per-kernel means per launch.
# usage: bash tools/pmc_stall_ilqr.sh TAG
set -o pipefail
TAG=$1
D=gpurun_out/$TAG; mkdir -p $D
export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
PB="SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $D/p$i -o run --output-format csv -- python3 tools/ilqr_time.py > $D/p$i.log 2>&1 || exit 1
done
python3 - $D > $D/stall.log <<'PY'
import csv, sys, glob, collections, re
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(ilqr_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
        if m:
            acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(f"== {k}")
    for c, v in sorted(cs.items()):
        print(f"  {c:26s} {sum(v)/len(v):18.0f}  ({len(v)} launches)")
PY
cat $D/stall.log
