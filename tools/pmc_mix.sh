#!/bin/bash
# VALU instruction mix of the bench's kernels (two PMC passes), summarised per launch.
set -o pipefail
D=gpurun_out/${1:-mix}; mkdir -p $D; export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-single --no-extras"
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT -d $D/m1 -o run --output-format csv -- $B > $D/m1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS -d $D/m2 -o run --output-format csv -- $B > $D/m2.log 2>&1 &&
python3 - $D <<'PY'
import csv, sys, collections
d = sys.argv[1]
for sub in ("m1", "m2"):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
        if "mppi_plan_kernel" in row["Kernel_Name"]:
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{k:28s} {sum(v)/len(v):16.0f}")
PY
