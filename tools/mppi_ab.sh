#!/bin/bash
# A/B of MPPI builds: mppi_plan_kernel average duration (kernel trace) and VALU instructions
# per launch (one PMC pass) for each libmpgpu variant, plus the bench's headline value.
# usage: bash tools/mppi_ab.sh TAG lib-suffix...   ("" = libmpgpu.so)
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 3 --no-cpu --no-extras"
for v in "$@"; do
  n=${v:-default}
  export MPGPU_LIB=$PWD/motionplanning_amd/lib/libmpgpu$v.so
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $D/k_$n -o run --output-format csv -- $B > $D/k_$n.log 2>&1 || exit 1
  timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $D/p_$n -o run --output-format csv -- $B --no-single > $D/p_$n.log 2>&1 || exit 1
  python3 - $D $n >> $D/ab.log <<'PY'
import csv, sys, collections, json
d, n = sys.argv[1], sys.argv[2]
out = [f"== {n}"]
for r in csv.DictReader(open(f"{d}/k_{n}/run_kernel_stats.csv")):
    if 'mppi_plan' in r['Name']:
        out.append("  %-40s %6s calls %9.1f us avg" % (r['Name'].split('(')[0][-40:], r['Calls'], float(r['AverageNs']) / 1e3))
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/p_{n}/run_counter_collection.csv")):
    if "mppi_plan_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    out.append(f"  {k:24s} {sum(v)/len(v):16.0f}")
for line in open(f"{d}/k_{n}.log"):
    if line.startswith("{"):
        j = json.loads(line)
        out.append(f"  bench value {j['value']:.4g} ms_per_step {j['ms_per_step']:.4f}")
print("\n".join(out))
PY
done
cat $D/ab.log
