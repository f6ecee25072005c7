"""Median back-to-back gap (next Start - this End) and duration per (kernel, grid, LDS) from a
rocprofv3 kernel trace: python3 gap_stats.py DIR/run_kernel_trace.csv"""
import csv
import statistics as st
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gaps, durs = defaultdict(list), defaultdict(list)
key = lambda r: (r["Kernel_Name"].split("(")[0][:40], r["Grid_Size_X"], r["LDS_Block_Size"])
last = {}
for a in rows:
    k = key(a)
    durs[k].append((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
    if k in last:  # previous launch of the same kernel/grid (other streams' launches in between)
        gaps[k].append((int(a["Start_Timestamp"]) - int(last[k]["End_Timestamp"])) / 1e3)
    last[k] = a
for k in durs:
    g = gaps.get(k, [0.0])
    print(f"{str(k):70s} n {len(durs[k]):4d} dur {st.median(durs[k]):8.1f} us  gap {st.median(g):6.2f} us")
