"""Per-launch durations and gaps of the Hybrid A* search loop from a rocprofv3 kernel trace.

usage: python tools/ha_trace_gap.py DIR   (DIR/run_kernel_trace.csv[.gz] of tools/ha_plan_time.py)
Prints, for the last plan in the trace, the launch count, the summed kernel time, the summed gaps
between consecutive HA launches, and the split at the tail shape (12-wave blocks).
"""
import csv
import gzip
import os
import re
import sys


def rows(d):
    p = os.path.join(d, "run_kernel_trace.csv")
    f = gzip.open(p + ".gz", "rt") if not os.path.exists(p) else open(p)
    with f:
        for r in csv.DictReader(f):
            yield r


def main(d):
    ks = []
    for r in rows(d):
        n = r["Kernel_Name"]
        m = re.search(r"::(\w+(?:<[^(]*?>)?)\(", n)
        name = m.group(1) if m else n
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ks.sort()
    # plans start at ha_init_kernel; take the last one
    starts = [i for i, k in enumerate(ks) if k[2] == "ha_init_kernel"]
    i0 = starts[-1]
    seq = [k for k in ks[i0:] if k[2].startswith(("ha_iter", "ha_step", "ha_book"))]
    tot = sum(e - s for s, e, _ in seq)
    gaps = sum(max(0, seq[i + 1][0] - seq[i][1]) for i in range(len(seq) - 1))
    by = {}
    for s, e, n in seq:
        c = by.setdefault(n, [0, 0.0])
        c[0] += 1
        c[1] += e - s
    print(f"launches {len(seq)}  kernel {tot / 1e6:.2f} ms  gaps {gaps / 1e6:.2f} ms  span {(seq[-1][1] - seq[0][0]) / 1e6:.2f} ms")
    for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
        print(f"  {n:32s} {c:5d} x {t / c / 1e3:7.2f} us = {t / 1e6:6.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
