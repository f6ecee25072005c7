"""Per-iteration split of the last mp_ha_plan in a rocprofv3 kernel trace: ha_iter / ha_book
durations over the plan's iterations (every 50th printed), their sums and the plan span."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = []
for r in rows:
    m = re.search(r"(ha_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
    if m:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
inits = [i for i, k in enumerate(ks) if k[2] == "ha_init_kernel"]
last = ks[inits[-1]:]
it = [k for k in last if k[2].startswith("ha_iter")]
bk = [k for k in last if k[2].startswith("ha_book")]
print("iterations %d  span %.2f ms  iter %.2f ms  book %.2f ms" % (
    len(it), (last[-1][1] - last[0][0]) / 1e6, sum(e - s for s, e, _ in it) / 1e6, sum(e - s for s, e, _ in bk) / 1e6))
print("  iter us:", " ".join("%.0f" % ((e - s) / 1e3) for s, e, _ in it[::50]))
print("  book us:", " ".join("%.0f" % ((e - s) / 1e3) for s, e, _ in bk[::50]))
