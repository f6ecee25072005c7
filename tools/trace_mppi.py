"""Print the last N MPPI kernels of a rocprofv3 --kernel-trace CSV as a timeline (us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = [r for r in rows if any(k in r["Kernel_Name"] for k in ("mppi", "noise", "final"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'].split('(')[0][-28:]:28s} q{r['Stream_Id']} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f}")
