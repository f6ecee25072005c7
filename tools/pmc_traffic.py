"""Per-launch HBM traffic of the dominant kernels from rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py DIR S K H  (DIR holds pmc1/ pmc2/ pmc3/ from tools/gpu_pass4.sh;
       S, K, H = the bench configuration those passes ran)

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM [CDNA4]): on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads -> doubled here;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Both count memory-side (fabric)
requests, so Infinity-Cache hits may be included.  Prints one JSON object.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

KERNELS = ("mppi_plan_kernel", "noise_prep_kernel")


def variant(name):
    """'void (anonymous namespace)::mppi_plan_kernel<512, 2, true>(mpk::...' -> 'mppi_plan_kernel<512, 2, true>'"""
    m = re.search(r"::(\w+(?:<[^(]*?>)?)\(", name)
    return m.group(1) if m else name


def load(path):
    vals = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            for k in KERNELS:
                if k in name:
                    vals[variant(name)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(d, S, K, H):
    out = {"source": d, "config": {"S": S, "K": K, "H": H}, "correction": "traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving)"}
    merged = defaultdict(dict)
    for sub in ("pmc1", "pmc2", "pmc3"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for k, counters in load(p).items():
            for c, v in counters.items():
                merged[k][c] = sum(v) / len(v)  # mean per launch
                merged[k][c + "_launches"] = len(v)
    for k, c in merged.items():
        e = dict(c)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["fetch_bytes"] = 2 * c["FETCH_SIZE"] * 1024
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        out[k] = e
    # the headline entry "mppi_plan_kernel": the variant of the S-scene launch the bench times (the
    # one writing the most per launch: other variants in the same run are the 1-scene and closed-loop
    # launches)
    plans = [k for k in merged if k.startswith("mppi_plan_kernel<")]
    if plans:
        head = max(plans, key=lambda k: (merged[k].get("WRITE_SIZE", 0), merged[k].get("SQ_WAVES", 0)))
        out["mppi_plan_kernel"] = dict(out[head], variant=head)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *map(int, sys.argv[2:5]))
