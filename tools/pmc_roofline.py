"""Per-kernel VALU rooflines of the iLQR and Hybrid A* legs from a rocprofv3 pass directory.

usage: python tools/pmc_roofline.py DIR > roofline.json
  DIR/pmc4/run_counter_collection.csv  SQ_INSTS_VALU, SQ_WAVES, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, ...
                                       (rocprofv3 --pmc over the bench command with its extras; pmc1 if absent)
  DIR/prof/run_kernel_stats.csv        average launch durations (rocprofv3 --kernel-trace --stats of
                                       the same bench command, a separate run)

For each kernel: mean SQ_INSTS_VALU per launch (wave-instructions), the kernel-trace mean duration,
achieved = insts / duration, frac = achieved / peak with peak = 1,024 SIMDs x 2.4 GHz / 4 cycles per
wave64 fp64 VALU instruction = 6.144e11 wave-insts/s (the same peak as the MPPI line's roofline.valu),
and the VALU-busy share of a resident wave's cycles (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES).
bench.py reads the JSON (--roofline) and attaches the entries to the iLQR and Hybrid A* lines.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

VALU_PEAK = 1024 * 2.4e9 / 4
KERNELS = ("ilqr_deriv_kernel", "ilqr_backward_quad_kernel", "ilqr_backward_staged_kernel", "ilqr_backward_kernel", "ilqr_forward_quad_kernel",
           "ilqr_search_kernel", "ilqr_search_rest_kernel", "ilqr_search_finish_kernel", "ilqr_rollout_kernel",
           "ha_iter_kernel", "ha_book_kernel", "ha_retrieve_kernel", "mppi_plan_kernel", "final_rollout_kernel")


def short(name):
    """'void (anonymous namespace)::ha_iter_kernel<4, 16>((anonymous ...' -> 'ha_iter_kernel<4, 16>'"""
    m = re.search(r"::(\w+(?:<[^(]*?>)?)\(", name)
    base = m.group(1) if m else name
    return base if base.split("<")[0] in KERNELS else None


def counters(path):
    vals = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return vals
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k:
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def durations(path):
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            if k:
                out[k] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"])}
    return out


def main(d):
    pm = os.path.join(d, "pmc4", "run_counter_collection.csv")  # gpu_pass3.sh: the bench with its extras
    cnt = counters(pm if os.path.exists(pm) else os.path.join(d, "pmc1", "run_counter_collection.csv"))
    dur = durations(os.path.join(d, "prof", "run_kernel_stats.csv"))
    out = {"source": d, "peak_wave_insts_per_s": VALU_PEAK, "kernels": {}}
    for k in sorted(set(cnt) | set(dur)):
        c = cnt.get(k, {})
        e = {}
        for name, v in c.items():
            e[name] = sum(v) / len(v)
        if c:
            e["launches_pmc"] = len(next(iter(c.values())))
        if k in dur:
            e["avg_ns"] = dur[k]["avg_ns"]
            e["calls_trace"] = dur[k]["calls"]
        if "SQ_INSTS_VALU" in e and "avg_ns" in e:
            e["valu_achieved"] = e["SQ_INSTS_VALU"] / (e["avg_ns"] * 1e-9)
            e["valu_frac"] = e["valu_achieved"] / VALU_PEAK
        if "SQ_ACTIVE_INST_VALU" in e and e.get("SQ_WAVE_CYCLES", 0) > 0:
            e["wave_valu_busy"] = e["SQ_ACTIVE_INST_VALU"] / e["SQ_WAVE_CYCLES"]  # per resident wave
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
