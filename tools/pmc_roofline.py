"""Per-kernel VALU rooflines of the iLQR and Hybrid A* legs from a rocprofv3 pass directory.

usage: python tools/pmc_roofline.py DIR > roofline.json
  DIR/pmc4/run_counter_collection.csv  SQ_INSTS_VALU, SQ_WAVES, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, ...
                                       (rocprofv3 --pmc over the bench command with its extras; pmc1 if absent)
  DIR/prof/run_kernel_stats.csv        average launch durations (rocprofv3 --kernel-trace --stats of
                                       the same bench command, a separate run)
  legs (tools/gpu_pass4.sh), each a kernel trace + a --pmc pass of one command that runs only that leg:
  DIR/prof_ilqr, DIR/pmc_ilqr          tools/ilqr_time.py --solve-only (one mp_ilqr_solve, configs[2])
  DIR/prof_ha,   DIR/pmc_ha            tools/ha_plan_time.py (mp_ha_plan, configs[3])

For each kernel: mean SQ_INSTS_VALU per launch (wave-instructions), the kernel-trace mean duration,
achieved = insts / duration, frac = achieved / peak with peak = 1,024 SIMDs x 2.4 GHz / 4 cycles per
wave64 fp64 VALU instruction = 6.144e11 wave-insts/s (the same peak as the MPPI line's roofline.valu),
and the VALU-busy share of a resident wave's cycles (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES).
Every launched kernel is kept (no name filter).  For a leg the kernels are ranked by their share of the
leg's summed kernel time (calls x average duration); the leg's setup kernels (the initial rollout of
the iLQR instances, the HA* primitive/wall tables) are included and show up with their small shares.
bench.py reads the JSON (--roofline) and attaches the legs to the iLQR and Hybrid A* lines.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

VALU_PEAK = 1024 * 2.4e9 / 4
LEGS = {"ilqr_solve": ("prof_ilqr", "pmc_ilqr"), "ha_plan": ("prof_ha", "pmc_ha")}


def short(name):
    """'void (anonymous namespace)::ha_iter_kernel<4, 16>((anonymous ...' -> 'ha_iter_kernel<4, 16>'"""
    m = re.search(r"::(\w+(?:<[^(]*?>)?)\(", name)
    if m:
        return m.group(1)
    m = re.match(r"(?:void\s+)?(\w+(?:<[^(]*?>)?)\(", name)
    return m.group(1) if m else name


def counters(path):
    vals = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return vals
    with open(path) as f:
        for row in csv.DictReader(f):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def durations(path):
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            e = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
            e["calls"] += int(row["Calls"])
            e["total_ns"] += float(row["TotalDurationNs"]) if "TotalDurationNs" in row else \
                float(row["AverageNs"]) * int(row["Calls"])
    for e in out.values():
        e["avg_ns"] = e["total_ns"] / max(1, e["calls"])
    return out


def entry(c, d):
    e = {}
    for name, v in c.items():
        e[name] = sum(v) / len(v)
    if c:
        e["launches_pmc"] = len(next(iter(c.values())))
    if d:
        e["avg_ns"] = d["avg_ns"]
        e["calls_trace"] = d["calls"]
    if "SQ_INSTS_VALU" in e and "avg_ns" in e:
        e["valu_achieved"] = e["SQ_INSTS_VALU"] / (e["avg_ns"] * 1e-9)
        e["valu_frac"] = e["valu_achieved"] / VALU_PEAK
    if "SQ_ACTIVE_INST_VALU" in e and e.get("SQ_WAVE_CYCLES", 0) > 0:
        e["wave_valu_busy"] = e["SQ_ACTIVE_INST_VALU"] / e["SQ_WAVE_CYCLES"]  # per resident wave
    return e


def leg(d, prof, pmc):
    dur = durations(os.path.join(d, prof, "run_kernel_stats.csv"))
    if not dur:
        return None
    cnt = counters(os.path.join(d, pmc, "run_counter_collection.csv"))
    total = sum(e["total_ns"] for e in dur.values())
    ks = []
    for k, dd in dur.items():
        e = entry(cnt.get(k, {}), dd)
        e.update(name=k, calls=dd["calls"], avg_us=dd["avg_ns"] / 1e3, total_ms=dd["total_ns"] / 1e6,
                 share=dd["total_ns"] / total)
        ks.append(e)
    ks.sort(key=lambda e: -e["total_ms"])
    return {"source": os.path.join(d, prof) + " + " + os.path.join(d, pmc), "total_ms": total / 1e6,
            "kernels": ks}


def main(d):
    pm = os.path.join(d, "pmc4", "run_counter_collection.csv")  # the bench with its extras
    cnt = counters(pm if os.path.exists(pm) else os.path.join(d, "pmc1", "run_counter_collection.csv"))
    dur = durations(os.path.join(d, "prof", "run_kernel_stats.csv"))
    out = {"source": d, "peak_wave_insts_per_s": VALU_PEAK, "kernels": {}, "legs": {}}
    for k in sorted(set(cnt) | set(dur)):
        out["kernels"][k] = entry(cnt.get(k, {}), dur.get(k))
    for name, (prof, pmc) in LEGS.items():
        lg = leg(d, prof, pmc)
        if lg:
            out["legs"][name] = lg
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
