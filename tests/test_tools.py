"""CPU tests of the measurement tooling: tools/pmc_roofline.py's per-leg ranking (the iLQR / Hybrid A*
rooflines of the bench line come from it) and bench.leg_roofline, on synthetic rocprofv3 CSVs."""
import csv
import importlib.util
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write_stats(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, calls, avg in rows:
            w.writerow([name, calls, calls * avg, avg, 0, avg, avg, 0])


def _write_pmc(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
        for name, counter, vals in rows:
            for v in vals:
                w.writerow([name, counter, v])


K_PIPE = "void (anonymous namespace)::ilqr_search_pipe_kernel<16, 4, 2>((anonymous namespace)::IlqrDev, int)"
K_FUSED = "(anonymous namespace)::ilqr_backward_fused_kernel((anonymous namespace)::IlqrDev, int, double const*)"
K_D4 = "void (anonymous namespace)::ilqr_deriv4_kernel((anonymous namespace)::IlqrDev, int)"


def test_leg_ranking_and_bench_roofline(tmp_path):
    d = str(tmp_path)
    _write_stats(os.path.join(d, "prof_ilqr", "run_kernel_stats.csv"),
                 [(K_FUSED, 25, 209_000.0), (K_PIPE, 45, 459_000.0), (K_D4, 37, 32_000.0)])
    _write_pmc(os.path.join(d, "pmc_ilqr", "run_counter_collection.csv"),
               [(K_PIPE, "SQ_INSTS_VALU", [1.0e8, 1.1e8]), (K_PIPE, "SQ_ACTIVE_INST_VALU", [3.0e8, 3.0e8]),
                (K_PIPE, "SQ_WAVE_CYCLES", [1.0e9, 1.0e9]), (K_D4, "SQ_INSTS_VALU", [9.0e6])])
    pr = _load("tools/pmc_roofline.py", "pmc_roofline")
    buf = io.StringIO()
    with redirect_stdout(buf):
        pr.main(d)
    rl = json.loads(buf.getvalue())
    leg = rl["legs"]["ilqr_solve"]
    names = [k["name"] for k in leg["kernels"]]
    assert names == ["ilqr_search_pipe_kernel<16, 4, 2>", "ilqr_backward_fused_kernel", "ilqr_deriv4_kernel"]
    assert abs(sum(k["share"] for k in leg["kernels"]) - 1.0) < 1e-12
    pipe = leg["kernels"][0]
    assert abs(pipe["SQ_INSTS_VALU"] - 1.05e8) < 1 and abs(pipe["wave_valu_busy"] - 0.3) < 1e-12
    assert abs(pipe["valu_frac"] - 1.05e8 / 459e-6 / pr.VALU_PEAK) < 1e-9
    assert "ha_plan" not in rl["legs"]  # no plan-only trace in this directory
    sys.path.insert(0, ROOT)
    bench = _load("bench.py", "bench_mod")
    rl["path"] = "x.json"
    out = bench.leg_roofline(rl, "ilqr_solve")
    assert out["kernel"] == "ilqr_search_pipe_kernel<16, 4, 2>" and out["bound"] == "valu"
    assert out["frac"] == pipe["valu_frac"] and out["share_of_leg"] == pipe["share"]
    assert [k["name"] for k in out["kernels"]] == names
    assert bench.leg_roofline(rl, "ha_plan") is None
