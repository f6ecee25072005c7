"""MPPI rollout-step throughput on MI355X (BASELINE.json metric).

One step = one MPPIPlan (OptimalControl/MPPI/src/MPPIUtils.jl:169-203) for each of
S scenes per GPU (default 8 = the per-GPU shard of configs[4], "64 scenes sharded
8xMI355X"); every scene is configs[1]: K=8192 rollouts, H=50 horizon steps, 7-state
dynamic bicycle, 100x100 occupancy grid, device Philox noise, the full
TrajectoryCollection (every rollout's trajectory and control list) written to HBM,
weights + MPPICtrl + final rollout.  One plan launch per step (Philox noise drawn inside the
rollout loop) + the final rollout of MPPICtrl on its context's side stream (final_stream=1;
--final-inline keeps it in the plan kernel); consecutive steps are independent batches and
alternate over --streams contexts (default 3, one stream each, calls_in_flight = 3: each launch takes
the one-rollout-per-lane layout, one wave per SIMD, so the calls in flight share every SIMD and
step i's serial final rollout and its straggler waves overlap steps i+1 and i+2); every step's
outputs are complete when the timed region's closing synchronize returns.  Inputs
are resident in HBM before the timed region.  N>1: one process per GPU, each
solves its own S scenes (weak scaling) and the ranks all-gather the optimal
controls over RCCL (the north star's exchange step).  The single-scene
(configs[1] exactly, latency-bound) rate is reported beside it in "single_scene".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scenes S] [--cpu-seconds T]
"""
import argparse
import ctypes
import json
import os
import sys
import time

# Hardware queues, before the HIP runtime starts (import torch): the headline's three contexts drive six streams
# (a plan stream and a final-rollout side stream each) beside torch's own, and at HIP's default of 4 queues per
# process streams share a queue, so the alternating calls serialise instead of overlapping (r06r, driver args,
# two contexts: 0.96e10 at 4 queues, 1.10-1.11e10 at 8; r06za, three contexts: 1.31e10 at 8, 1.36e10 at 12).
_HWQ = os.environ.get("GPU_MAX_HW_QUEUES", "")
if not _HWQ.isdigit() or int(_HWQ) < 12:
    os.environ["GPU_MAX_HW_QUEUES"] = "12"

import numpy as np
import torch  # import before libmpgpu so both share torch's HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASE = json.load(open(os.path.join(ROOT, "BASELINE.json")))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X fp64 vector (AMD spec)
VALU_SIMDS, VALU_CLOCK_HZ, FP64_ISSUE_CYCLES = 1024, 2.4e9, 4  # 256 CUs x 4 SIMD-32; wave64 fp64 op = 4 cycles


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scenes", type=int, default=8, help="scenes per GPU per step (configs[4] shard)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--rotate", type=int, default=3, help="output buffer sets rotated (>256 MB MALL at S=8)")
    ap.add_argument("--no-single", action="store_true", help="skip the single-scene (configs[1]) line")
    ap.add_argument("--no-whole", action="store_true", help="skip the configs[4]-whole (64 scenes, one GPU) line")
    ap.add_argument("--streams", type=int, default=3,
                    help="contexts (streams) the headline's consecutive independent plan calls alternate over")
    ap.add_argument("--roofline", default=os.path.join(ROOT, "profiles", "roofline_latest.json"),
                    help="per-kernel VALU counts + durations (tools/pmc_roofline.py) for the iLQR / HA* rooflines")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="rocprofv3 PMC summary (tools/pmc_traffic.py) for roofline.traffic")
    ap.add_argument("--final-inline", action="store_true",
                    help="final rollout at the end of the plan kernel (final_stream=0) instead of the side stream")
    ap.add_argument("--no-extras", action="store_true", help="skip the iLQR (configs[2]) and Hybrid A* (configs[3]) lines")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal of N>1 on a one-GPU box: every rank on cuda:0, gloo instead of RCCL")
    return ap.parse_args()


def algorithmic_bytes(S, K, H):
    """Compulsory HBM bytes of one mppi_plan_kernel launch: per rollout-step
    16 B control + 56 B state written (the TrajectoryCollection; device Philox noise is drawn
    in registers, nothing read); per rollout the initial state row, cost and feasibility flag."""
    per_rollout = H * (16 + 56) + 56 + 8 + 1
    return S * K * per_rollout


def host_cpu():
    """The host CPU model (lscpu's "Model name", from /proc/cpuinfo) and the CPUs this process may use."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    return {"model": model, "host_cpus": os.cpu_count(), "usable_cpus": usable}


def gather_f64(vals, dev):
    """all_gather of a short float64 vector from every rank -> list of lists (rank order)."""
    world = dist.get_world_size()
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor(vals, dtype=torch.float64, device=dev if on_dev else "cpu")
    if on_dev:
        out = torch.empty((world, len(vals)), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(out, t)
        return out.cpu().tolist()
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.tolist() for p in parts]


def run(a, S, ctx, dev, world, rank, steps, warmup, rotate, cfg5=True, nstreams=1):
    """Time `steps` plan calls of S scenes; returns (elapsed_s_max, kernel_ms_mean, valid, K, H, fc, fields).
    cfg5: the scenes are rank r's block [rS, (r+1)S) of configs[4]'s 64 (own X0 and own obstacle_field.mat
    grid each, configs.cfg5_shard); else S copies of configs[1]'s scene.
    nstreams > 1: consecutive (independent) calls alternate over that many contexts -- one stream each --
    so call i+1's rollouts fill the SIMDs call i's last waves leave idle (the straggler window of a lone
    launch); each call's outputs are complete when the closing synchronize returns."""
    from motionplanning_amd import configs
    from motionplanning_amd.abi import MP_NOISE_PHILOX, ptr

    if cfg5:
        c = configs.cfg5_shard(rank * S, S, noise_mode=MP_NOISE_PHILOX, seed=20260415)
        X0, goal, grid, fields = c["X0"], c["goal"], c["grid"], c["fields"]
    else:
        c = configs.cfg2(noise_mode=MP_NOISE_PHILOX, seed=20260415)
        X0, goal, grid, fields = np.tile(c["X0"], (S, 1)), np.tile(c["goal"], (S, 1)), np.tile(c["grid"], (S, 1, 1)), []
    p = c["params"]
    p.scene_base = rank * S  # global scene ids: rank r plans scenes [rS, (r+1)S) of the job
    p.final_stream = 0 if a.final_inline else 1  # final rollout on the side stream, overlapping the next step
    p.calls_in_flight = nstreams  # the launch layout for nstreams calls sharing the device (include/mpgpu.h)
    K, H = p.K, p.H

    def t(x, dt=torch.float64):
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dt, device=dev).contiguous()

    dX0, dgoal = t(X0), t(goal)
    dun = t(np.zeros((S, H, 2)))
    dgrid = t(grid, torch.uint8)
    from motionplanning_amd.context import Context
    ctxs = [ctx] + [Context(ctx.device) for _ in range(nstreams - 1)]
    for c_ in ctxs[1:]:
        c_.lib.mp_ctx_kernel_timing(c_.handle, 1)
    tstreams = [torch.cuda.ExternalStream(c_.stream, device=dev) for c_ in ctxs]
    sets = []
    # output sets: a multiple of the stream count, so two calls in flight on different streams never share one
    nsets = -(-max(1, rotate) // nstreams) * nstreams
    for _ in range(nsets):
        sets.append(dict(
            U=torch.empty((S, H, 2), dtype=torch.float64, device=dev),
            traj=torch.empty((S, H + 1, 7), dtype=torch.float64, device=dev),
            cost=torch.empty(S, dtype=torch.float64, device=dev),
            feas=torch.empty(S, dtype=torch.int32, device=dev),
            rc=torch.empty(S, dtype=torch.int32, device=dev),
            fc=torch.empty(S, dtype=torch.int32, device=dev),
            ctraj=torch.empty((S, H + 1, 7, K), dtype=torch.float64, device=dev),  # SoA (include/mpgpu.h)
            cctrl=torch.empty((S, H, K, 2), dtype=torch.float64, device=dev),
            ccost=torch.empty((S, K), dtype=torch.float64, device=dev),
            cfeas=torch.empty((S, K), dtype=torch.uint8, device=dev),
        ))
    gathered = [torch.empty((world * S, H, 2), dtype=torch.float64, device=dev) for _ in range(nstreams)]

    def step(i):
        b = sets[i % len(sets)]
        c_ = ctxs[i % nstreams]
        p.offset = i
        c_.check(c_.lib.mp_mppi_plan_dev(
            c_.handle, ctypes.byref(p), S, ptr(dX0), ptr(dgoal), ptr(dun), None, ptr(dgrid), None, ptr(b["U"]),
            ptr(b["traj"]), ptr(b["cost"]), ptr(b["feas"]), ptr(b["rc"]), ptr(b["fc"]), ptr(b["ctraj"]),
            ptr(b["cctrl"]), ptr(b["ccost"]), ptr(b["cfeas"])))
        if world > 1 and dist.get_backend() == "nccl":
            with torch.cuda.stream(tstreams[i % nstreams]):  # RCCL, on the stream of the call's context
                dist.all_gather_into_tensor(gathered[i % nstreams], b["U"])
        elif world > 1:  # --share-device rehearsal over gloo: host copies
            parts = [torch.empty((S, H, 2), dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, b["U"].cpu())
            gathered[i % nstreams].copy_(torch.cat(parts))

    def sync():
        for c_ in ctxs:
            c_.check(c_.lib.mp_ctx_synchronize(c_.handle))
        torch.cuda.synchronize()

    def kernel_ms():  # summed HIP-event spans and launch counts over the contexts (resets them)
        tot, n = 0.0, 0
        for c_ in ctxs:
            ms, cnt = ctypes.c_double(), ctypes.c_int32()
            c_.check(c_.lib.mp_ctx_kernel_ms(c_.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            tot, n = tot + ms.value, n + cnt.value
        return tot, n

    for i in range(warmup):
        step(i)
    sync()
    kernel_ms()  # drop the warmup events
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms_sum, cnt = kernel_ms()
    kern_ms = ms_sum / max(1, cnt)
    ok = all(bool((b["rc"] == K + 1).all().item()) and bool(torch.isfinite(b["cost"]).all().item())
             for b in sets[: min(len(sets), warmup + steps)])
    if world > 1:
        rows = gather_f64([elapsed, kern_ms, 0.0 if ok else 1.0], dev)
        elapsed, kern_ms = max(r[0] for r in rows), max(r[1] for r in rows)
        ok = all(r[2] == 0.0 for r in rows)
    for c_ in ctxs[1:]:
        c_.close()
    return elapsed, kern_ms, ok, K, H, p.feasibility_count, fields


def main():
    a = parse()
    # `--gpus N` without a launcher: N fresh rank processes of this same command (before any GPU call)
    from motionplanning_amd.launch import relaunch_if_needed

    status = relaunch_if_needed(a.gpus)
    if status is not None:
        sys.exit(status)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = 0 if a.share_device else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if a.share_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    # which ranks joined, on which GPU (PCI bus id): proof that N ranks ran on N devices
    pci = getattr(torch.cuda.get_device_properties(gpu), "pci_bus_id", -1)
    joined = gather_f64([rank, local, gpu, pci], dev) if world > 1 else [[0, local, gpu, pci]]

    from motionplanning_amd.context import Context

    ctx = Context(gpu)
    ctx.lib.mp_ctx_kernel_timing(ctx.handle, 1)
    stream = torch.cuda.ExternalStream(ctx.stream, device=dev)
    torch.cuda.set_stream(stream)  # RCCL all_gather is ordered after the plan kernel

    S = a.scenes
    # The GPU legs of the extras (iLQR, Hybrid A*, tracker, closed loop) run first and the headline after
    # them, on a GPU that has been busy for seconds as in continuous serving: after an idle box, W = 5
    # warmup steps (1.5 ms of work) leave the clocks ramping through a short timed region (r04d: 20 timed
    # steps give a 0.298 ms plan kernel after 5 warmup steps, 0.280 ms after 2,000).  The timed region
    # itself is unchanged: exactly K steps, every output complete.  CPU baselines run last (the GPU idles).
    cpu_jobs = [] if (rank == 0 and world == 1 and not a.no_cpu) else None
    extras = {}
    if not a.no_extras:
        extras["ilqr"] = bench_ilqr(ctx, world, rank, cpu=cpu_jobs)
        extras["hybrid_astar"] = bench_hastar(ctx, world, rank, cpu=cpu_jobs)
        extras["closed_loop"] = bench_closed_loop(ctx, world, rank, cpu=cpu_jobs)
    elapsed, kern_ms, ok, K, H, fc, fields = run(a, S, ctx, dev, world, rank, a.steps, a.warmup, a.rotate,
                                                 nstreams=max(1, a.streams))
    value = world * S * K * H * a.steps / elapsed
    nbytes = algorithmic_bytes(S, K, H)
    # the device time per launch: with one stream the launch's own HIP-event span; with several the launches
    # overlap (each span covers the time it shares the device), so the timed region per step -- an upper bound
    # on the device time per launch, idle gaps included
    t_launch = kern_ms if a.streams <= 1 else elapsed / a.steps * 1e3
    achieved = nbytes / (t_launch * 1e-3) / 1e9
    out = {
        "metric": BASE["metric"],
        "value": value,
        "unit": "rollout-steps/s",
        # distinct devices the ranks ran on: a --share-device rehearsal runs every rank on cuda:0 and
        # reports 1 here (its aggregate is a one-GPU number, see "rehearsal")
        "n_gpus": len({(int(r[2]), int(r[3])) for r in joined}),
        "ranks": [{"rank": int(r[0]), "local_rank": int(r[1]), "device": int(r[2]), "pci_bus_id": int(r[3])}
                  for r in joined],
        "gpus_requested": a.gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded Philox noise drawn on device); per-scene 100x100 occupancy grids rasterised "
                "from PathPlanning/Scenarios/obstacle_field.mat fields (rescaled, tests/golden/obstacle_fields_64.npz)",
        "config": {
            "workload": f"configs[4] per-GPU shard: {S} of the 64 independent scenes per GPU (scene g: own X0 and "
                        "obstacle_field.mat field g+1), each configs[1] (MPPI K=8192 H=50 dynamic bicycle, 2-D "
                        "occupancy-grid cost, full TrajectoryCollection, weights + MPPICtrl + final rollout)",
            "obstacle_fields_rank0": fields,
            "K": K, "H": H, "scenes_per_gpu": S, "feasibility_count": fc,
            "final_rollout": "in plan kernel" if a.final_inline else
                             "side stream (final_stream=1): overlaps the next step's rollouts",
            "streams": max(1, a.streams),
            "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
            "parallelism": f"scene-sharded x{world}" + ((" + gloo all_gather(MPPICtrl), all ranks on cuda:0 "
                                                          "(--share-device rehearsal)") if a.share_device and world > 1
                                                         else " + RCCL all_gather(MPPICtrl)" if world > 1 else ""),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "kernel": "mppi_plan_kernel", "kernel_ms": kern_ms, "algorithmic_bytes": nbytes,
            "launches_in_flight": max(1, a.streams), "device_ms_per_launch": t_launch,
            "time_basis": ("kernel_ms: the mean HIP-event span of one launch (rocprofv3's average duration); "
                           "achieved divides by device_ms_per_launch = " +
                           ("kernel_ms" if a.streams <= 1 else
                            f"timed region / steps ({a.streams} launches in flight on {a.streams} streams overlap, "
                            "so one launch's span is ~that many device times per launch)")),
        },
        "valid": ok,
        # what ran before the timed region (round-4+ headlines are timed on a warm GPU, earlier
        # rounds' after the warmup steps only), and what the roofline's top-level fields price
        "order": ("extras GPU legs (iLQR, Hybrid A*, tracker, closed loop), then W warmup + K timed headline "
                  "steps, then CPU baselines") if not a.no_extras else "W warmup + K timed headline steps",
        "roofline_note": "top-level roofline fields = the bound that binds (fp64 VALU issue when the PMC "
                         "traffic file carries SQ_INSTS_VALU, else HBM); the HBM fraction is under roofline.hbm",
    }
    if a.share_device and world > 1:
        out["rehearsal"] = (f"--share-device: {world} ranks on one GPU over gloo; value is that one GPU's "
                            "aggregate, not a multi-GPU result")
    tr = load_traffic(a.traffic, S, K, H)
    if tr is not None:
        out["roofline"]["traffic"] = tr["traffic_bytes"]
        out["roofline"]["traffic_source"] = tr["source"]
        out["roofline"]["counters_note"] = ("PMC counters (FETCH_SIZE / WRITE_SIZE / SQ_*) per launch from the builder's "
                                            "rocprofv3 pass recorded in " + os.path.relpath(a.traffic, ROOT) +
                                            " (rocprofv3 cannot run inside this bench); kernel_ms is this run's "
                                            "live HIP-event time")
        if tr.get("valu_insts"):
            # the bound that binds: fp64 VALU issue.  A wave64 fp64 instruction occupies a SIMD-32
            # for 4 cycles (78.6 TF fp64 vector = 1024 SIMDs x 2.4 GHz x 16 FMA lanes x 2), so the
            # chip issues at most 1024 * 2.4e9 / 4 = 6.14e11 wave-level fp64 instructions per s.
            peak = VALU_SIMDS * VALU_CLOCK_HZ / FP64_ISSUE_CYCLES
            rate = tr["valu_insts"] / (t_launch * 1e-3)
            out["roofline"]["valu"] = {
                "insts_per_launch": tr["valu_insts"], "achieved": rate, "peak": peak, "unit": "wave-insts/s",
                "frac": rate / peak, "source": tr["source"] + " SQ_INSTS_VALU",
            }
            # the bound that binds is fp64 VALU issue: the headline fields carry it, the
            # HBM roofline (algorithmic bytes / live kernel time vs 8 TB/s) is kept beside it under "hbm"
            hbm = {k: out["roofline"][k] for k in ("achieved", "peak", "unit", "frac")}
            hbm["algorithmic_bytes"] = nbytes
            out["roofline"].update(bound="valu", achieved=rate, peak=peak, unit="wave-insts/s", frac=rate / peak,
                                   hbm=hbm)
            if tr.get("valu_active") and tr.get("wave_cycles") and tr.get("waves"):
                # measured, clock-independent: the share of each SIMD's time its waves spend issuing VALU
                # instructions = (VALU-issue quad-cycles / wave quad-cycles) x waves per SIMD
                out["roofline"]["valu"]["simd_busy"] = (tr["valu_active"] / tr["wave_cycles"]
                                                        * tr["waves"] / VALU_SIMDS)
                out["roofline"]["valu"]["simd_busy_source"] = (tr["source"] + " SQ_ACTIVE_INST_VALU / "
                                                               "SQ_WAVE_CYCLES x SQ_WAVES / 1024 SIMDs")
    if not a.no_whole and world == 1 and S < 64:
        # configs[4] whole on this one GPU: the 64 scenes in one call (the strong-scaling base of configs[4];
        # one rollout per lane, 2 waves per SIMD), 1.9 GB of TrajectoryCollection per step
        sw = max(2, a.steps // 4)
        e64, k64, ok64 = run(a, 64, ctx, dev, world, rank, sw, max(1, a.warmup // 2), 2)[:3]
        out["configs4_whole"] = {
            "workload": "configs[4] whole: all 64 scenes (obstacle_field.mat fields 1-64) in one call on one GPU",
            "value": 64 * K * H * sw / e64, "unit": "rollout-steps/s", "steps": sw, "ms_per_step": e64 / sw * 1e3,
            "kernel_ms": k64, "hbm_frac": algorithmic_bytes(64, K, H) / (k64 * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "valid": ok64,
        }
    if not a.no_single and S != 1:
        e1, k1, ok1 = run(a, 1, ctx, dev, world, rank, a.steps, a.warmup, 12, cfg5=False)[:3]
        out["single_scene"] = {
            "workload": "configs[1] exactly: one scene per GPU per step (latency-bound serial chain)",
            "value": world * K * H * a.steps / e1, "ms_per_step": e1 / a.steps * 1e3, "kernel_ms": k1,
            "roofline_frac": algorithmic_bytes(1, K, H) / (k1 * 1e-3) / 1e9 / HBM_PEAK_GBS, "valid": ok1,
        }
    if not a.no_extras:
        out.update(extras)
        rl = load_roofline(a.roofline)
        if rl:
            # the kernels of a whole mp_ilqr_solve / mp_ha_plan, ranked by their share of its kernel time
            # (tools/pmc_roofline.py legs, from solve-only / plan-only traces); the largest is the headline
            out["ilqr"]["roofline"] = leg_roofline(rl, "ilqr_solve")
            out["hybrid_astar"]["roofline"] = leg_roofline(rl, "ha_plan")
    if cpu_jobs is not None:
        for target, key, fn in cpu_jobs:  # the extras' CPU baselines, after every GPU measurement
            target[key] = fn()
        if a.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
    # the headline numbers of every leg once more at the END of the line (the driver keeps its tail)
    sm = {"mppi_rollout_steps_per_s": out["value"], "mppi_ms_per_step": out["ms_per_step"],
          "mppi_plan_kernel_ms": kern_ms}
    if "configs4_whole" in out:
        sm["configs4_whole_rollout_steps_per_s"] = out["configs4_whole"]["value"]
    if "single_scene" in out:
        sm["configs1_single_scene_rollout_steps_per_s"] = out["single_scene"]["value"]
    if "ilqr" in out:
        sm["ilqr_solve_ms"] = out["ilqr"]["solve"]["ms"]
        sm["ilqr_pass_ms"] = out["ilqr"]["ms_per_pass"]
    if "hybrid_astar" in out:
        sm["hybrid_astar_plan_ms"] = out["hybrid_astar"]["ms_total"]
        if "shards_world8" in out["hybrid_astar"]:
            sw8 = out["hybrid_astar"]["shards_world8"]
            sm["hybrid_astar_world8_projection"] = {k: sw8[k]["projected_speedup"] for k in ("contiguous", "strided") if k in sw8}
    if "closed_loop" in out:
        sm["closed_loop_ms_per_replan"] = out["closed_loop"].get("ms_per_replan")
    out["summary"] = sm
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def load_traffic(path, S, K, H):
    """roofline.traffic: HBM bytes per mppi_plan_kernel launch from a rocprofv3 --pmc run of this
    same bench command (FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected by tools/pmc_traffic.py);
    used only if that run had the same S, K, H."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    e = d.get("mppi_plan_kernel", {})
    if "traffic_bytes" not in e or d.get("config") != {"S": S, "K": K, "H": H}:
        return None
    return {"traffic_bytes": e["traffic_bytes"], "valu_insts": e.get("SQ_INSTS_VALU"),
            "valu_active": e.get("SQ_ACTIVE_INST_VALU"), "wave_cycles": e.get("SQ_WAVE_CYCLES"),
            "waves": e.get("SQ_WAVES"), "source": os.path.relpath(path, ROOT)}


def load_roofline(path):
    try:
        return json.load(open(path)) | {"path": os.path.relpath(path, ROOT)}
    except (OSError, ValueError):
        return None


def leg_roofline(rl, leg):
    """VALU roofline of one latency/VALU-bound leg: every kernel a solve-only (plan-only) rocprofv3 trace
    launched, ranked by its share of the leg's kernel time, with SQ_INSTS_VALU per launch (a --pmc pass of
    the same command) / the trace's average duration vs the fp64 VALU issue peak.  The largest kernel is
    the headline ("kernel")."""
    lg = rl.get("legs", {}).get(leg)
    if not lg or not lg.get("kernels"):
        return None
    ks = lg["kernels"]
    head = ks[0]
    return {"bound": "valu", "kernel": head["name"], "share_of_leg": head["share"],
            "achieved": head.get("valu_achieved"), "peak": rl["peak_wave_insts_per_s"], "unit": "wave-insts/s",
            "frac": head.get("valu_frac"), "traffic": None,
            "kernels": [{k: e.get(k) for k in ("name", "calls", "avg_us", "share", "SQ_INSTS_VALU", "valu_frac",
                                               "wave_valu_busy", "SQ_WAVES")} for e in ks],
            "leg_kernel_ms": lg["total_ms"], "source": rl["path"] + " legs." + leg + " (from " + lg["source"] + ")"}


def _sync_max(x, world, dev):
    if world == 1:
        return x
    return max(r[0] for r in gather_f64([x], dev))


def bench_ilqr(ctx, world, rank, cpu=None, reps=20, B=4096, N=100):
    """configs[2]: one backward Riccati sweep + one forward trial (alpha = 1) over B=4096
    initial states x H=100 knots per GPU (weak scaling), inputs resident in HBM (the _dev entry
    points).  Unit: one instance-knot of (backward + forward).  kernel_ms: the HIP-event time of
    the deriv + backward + forward kernels per pass."""
    from motionplanning_amd import ilqr
    from motionplanning_amd.abi import ptr

    dev = torch.device("cuda", torch.cuda.current_device())
    p = ilqr.params(N=N)
    x0, U = ilqr.cfg3_instances(B, N, seed=3 + rank)
    X, J = ilqr.ilqr_rollout(p, x0, U, ctx=ctx)
    dX, dU = torch.as_tensor(X, device=dev), torch.as_tensor(U, device=dev)
    dk = torch.empty((B, N - 1, 2), dtype=torch.float64, device=dev)
    dK = torch.empty((B, N - 1, 4, 2), dtype=torch.float64, device=dev)
    dXn, dUn = torch.empty_like(dX), torch.empty_like(dU)
    dJn = torch.empty(B, dtype=torch.float64, device=dev)
    dal = torch.ones(B, dtype=torch.float64, device=dev)

    def one():
        ctx.check(ctx.lib.mp_ilqr_backward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk), ptr(dK)))
        ctx.check(ctx.lib.mp_ilqr_forward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk), ptr(dK),
                                              ptr(dal), ptr(dXn), ptr(dUn), ptr(dJn)))

    one()
    torch.cuda.synchronize()
    ms, cnt = ctypes.c_double(), ctypes.c_int32()
    ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    torch.cuda.synchronize()
    el = _sync_max(time.perf_counter() - t0, world, dev)
    ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
    kms = _sync_max(ms.value / reps, world, dev)
    units = B * (N - 1)
    Jn = dJn.cpu().numpy()
    out = {"metric": "iLQR instance-knots/s (backward Riccati + forward trial), H=100, 4096 instances per GPU",
           "value": world * units * reps / el, "kernel_rate": world * units / (kms * 1e-3), "kernel_ms": kms,
           "ms_per_pass": el / reps * 1e3, "dtype": "f64", "scaling": "weak", "valid": bool(np.isfinite(Jn).all()),
           "bound": "latency (fp64 FD derivatives; serial Riccati sweep per instance)"}
    # the whole ILQR.jl loop (mp_ilqr_solve: backward + 16-wide quad line search per iteration, at most
    # 60 iterations; instances that never find a decrease stop at max_ls and are reported, not hidden)
    # on device buffers (mp_ilqr_solve_dev: the initial guess resident in HBM, solved in place; each run starts
    # from a device copy made before its timed region), like the rest of the bench
    ps = ilqr.params(N=N, max_iter=60)
    sX0, sU0 = torch.as_tensor(X, device=dev), torch.as_tensor(U, device=dev)
    sX, sU = torch.empty_like(sX0), torch.empty_like(sU0)
    sJ = torch.empty(B, dtype=torch.float64, device=dev)
    sit = torch.empty(B, dtype=torch.int32, device=dev)

    def solve():
        sX.copy_(sX0)
        sU.copy_(sU0)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        ok_ = ilqr.ilqr_solve_dev(ps, sX, sU, sJ, sit, ctx=ctx)
        return _sync_max(time.perf_counter() - t0, world, dev), ok_

    for _ in range(2):  # warm-up (workspaces, clocks: the solve time settles after ~2 solves)
        solve()
    runs = []
    for _ in range(3):  # the median of three timed solves (one solve moves +-1.5 ms with the clock ramp)
        el_, okk = solve()
        runs.append(el_)
    es = sorted(runs)[1]
    its = sit.cpu().numpy()
    out["solve"] = {"workload": f"mp_ilqr_solve_dev, {B} instances x H={N}, max_iter 60 (inputs resident in HBM)",
                    "ms": es * 1e3, "ms_runs": [r * 1e3 for r in runs],
                    "iterations_max": int(its.max()), "iterations_mean": float(its.mean()),
                    "all_converged": bool(okk)}
    def cpu_leg():
        import oracle

        def work(i):
            ko, Ko = oracle.ilqr_backward(p, X[i % B], U[i % B])
            oracle.ilqr_forward(p, X[i % B], U[i % B], ko, Ko, 1.0)
            return N - 1

        T = cpu_threads()
        u, n, dt = timed_pool(work, 3.0, T)
        return {"value": u / dt, "unit": "instance-knots/s", "cores": T, "kind": "port",
                "sample": f"{n} instances (backward + forward, H=100) in {dt:.1f} s on {T} threads, scalar C oracle"}

    defer(cpu, out, "cpu_baseline", cpu_leg)
    return out


def bench_hastar(ctx, world, rank, cpu=None):
    """configs[3]: planHybridAstar! for 256 parking scenarios (128 perpendicular + 128 parallel,
    seeded starts), sharded across ranks (strong scaling), each rank a lockstep batch search
    (per iteration one fused RS-connect + 62-neighbour expansion launch and one bookkeeping
    launch, enqueued without host round trips).  Unit: one node
    expansion (pop: RS_connected + FindNewNode over 62 primitives).  Scenarios whose open
    list empties (or that hit max_pops) end not-found exactly as the reference/oracle does;
    "found" counts the rest (tests/test_gpu_hastar.py pins the outcomes to the oracle)."""
    from motionplanning_amd import distributed as D
    from motionplanning_amd import hybrid_astar as ha

    dev = torch.device("cuda", torch.cuda.current_device())
    hs = ha.scenario_batch(256, seed=4)
    for _ in range(4):  # warm-up: same batch size (workspaces, clocks: the plan time settles after ~4 plans)
        D.hybrid_astar_sharded(ha.scenario_batch(256, seed=5), ctx=ctx)
    runs = []
    for _ in range(3):  # the median of three timed plans of the same batch
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        g = D.hybrid_astar_sharded(hs, ctx=ctx)
        runs.append(_sync_max(time.perf_counter() - t0, world, dev))
    el = sorted(runs)[1]
    pops = int(g["pops"].sum())
    out = {"metric": "Hybrid A* node expansions/s (RS_connected + 62-neighbour FindNewNode per pop), 256 scenarios",
           "value": pops / el, "neighbour_evals_per_s": pops * 62 / el, "ms_total": el * 1e3,
           "ms_runs": [r * 1e3 for r in runs],
           "scenarios": len(hs), "found": int(g["found"].sum()), "total_pops": pops, "scaling": "strong",
           "dtype": "f64", "valid": bool((g["pops"] > 0).all()),
           "bound": "latency (device-resident lockstep search, no host round trip)"}
    if world == 1:
        out["shards_world8"] = hastar_shard_projection(ctx, el)
    def cpu_leg():
        import oracle

        h0 = hs[0]
        p = ha.params_of(h0)
        sc, pc = oracle.ha_neighbor_origin(h0.s.expand_time, h0.s.steer_set, h0.s.gear_set)

        def work(i):
            h = hs[i]
            return oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc,
                                  pc)["pops"]

        T = cpu_threads()
        cp, n, dt = timed_pool(work, 3.0, T, limit=len(hs))
        return {"value": cp / dt, "unit": "node expansions/s", "cores": T, "kind": "port",
                "sample": f"{n} scenarios ({cp} pops) in {dt:.1f} s on {T} threads, scalar C oracle"}

    defer(cpu, out, "cpu_baseline", cpu_leg)
    out["tracker"] = bench_tracker(ctx, world, rank, hs, cpu=cpu)
    return out


def hastar_shard_projection(ctx, t_all, world=8):
    """The one-GPU proxy of configs[3]'s 1->8 strong scaling: each of the 8 shards a world-8 job would
    give one rank, planned alone on this GPU (median of 3), for the contiguous split (the default again
    from round 5, distributed.HA_STRIDED) and the strided one (round 4's).  The 8-GPU plan time is
    at least the slowest shard's, so T(256) / max T(shard) projects the speed-up."""
    from motionplanning_amd import distributed as D
    from motionplanning_amd import hybrid_astar as ha

    out = {"workload": f"scenario_batch(256, seed=4) split {world} ways, each shard planned alone on one GPU",
           "kind": "projection from one GPU (not a multi-GPU measurement)",
           "t256_ms": t_all * 1e3}
    for name, strided in (("contiguous", False), ("strided", True)):
        hs = ha.scenario_batch(256, seed=4)
        ms, pops = [], []
        for r in range(world):
            mine = [hs[i] for i in D.shard_indices(len(hs), r, world, strided)]
            runs = []
            for _ in range(3):
                t0 = time.perf_counter()
                ha.plan_batch(mine, ctx=ctx)
                runs.append(time.perf_counter() - t0)
            ms.append(sorted(runs)[1] * 1e3)
            pops.append(max(h.r.loop_count for h in mine))
        sp = t_all * 1e3 / max(ms)
        out[name] = {"shard_ms": ms, "shard_max_pops": pops, "projected_speedup": sp,
                     "projected_efficiency": sp / world}
    return out


def bench_tracker(ctx, world, rank, hs, cpu=None):
    """The HA* -> tracker hand-off + tracker closed loop (HybridAstar/main_Tracker.jl:42-137) for the
    scenarios this rank planned in bench_hastar: retrievePath (mp_ha_retrieve_path) then every found
    path tracked in lockstep (mp_ha_track, one wave per scenario) until its closest point is the last.
    Unit: one tracker simulation step (1 ms of simulated time: three time argmins, two findclosest
    windows, inverseKinematic, PI correction, kinematic Euler step)."""
    from motionplanning_amd import distributed as D
    from motionplanning_amd import tracker

    dev = torch.device("cuda", torch.cuda.current_device())
    D.track_sharded(hs, ctx=ctx)  # warm-up (workspaces) on the same batch
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    g = D.track_sharded(hs, ctx=ctx)
    el = _sync_max(time.perf_counter() - t0, world, dev)
    steps = int(g["n_steps"].sum())
    done = int((g["status"] == tracker.MP_TRACK_DONE).sum())
    out = {"metric": "HA* path tracker simulation steps/s (retrievePath + main_Tracker.jl loop), configs[3] paths",
           "value": steps / el, "ms_total": el * 1e3, "tracked": done,
           "no_path": int((g["status"] == tracker.MP_TRACK_NOPATH).sum()), "total_steps": steps,
           "max_steps_per_scenario": int(g["n_steps"].max()), "scaling": "strong", "dtype": "f64",
           "valid": done == int((g["status"] != tracker.MP_TRACK_NOPATH).sum()),
           "bound": "latency (one serial 1 kHz loop per scenario, one wave each)"}
    mine = [h for h in hs if h.r.tracking is not None and h.r.tracking["status"] == "done"]

    def cpu_leg():
        import oracle

        p = tracker.params_of(tracker.settings_for(mine[0]))

        def work(i):
            h = mine[i]
            return oracle.track(p, h.s.starting_real, h.r.tol_length, h.r.interp_values)["n_steps"]

        T = cpu_threads()
        cs, n, dt = timed_pool(work, 3.0, T, limit=len(mine))
        return {"value": cs / dt, "unit": "tracker steps/s", "cores": T, "kind": "port",
                "sample": f"{n} tracked paths ({cs} steps) in {dt:.1f} s on {T} threads, scalar C "
                          "oracle (full-scan argmins as the reference)"}

    if mine:
        defer(cpu, out, "cpu_baseline", cpu_leg)
    return out


def bench_closed_loop(ctx, world, rank, cpu=None, S=8, sim_s=2.0):
    """configs[4]-style multi-ego closed loop (OptimalControl/MPPI/main.jl:55-83 per scene): S scenes per
    GPU, each replanning configs[1] (K=8192, H=50, grid, device Philox) every 100 plant steps of the
    1 kHz Euler plant, for sim_s seconds of simulated time (goals out of reach: no early stop), all on
    the device (mp_mppi_closed_loop: plan kernel + plant kernel per replan, the final rollouts on the
    side stream beside the plant).  Plus the reference's own run (MPPI/main.jl exactly: one scene,
    K=1500, N=20, three circles, up to 15 s) timed end to end against the oracle's."""
    from motionplanning_amd import configs
    from motionplanning_amd.mppi import mppi_closed_loop_batch

    dev = torch.device("cuda", torch.cuda.current_device())
    c = configs.cfg2()
    p = c["params"]
    p.scene_base = rank * S
    K, H = p.K, p.H
    upd, hold = configs.mppi_hold_index(H * p.dt, H)
    steps = int(round(sim_s / configs.PLANT_DT_REF))
    X0 = np.tile(c["X0"], (S, 1))
    X0[:, 1] = np.linspace(-0.5, 0.5, S) if S > 1 else 0.0
    goal = np.tile([1e4, 0.0], (S, 1))
    grid = np.tile(c["grid"], (S, 1, 1))
    U0 = np.zeros((S, H, 2))

    def once(seed):
        p.seed = seed
        return mppi_closed_loop_batch(p, X0, goal, U0, hold, upd, steps, configs.PLANT_DT_REF, 6.0, None, grid,
                                      None, logs=False, ctx=ctx)

    once(1)  # warm-up: workspaces
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    g = once(2)
    el = _sync_max(time.perf_counter() - t0, world, dev)
    R = int(g["n_replans"].max())
    out = {"metric": "MPPI closed loop (MPPI/main.jl:55-83), S scenes x configs[1] replanned every 100 plant steps",
           "value": world * S * K * H * R / el, "unit": "rollout-steps/s (incl. plant)", "scenes_per_gpu": S,
           "replans": R, "plant_steps": steps, "ms_per_replan": el / R * 1e3, "ms_total": el * 1e3,
           "scaling": "weak", "dtype": "f64", "valid": bool((g["n_rows"] == steps + 1).all() and not g["nan"])}
    # the reference's run, whole
    pr = configs.mppi_params(K=1500, H=20, T=3.0, n_obs=3, noise_mode=1, seed=7)
    u2, h2 = configs.mppi_hold_index(3.0, 20)
    ms = int(np.floor(configs.SIM_TIME_REF / configs.PLANT_DT_REF))
    obs = np.array(configs.OBSTACLES_REF)[None]
    args = (np.array(configs.X0_REF)[None], np.array(configs.GOAL_REF)[None], np.zeros((1, 20, 2)), h2, u2, ms,
            configs.PLANT_DT_REF, configs.GOAL_RADIUS_MPPI, obs)
    mppi_closed_loop_batch(pr, *args, logs=False, ctx=ctx)
    t0 = time.perf_counter()
    gr = mppi_closed_loop_batch(pr, *args, logs=False, ctx=ctx)
    e2 = time.perf_counter() - t0
    out["reference_run"] = {"workload": "MPPI/main.jl: 1 scene, K=1500, N=20, 3 circles, 100 plant steps per "
                                        "replan, until within 6 m of the goal or 15 s",
                            "ms_total": e2 * 1e3, "replans": int(gr["n_replans"][0]),
                            "ms_per_replan": e2 / max(1, int(gr["n_replans"][0])) * 1e3,
                            "plant_rows": int(gr["n_rows"][0])}
    def cpu_leg():
        import oracle

        t0 = time.perf_counter()
        o = oracle.mppi_closed_loop(pr, args[0][0], args[1][0], args[2][0], h2, u2, ms, configs.PLANT_DT_REF,
                                    configs.GOAL_RADIUS_MPPI, obstacles=obs[0])
        e3 = time.perf_counter() - t0
        return {"ms_total": e3 * 1e3, "replans": o["n_replans"], "cores": 1, "kind": "port",
                "sample": "the same whole run (same Philox seed) on the scalar C oracle, 1 thread"}

    defer(cpu, out["reference_run"], "cpu_baseline", cpu_leg)
    return out


def defer(jobs, target, key, fn):
    """Queue a CPU baseline (target[key] = fn()) to run after every GPU measurement; jobs None: skip."""
    if jobs is not None:
        jobs.append((target, key, fn))


def cpu_threads():
    """Host threads for the CPU baselines: MPGPU_CPU_THREADS, else OMP_NUM_THREADS (16 on the GPU box,
    this job's CPU share), else min(16, cpu_count)."""
    v = os.environ.get("MPGPU_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return max(1, int(v)) if v else min(16, os.cpu_count() or 1)


def timed_pool(work, budget_s, threads, limit=None):
    """Run work(i) for i = 0, 1, ... (i < limit) on `threads` Python threads until budget_s has passed
    and return (units summed, items, seconds).  The oracle's ctypes calls release the GIL, so the
    threads run the scalar C restatement in parallel, one independent solve per call."""
    import threading

    lock = threading.Lock()
    state = {"next": 0, "units": 0, "items": 0}
    t0 = time.perf_counter()
    stop = t0 + budget_s

    def worker():
        while time.perf_counter() < stop:
            with lock:
                i = state["next"]
                if limit is not None and i >= limit:
                    return
                state["next"] = i + 1
            u = work(i)
            with lock:
                state["units"] += u
                state["items"] += 1

    ths = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return state["units"], state["items"], time.perf_counter() - t0


def cpu_baseline(budget_s):
    """The oracle (scalar C port) on the same cfg2 workload, bounded to ~budget_s: one thread for a
    third of the budget, then every host thread of this job's share (independent MPPIPlan solves
    per thread, as the GPU runs independent scenes)."""
    import oracle
    from motionplanning_amd import configs
    from motionplanning_amd.abi import MP_NOISE_PHILOX

    c = configs.cfg2(noise_mode=MP_NOISE_PHILOX)
    p0 = c["params"]

    def work(i):
        p = type(p0).from_buffer_copy(p0)  # per-call params: the Philox counter word differs
        p.offset = i
        oracle.mppi_plan(p, c["X0"], c["goal"], c["unom"], None, c["grid"], None)
        return p.K * p.H

    u1, n1, t1 = timed_pool(work, budget_s / 3, 1)
    T = cpu_threads()
    uT, nT, tT = timed_pool(work, budget_s, T)
    host = host_cpu()
    out = {"value": uT / tT, "unit": "rollout-steps/s", "cores": T, "kind": "port", "host": host,
           "sample": f"{nT} full cfg2 MPPIPlan solves (K=8192, H=50, grid, Philox noise) in {tT:.1f} s on {T} "
                     f"threads (one solve per thread at a time), scalar C oracle, {os.cpu_count()}-CPU host",
           "single_thread": {"value": u1 / t1, "cores": 1, "sample": f"{n1} solves in {t1:.1f} s"},
           "why_these_threads": "the GPU pool gives each one-GPU job a 16-CPU share of the host (it sets "
                                "OMP_NUM_THREADS=16 and asks worker pools to stay within it); the other CPUs of "
                                "the affinity set belong to the other GPUs' jobs, so they are not timed"}
    # all cores of the affinity set: the solves are independent, so the measured per-thread
    # rate at T threads scaled to every usable CPU is an upper bound on what the whole host would give
    n_all = host["usable_cpus"] or T
    out["all_cores_projection"] = {"value": uT / tT / T * n_all, "cores": n_all, "kind": "projected",
                                   "basis": f"measured {uT / tT / T:.4g} rollout-steps/s per thread at {T} threads "
                                            f"x {n_all} usable CPUs (linear: no shared state between solves)"}
    return out


if __name__ == "__main__":
    main()
