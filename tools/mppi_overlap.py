"""Consecutive independent MPPI plan calls overlapped on several contexts (streams) of one GPU
(the straggler window of a lone launch).  The bench workload (configs[4]'s 8-scene
shard, device Philox noise, full TrajectoryCollection, final rollout on the side stream); call i runs on
context i mod C.  Prints rollout-steps/s per (contexts, lane layout).

  python tools/mppi_overlap.py [--ctx 1 2] [--lpr 0 1 2] [--steps 200] [--warmup 40] [--timing]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--lpr", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--scenes", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--final", type=int, nargs="+", default=[1], help="final_stream values to try (0: inline)")
    ap.add_argument("--timing", action="store_true", help="per-launch HIP-event timing on (as bench.py)")
    a = ap.parse_args()
    from motionplanning_amd import configs
    from motionplanning_amd.abi import MP_NOISE_PHILOX, ptr
    from motionplanning_amd.context import Context

    dev = torch.device("cuda", 0)
    S = a.scenes
    c = configs.cfg5_shard(0, S, noise_mode=MP_NOISE_PHILOX, seed=20260415)
    p = c["params"]
    K, H = p.K, p.H
    t = lambda x, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(x), dtype=dt, device=dev)
    X0, goal, un, grid = t(c["X0"]), t(c["goal"]), t(np.zeros((S, H, 2))), t(c["grid"], torch.uint8)
    ctxs = [Context(0) for _ in range(max(a.ctx))]
    for x in ctxs:
        x.lib.mp_ctx_kernel_timing(x.handle, 1 if a.timing else 0)
    sets = []
    for _ in range(3 * max(a.ctx)):
        sets.append({k: torch.empty(v, dtype=dt, device=dev) for k, (v, dt) in dict(
            U=((S, H, 2), torch.float64), traj=((S, H + 1, 7), torch.float64), cost=((S,), torch.float64),
            fe=((S,), torch.int32), rc=((S,), torch.int32), fc=((S,), torch.int32),
            ct=((S, H + 1, 7, K), torch.float64), cc=((S, H, K, 2), torch.float64), ck=((S, K), torch.float64),
            cf=((S, K), torch.uint8)).items()})

    def step(i, C):
        ctx = ctxs[i % C]
        o = sets[i % len(sets)]
        p.offset = i
        ctx.check(ctx.lib.mp_mppi_plan_dev(ctx.handle, ctypes.byref(p), S, ptr(X0), ptr(goal), ptr(un), None,
                                           ptr(grid), None, ptr(o["U"]), ptr(o["traj"]), ptr(o["cost"]), ptr(o["fe"]),
                                           ptr(o["rc"]), ptr(o["fc"]), ptr(o["ct"]), ptr(o["cc"]), ptr(o["ck"]),
                                           ptr(o["cf"])))

    def sync():
        for x in ctxs:
            x.synchronize()
        torch.cuda.synchronize()

    for rep in range(a.reps):
        for C in a.ctx:
          p.calls_in_flight = C
          for fs in a.final:
            p.final_stream = fs
            for lpr in a.lpr:
                if lpr:
                    os.environ["MPGPU_LPR"] = str(lpr)
                else:
                    os.environ.pop("MPGPU_LPR", None)
                for i in range(a.warmup):
                    step(i, C)
                sync()
                t0 = time.perf_counter()
                for i in range(a.steps):
                    step(a.warmup + i, C)
                sync()
                el = time.perf_counter() - t0
                ok = all(bool((o["rc"] == K + 1).all().item()) for o in sets)
                print(f"rep {rep} contexts {C} final_stream {fs} lpr {lpr or 'auto'}: {S * K * H * a.steps / el:.4e} rollout-steps/s, "
                      f"{el / a.steps * 1e3:.4f} ms/step, valid {ok}", flush=True)
    os.environ.pop("MPGPU_LPR", None)


if __name__ == "__main__":
    main()
