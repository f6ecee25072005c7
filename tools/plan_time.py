"""Plan-kernel time (HIP events, mp_ctx_kernel_ms) of mppi_plan_kernel for a grid of scene counts and
lane layouts (the MPGPU_LPR test hook), configs[1] scenes with device Philox noise and the full
TrajectoryCollection, as bench.py runs them.

  python tools/plan_time.py [--scenes 8 16] [--lpr 1 2] [--reps 20]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, nargs="+", default=[8, 16])
    ap.add_argument("--lpr", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from motionplanning_amd import configs
    from motionplanning_amd.abi import MP_NOISE_PHILOX, ptr
    from motionplanning_amd.context import Context

    dev = torch.device("cuda", 0)
    ctx = Context(0)
    ctx.lib.mp_ctx_kernel_timing(ctx.handle, 1)
    c = configs.cfg2(noise_mode=MP_NOISE_PHILOX)
    p = c["params"]
    p.final_stream = 1
    K, H = p.K, p.H
    for S in a.scenes:
        t = lambda x, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(x), dtype=dt, device=dev)
        X0 = t(np.tile(c["X0"], (S, 1)))
        goal = t(np.tile(c["goal"], (S, 1)))
        un = t(np.zeros((S, H, 2)))
        grid = t(np.tile(c["grid"], (S, 1, 1)), torch.uint8)
        o = {k: torch.empty(v, dtype=dt, device=dev) for k, (v, dt) in dict(
            U=((S, H, 2), torch.float64), traj=((S, H + 1, 7), torch.float64), cost=((S,), torch.float64),
            fe=((S,), torch.int32), rc=((S,), torch.int32), fc=((S,), torch.int32),
            ct=((S, H + 1, 7, K), torch.float64), cc=((S, H, K, 2), torch.float64), ck=((S, K), torch.float64),
            cf=((S, K), torch.uint8)).items()}
        for lpr in a.lpr:
            os.environ["MPGPU_LPR"] = str(lpr)
            ms, cnt = ctypes.c_double(), ctypes.c_int32()
            for i in range(a.reps + 3):
                p.offset = i
                ctx.check(ctx.lib.mp_mppi_plan_dev(ctx.handle, ctypes.byref(p), S, ptr(X0), ptr(goal), ptr(un),
                                                   None, ptr(grid), None, ptr(o["U"]), ptr(o["traj"]),
                                                   ptr(o["cost"]), ptr(o["fe"]), ptr(o["rc"]), ptr(o["fc"]),
                                                   ptr(o["ct"]), ptr(o["cc"]), ptr(o["ck"]), ptr(o["cf"])))
                if i == 2:
                    torch.cuda.synchronize()
                    ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            torch.cuda.synchronize()
            ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            kms = ms.value / max(1, cnt.value)
            print(f"S={S:3d} LPR={lpr}  kernel {kms * 1e3:8.1f} us  "
                  f"{S * K * H / (kms * 1e-3):.3e} rollout-steps/s", flush=True)


if __name__ == "__main__":
    main()
