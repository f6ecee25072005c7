"""Time the iLQR device passes at configs[2] (B=4096, N=100): backward (deriv + Riccati) and
forward trial on HBM-resident inputs, plus a full mp_ilqr_solve.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from motionplanning_amd import ilqr
from motionplanning_amd.abi import ptr
from motionplanning_amd.context import default_context

B, N, reps = 4096, 100, 20
solve_only = "--solve-only" in sys.argv
ctx = default_context(0)
ctx.lib.mp_ctx_kernel_timing(ctx.handle, 1)
dev = torch.device("cuda", 0)
p = ilqr.params(N=N)
x0, U = ilqr.cfg3_instances(B, N, seed=3)
X, J = ilqr.ilqr_rollout(p, x0, U, ctx=ctx)
stream = torch.cuda.ExternalStream(ctx.stream, device=dev)
with torch.cuda.stream(stream):
    dX, dU = torch.as_tensor(X, device=dev), torch.as_tensor(U, device=dev)
    dk = torch.empty((B, N - 1, 2), dtype=torch.float64, device=dev)
    dK = torch.empty((B, N - 1, 4, 2), dtype=torch.float64, device=dev)
    dXn, dUn = torch.empty_like(dX), torch.empty_like(dU)
    dJn = torch.empty(B, dtype=torch.float64, device=dev)
    dal = torch.ones(B, dtype=torch.float64, device=dev)
    ctx.synchronize()
    ms, cnt = ctypes.c_double(), ctypes.c_int32()
    for name, fn in () if solve_only else (
        ("backward", lambda: ctx.lib.mp_ilqr_backward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk),
                                                          ptr(dK))),
        ("forward", lambda: ctx.lib.mp_ilqr_forward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk),
                                                        ptr(dK), ptr(dal), ptr(dXn), ptr(dUn), ptr(dJn))),
    ):
        ctx.check(fn())
        ctx.synchronize()
        ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.check(fn())
        ctx.synchronize()
        el = (time.perf_counter() - t0) / reps
        ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
        print(f"{name}: {el * 1e3:.3f} ms wall, {ms.value / reps:.3f} ms kernel", flush=True)
    if "--alpha-mix" in sys.argv:  # forward trial cost vs the spread of alpha inside a wave (16 instances)
        for label, a in (("alpha 1", torch.ones(B, dtype=torch.float64)),
                         ("alpha 2^-(b%16)", torch.ldexp(torch.ones(B, dtype=torch.float64), -(torch.arange(B) % 16))),
                         ("alpha 2^-(b/256)", torch.ldexp(torch.ones(B, dtype=torch.float64), -(torch.arange(B) // 256))),
                         ("alpha 2^-20", torch.full((B,), 2.0 ** -20, dtype=torch.float64))):
            dal.copy_(a)
            ctx.synchronize()
            ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            for _ in range(reps):
                ctx.check(ctx.lib.mp_ilqr_forward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk), ptr(dK),
                                                      ptr(dal), ptr(dXn), ptr(dUn), ptr(dJn)))
            ctx.synchronize()
            ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            print(f"forward {label}: {ms.value / reps:.3f} ms kernel", flush=True)
for rep in range(int(sys.argv[sys.argv.index("--solve-reps") + 1]) if "--solve-reps" in sys.argv else 1):  # (the first includes workspace allocation)
    t0 = time.perf_counter()
    Xs, Us, Js, it, ok = ilqr.ilqr_solve(ilqr.params(N=N, max_iter=60), X, U, ctx=ctx)
    print(f"solve: {(time.perf_counter() - t0) * 1e3:.1f} ms, iterations max {it.max()} mean {it.mean():.1f}, ok {ok}",
          flush=True)
