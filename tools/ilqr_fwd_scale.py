"""Forward-trial kernel time vs occupancy: mp_ilqr_forward_dev (one quad-lane trial per instance) at
B = 4096 / 16384 / 65536 instances x H=100 (0.25 / 1 / 4 waves per SIMD), to separate the trial's
latency from its throughput limit (compare the line-search round 0 at 4 waves per SIMD)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from motionplanning_amd import ilqr
from motionplanning_amd.abi import ptr
from motionplanning_amd.context import default_context

ctx = default_context(0)
ctx.lib.mp_ctx_kernel_timing(ctx.handle, 1)
dev = torch.device("cuda", 0)
N, reps = 100, 10
p = ilqr.params(N=N)
x0, U = ilqr.cfg3_instances(4096, N, seed=3)
X, _ = ilqr.ilqr_rollout(p, x0, U, ctx=ctx)
stream = torch.cuda.ExternalStream(ctx.stream, device=dev)
with torch.cuda.stream(stream):
    for rep in (1, 4, 16):
        B = 4096 * rep
        dX = torch.as_tensor(np.tile(X, (rep, 1, 1)), device=dev)
        dU = torch.as_tensor(np.tile(U, (rep, 1, 1)), device=dev)
        dk = torch.empty((B, N - 1, 2), dtype=torch.float64, device=dev)
        dK = torch.empty((B, N - 1, 4, 2), dtype=torch.float64, device=dev)
        ctx.check(ctx.lib.mp_ilqr_backward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk), ptr(dK)))
        dXn, dUn = torch.empty_like(dX), torch.empty_like(dU)
        dJn = torch.empty(B, dtype=torch.float64, device=dev)
        dal = torch.ones(B, dtype=torch.float64, device=dev)
        ms, cnt = ctypes.c_double(), ctypes.c_int32()
        for label, a in (("alpha 1", 1.0), ("alpha 2^-(b%16)", None)):
            if a is None:
                dal.copy_(torch.ldexp(torch.ones(B, dtype=torch.float64), -(torch.arange(B) % 16)))
            ctx.synchronize()
            ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            for _ in range(reps):
                ctx.check(ctx.lib.mp_ilqr_forward_dev(ctx.handle, ctypes.byref(p), B, ptr(dX), ptr(dU), ptr(dk), ptr(dK),
                                                      ptr(dal), ptr(dXn), ptr(dUn), ptr(dJn)))
            ctx.synchronize()
            ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
            print(f"B={B:6d} ({B * 4 // 64 / 1024:.2f} waves/SIMD) {label}: forward {ms.value / reps * 1e3:.1f} us",
                  flush=True)
