"""Time the HA* -> tracker hand-off + tracker loop (mp_ha_track) on configs[3]'s planned paths:
plan 256 scenarios, retrieve, then track a few times (kernel time by HIP events)."""
import ctypes
import sys
import time

sys.path.insert(0, ".")
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd import tracker
from motionplanning_amd.context import default_context

ctx = default_context(0)
hs = ha.scenario_batch(256, seed=4)
ha.plan_batch(hs, ctx=ctx)
ha.retrieve_batch(hs, ctx=ctx)
ctx.lib.mp_ctx_kernel_timing(ctx.handle, 1)
ms, cnt = ctypes.c_double(), ctypes.c_int32()
for rep in range(3):
    t0 = time.perf_counter()
    tracker.track_batch(hs, ctx=ctx)
    el = time.perf_counter() - t0
    ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
    steps = [h.r.tracking["n_steps"] for h in hs]
    print(f"track 256: {el * 1e3:.1f} ms wall, kernel {ms.value:.1f} ms, steps {sum(steps)}, max {max(steps)}, "
          f"{ms.value * 1e3 / max(steps):.2f} us per step of the longest scenario", flush=True)
