"""Time the Hybrid A* device parts separately (mp_ha_expand / mp_ha_rs_connect) at batch B."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.abi import ptr
from motionplanning_amd.context import default_context

ctx = default_context(0)
ctx.lib.mp_ctx_kernel_timing(ctx.handle, 1)
h = ha.driver_searcher(ha.PERPENDICULAR)
p = ha.params_of(h)
ha.install_primitives(h, ctx)
walls = np.array(h.s.obstacle_list)
for B in (1, 16, 256):
    r = np.random.default_rng(1)
    nodes = np.c_[r.choice(np.arange(-5, 10.01, 0.5), B), r.choice(np.arange(0, 10.01, 0.5), B),
                  r.integers(-12, 13, B) * np.pi / 12]
    goal = np.tile(h.s.ending_states, (B, 1))
    W = np.tile(walls, (B, 1, 1))
    nb, idx = np.zeros((B, 62, 3)), np.zeros((B, 62), np.int64)
    fr, hh = np.zeros((B, 62), np.uint8), np.zeros((B, 62))
    ok, path, ln = np.zeros(B, np.uint8), np.zeros((B, 501, 3)), np.zeros(B, np.int32)
    ms, cnt = ctypes.c_double(), ctypes.c_int32()
    for what in ("expand", "rs"):
        for rep in range(4):
            if what == "expand":
                ctx.check(ctx.lib.mp_ha_expand(ctx.handle, ctypes.byref(p), B, ptr(nodes), ptr(goal), ptr(W), ptr(nb),
                                               ptr(idx), ptr(fr), ptr(hh)))
            else:
                ctx.check(ctx.lib.mp_ha_rs_connect(ctx.handle, ctypes.byref(p), B, ptr(nodes), ptr(goal), ptr(W),
                                                   ptr(ok), ptr(path), ptr(ln)))
            ctx.check(ctx.lib.mp_ctx_kernel_ms(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt)))
        print(f"B={B:4d} {what:6s} kernel {ms.value * 1e3:9.1f} us", flush=True)
    print(f"B={B:4d} free neighbours {fr.mean():.3f} of 62 per node; groups with any free "
          f"{np.mean([fr[b, g * 16:(g + 1) * 16].any() for b in range(B) for g in range(4)]):.3f}", flush=True)
