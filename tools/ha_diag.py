"""Dump GPU vs oracle RS_connected paths for random nodes (debug aid)."""
import ctypes
import faulthandler

import numpy as np

faulthandler.dump_traceback_later(100, exit=True)
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.abi import ptr
from motionplanning_amd.context import default_context

ctx = default_context(0)
h = ha.driver_searcher(ha.PERPENDICULAR)
p = ha.params_of(h)
walls = np.array(h.s.obstacle_list)
r = np.random.default_rng(1)
B = 64
nodes = np.c_[r.choice(np.arange(-5, 10.01, 0.5), B), r.choice(np.arange(0, 10.01, 0.5), B),
              r.integers(-12, 13, B) * np.pi / 12]
goal = np.tile(h.s.ending_states, (B, 1))
W = np.tile(walls, (B, 1, 1))
ok, path, ln = np.zeros(B, np.uint8), np.zeros((B, 501, 3)), np.zeros(B, np.int32)
ctx.check(ctx.lib.mp_ha_rs_connect(ctx.handle, ctypes.byref(p), B, ptr(nodes), ptr(goal), ptr(W), ptr(ok), ptr(path), ptr(ln)))
np.savez("gpurun_out/ha_rs.npz", nodes=nodes, ok=ok, path=path, ln=ln)
print("saved")
