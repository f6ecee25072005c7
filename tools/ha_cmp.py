"""Debug aid: mismatching Hybrid A* heuristics / allpath costs, GPU vs oracle."""
import ctypes
import math
import sys

import numpy as np

sys.path.insert(0, ".")
import oracle
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.abi import ptr
from motionplanning_amd.context import default_context

ctx = default_context(0)
h = ha.driver_searcher(ha.PERPENDICULAR)
p = ha.params_of(h)
sc, pc = ha.install_primitives(h, ctx)
walls = np.array(h.s.obstacle_list)
r = np.random.default_rng(1)
B = 64
nodes = np.c_[r.choice(np.arange(-5, 10.01, 0.5), B), r.choice(np.arange(0, 10.01, 0.5), B),
              r.integers(-12, 13, B) * np.pi / 12]
goal = np.tile(h.s.ending_states, (B, 1))
W = np.tile(walls, (B, 1, 1))
nb, idx = np.zeros((B, 62, 3)), np.zeros((B, 62), np.int64)
fr, hh = np.zeros((B, 62), np.uint8), np.zeros((B, 62))
ctx.check(ctx.lib.mp_ha_expand(ctx.handle, ctypes.byref(p), B, ptr(nodes), ptr(goal), ptr(W), ptr(nb), ptr(idx),
                               ptr(fr), ptr(hh)))
bad = []
for b in range(B):
    nbo, idxo, fro, ho = oracle.ha_expand(p, nodes[b], goal[b], walls, sc, pc)
    for k in range(62):
        if fro[k] and hh[b, k] != ho[k]:
            bad.append((b, k, hh[b, k], ho[k], nbo[k]))
print("mismatches", len(bad))
for t in bad[:5]:
    print(t)
# allpath on the normalised states of the mismatching neighbours
ns = []
for b, k, _, _, st in bad[:50]:
    g = goal[b]
    dx, dy = (g[0] - st[0]) / p.minR, (g[1] - st[1]) / p.minR
    c, s = oracle.m("cos", st[2]), oracle.m("sin", st[2])
    ns.append([dx * c + dy * s, -dx * s + dy * c, g[2] - st[2]])
if ns:
    best, cost, cmds = ha.allpath(np.array(ns), ctx=ctx)
    for i in range(len(ns)):
        bo, co, mo = oracle.ha_allpath(ns[i])
        d = np.nonzero(~((cost[i] == co) | (np.isnan(cost[i]) & np.isnan(co))))[0]
        if len(d):
            print("allpath diff state", ns[i], "candidates", d[:8], cost[i][d[:4]], co[d[:4]])
