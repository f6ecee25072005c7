"""Lone-scene Hybrid A* latency: the longest search of configs[3]'s batch (scenario_batch(256, seed=4), 729
pops) planned alone (B = 1) -- what bounds every world-8 shard holding it -- and a 32-scenario strided shard
holding it.  Prints ms per plan and us per search iteration (median of 5)."""
import sys
import time

sys.path.insert(0, ".")
from motionplanning_amd import distributed as D
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.context import default_context

ctx = default_context(0)
hs = ha.scenario_batch(256, seed=4)
ha.plan_batch(hs, ctx=ctx)
pops = [h.r.loop_count for h in hs]
i_max = max(range(len(hs)), key=lambda i: pops[i])
reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5


def timed(batch):
    runs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ha.plan_batch(batch, ctx=ctx)
        runs.append(time.perf_counter() - t0)
    return sorted(runs)[len(runs) // 2]


lone = [ha.scenario_batch(256, seed=4)[i_max]]
t = timed(lone)
it = lone[0].r.loop_count
print(f"lone scenario {i_max}: {t * 1e3:.2f} ms for {it} pops = {t * 1e6 / it:.1f} us per iteration "
      f"(library call {lone[0].r.planning_time * 1e3:.2f} ms)", flush=True)
for strided in (() if '--lone-only' in sys.argv else (True,)):
    hs8 = ha.scenario_batch(256, seed=4)
    for r in range(8):
        idx = D.shard_indices(256, r, 8, strided)
        if i_max in idx:
            mine = [hs8[i] for i in idx]
            t = timed(mine)
            print(f"strided shard {r} ({len(mine)} scenarios, holds {i_max}): {t * 1e3:.2f} ms = "
                  f"{t * 1e6 / max(h.r.loop_count for h in mine):.1f} us per iteration", flush=True)
