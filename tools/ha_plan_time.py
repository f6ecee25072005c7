"""Time mp_ha_plan on configs[3] (256 scenarios) a few times: the whole plan_batch call and the library
call inside it (r.planning_time); with MPGPU_HA_PROFILE=1 the library prints its host pop /
launch+kernel+copies / bookkeeping split per plan."""
import sys
import time

sys.path.insert(0, ".")
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.context import default_context

ctx = default_context(0)
ha.plan_batch(ha.scenario_batch(4, seed=5), ctx=ctx)
hs = ha.scenario_batch(256, seed=4)
for rep in range(5):
    t0 = time.perf_counter()
    ha.plan_batch(hs, ctx=ctx)
    el = time.perf_counter() - t0
    pops = [h.r.loop_count for h in hs]
    print(f"plan 256: {el * 1e3:.1f} ms (library call {hs[0].r.planning_time * 1e3:.1f} ms), pops {sum(pops)}, "
          f"max pops {max(pops)}, found {sum(h.r.found for h in hs)}", flush=True)
