"""Time mp_ha_plan on configs[3] (256 scenarios) a few times: the whole plan_batch call and the library
call inside it (r.planning_time).  --shards: also the one-GPU world-8 projection of
bench.py (each strided / contiguous shard planned alone, median of 3; a projection, not a multi-GPU run)."""
import sys
import time

sys.path.insert(0, ".")
from motionplanning_amd import distributed as D
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.context import default_context

ctx = default_context(0)
ha.plan_batch(ha.scenario_batch(4, seed=5), ctx=ctx)
hs = ha.scenario_batch(256, seed=4)
els = []
for rep in range(5):
    t0 = time.perf_counter()
    ha.plan_batch(hs, ctx=ctx)
    el = time.perf_counter() - t0
    els.append(el)
    pops = [h.r.loop_count for h in hs]
    print(f"plan 256: {el * 1e3:.1f} ms (library call {hs[0].r.planning_time * 1e3:.1f} ms), pops {sum(pops)}, "
          f"max pops {max(pops)}, found {sum(h.r.found for h in hs)}", flush=True)
print("scenes still searching after iteration k: " + " ".join(
    f"{k}:{sum(p > k for p in pops)}" for k in (50, 100, 200, 300, 400, 500, 600, 700)), flush=True)
if "--shards" in sys.argv:
    t_all = sorted(els)[len(els) // 2]
    for name, strided in (("contiguous", False), ("strided", True)):
        ms = []
        hs8 = ha.scenario_batch(256, seed=4)
        for r in range(8):
            mine = [hs8[i] for i in D.shard_indices(256, r, 8, strided)]
            runs = []
            for _ in range(3):
                t0 = time.perf_counter()
                ha.plan_batch(mine, ctx=ctx)
                runs.append(time.perf_counter() - t0)
            ms.append(sorted(runs)[1] * 1e3)
        print(f"world-8 projection ({name}): shards " + " ".join(f"{m:.1f}" for m in ms) +
              f" ms, projected speed-up {t_all * 1e3 / max(ms):.2f}x", flush=True)
