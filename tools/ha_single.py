"""Per-iteration latency of the device-resident Hybrid A* loop for small batches (the tail regime of
configs[3], where few scenarios are still searching): plan B copies of a driver scene a few times."""
import sys
import time

sys.path.insert(0, ".")
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd.context import default_context

ctx = default_context(0)
for B in (1, 8, 64, 256):
    hs = [ha.driver_searcher(ha.PERPENDICULAR) for _ in range(B)]
    ha.plan_batch(hs, ctx=ctx)
    best = 1e9
    for rep in range(3):
        t0 = time.perf_counter()
        ha.plan_batch(hs, ctx=ctx)
        best = min(best, time.perf_counter() - t0)
    it = hs[0].r.loop_count
    print(f"B={B:4d} (perpendicular driver scene x B): {best * 1e3:.2f} ms for {it} iterations = "
          f"{best * 1e6 / it:.1f} us per iteration", flush=True)
