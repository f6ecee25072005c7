"""Repeat test_gpu_hastar's lockstep batch check and name the scenarios that differ from the oracle (where their
pop sequence first diverges), to chase a run-to-run difference.

  python tools/ha_batch_check.py [n] [seed] [repeats] [--pre]
  --pre: plan the two driver scenes first (the order of tests/test_gpu_hastar.py)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from motionplanning_amd import hybrid_astar as ha  # noqa: E402
from motionplanning_amd.context import Context  # noqa: E402


def main():
    av = [x for x in sys.argv[1:] if not x.startswith('--')]
    n = int(av[0]) if len(av) > 0 else 32
    seed = int(av[1]) if len(av) > 1 else 4
    reps = int(av[2]) if len(av) > 2 else 3
    ctx = Context(0)
    if "--pre" in sys.argv:
        for scene in (ha.PERPENDICULAR, ha.PARALLEL):
            h = ha.driver_searcher(scene)
            ha.install_primitives(h, ctx)
            ha.planHybridAstar_(h, ctx=ctx)
            print(f"driver scene: {h.r.loop_count} pops", flush=True)
    h0 = ha.driver_searcher(ha.PERPENDICULAR)
    p = ha.params_of(h0)
    sc, pc = ha.install_primitives(h0, ctx)
    refs = None
    for rep in range(reps):
        hs = ha.scenario_batch(n, seed=seed)
        if refs is None:
            refs = [oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
                    for h in hs]
        ha.plan_batch(hs, ctx=ctx)
        bad = []
        for i, (h, ref) in enumerate(zip(hs, refs)):
            ps, rs = np.asarray(h.r.pop_sequence), np.asarray(ref["pop_seq"])
            same = (h.r.found == ref["found"] and h.r.loop_count == ref["pops"] and h.r.n_nodes == ref["n_nodes"]
                    and np.array_equal(ps, rs) and np.array_equal(h.r.hybrid_astar_states.T, ref["states"])
                    and np.array_equal(h.r.RSpath_final.T, ref["rs_path"]))
            if not same:
                m = min(len(ps), len(rs))
                d = np.nonzero(ps[:m] != rs[:m])[0]
                bad.append((i, int(h.r.loop_count), int(ref["pops"]), int(d[0]) if len(d) else -1,
                            bool(h.r.found), bool(ref["found"])))
        print(f"rep {rep}: {len(bad)} of {n} differ" + "".join(
            f"\n  scenario {i}: pops {a} (oracle {b}), first divergence at pop {d}, found {f} (oracle {g})"
            for i, a, b, d, f, g in bad), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
