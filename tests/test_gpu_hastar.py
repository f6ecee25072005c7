"""GPU parity for the Hybrid A* hot path (mp_ha_*) vs the CPU oracle — BIT-EXACT discrete
outputs (Encode indices, collision booleans, heuristics, pop order, node counts, paths).
Parity against Julia itself is unpinned (no reference artifact)."""
import numpy as np
import pytest

import oracle
from motionplanning_amd import hybrid_astar as ha

pytestmark = pytest.mark.gpu


def _setup(ctx, scene=ha.PERPENDICULAR):
    h = ha.driver_searcher(scene)
    p = ha.params_of(h)
    sc, pc = ha.install_primitives(h, ctx)
    sco, pco = oracle.ha_neighbor_origin(h.s.expand_time, h.s.steer_set, h.s.gear_set)
    assert np.array_equal(sc, sco) and np.array_equal(pc, pco)
    return h, p, sc, pc


def test_expand_and_rs_connect_bitexact(ctx):
    import ctypes

    from motionplanning_amd.abi import ptr

    h, p, sc, pc = _setup(ctx)
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
    ok, path, ln = np.zeros(B, np.uint8), np.zeros((B, 501, 3)), np.zeros(B, np.int32)
    ctx.check(ctx.lib.mp_ha_rs_connect(ctx.handle, ctypes.byref(p), B, ptr(nodes), ptr(goal), ptr(W), ptr(ok),
                                       ptr(path), ptr(ln)))
    n_free = 0
    for b in range(B):
        nbo, idxo, fro, ho = oracle.ha_expand(p, nodes[b], goal[b], walls, sc, pc)
        assert np.array_equal(nb[b], nbo) and np.array_equal(idx[b], idxo) and np.array_equal(fr[b], fro)
        assert np.array_equal(hh[b][fro == 1], ho[fro == 1])
        n_free += int(fro.sum())
        oko, patho = oracle.ha_rs_connect(p, nodes[b], goal[b], walls)
        assert bool(ok[b]) == oko and ln[b] == len(patho)
        assert np.array_equal(path[b, : ln[b]], patho)
    assert 0 < n_free < B * 62  # both branches exercised


@pytest.mark.parametrize("scene,pops", [(ha.PERPENDICULAR, 275), (ha.PARALLEL, 120)])
def test_driver_scene_plan_bitexact(ctx, scene, pops):
    h, p, sc, pc = _setup(ctx, scene)
    ha.planHybridAstar_(h, ctx=ctx)
    ref = oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
    assert h.r.found and ref["found"] and h.r.loop_count == ref["pops"] == pops
    assert h.r.n_nodes == ref["n_nodes"]
    assert np.array_equal(h.r.pop_sequence, ref["pop_seq"])  # expanded-node set, in pop order
    assert np.array_equal(h.r.hybrid_astar_states.T, ref["states"])
    assert np.array_equal(h.r.RSpath_final.T, ref["rs_path"])


@pytest.mark.parametrize("n,seed", [(32, 4), (96, 11)])
def test_scenario_batch_lockstep_bitexact(ctx, n, seed):
    """BASELINE cfg4 shape (perpendicular + parallel scenarios, seeded starts) in lockstep: found flag, pop
    count, node count and the full pop sequence identical to the oracle's sort-every-iteration open list."""
    hs = ha.scenario_batch(n, seed=seed)
    _, p, sc, pc = _setup(ctx)
    ha.plan_batch(hs, ctx=ctx)
    bad = []
    for i, h in enumerate(hs):
        ref = oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
        same = (h.r.found == ref["found"] and h.r.loop_count == ref["pops"] and h.r.n_nodes == ref["n_nodes"]
                and np.array_equal(h.r.pop_sequence, ref["pop_seq"])
                and np.array_equal(h.r.hybrid_astar_states.T, ref["states"])
                and np.array_equal(h.r.RSpath_final.T, ref["rs_path"]))
        if not same:
            ps, rs = np.asarray(h.r.pop_sequence), np.asarray(ref["pop_seq"])
            m = min(len(ps), len(rs))
            d = np.nonzero(ps[:m] != rs[:m])[0]
            bad.append((i, int(h.r.loop_count), int(ref["pops"]), int(d[0]) if len(d) else -1))
    assert not bad, f"scenarios differing (index, pops, oracle pops, first divergent pop): {bad}"


def test_pipelined_tail_without_persistent_launch_bitexact(ctx):
    """The per-iteration pipelined tail (ha_pipe_kernel, the path a device without cooperative launches
    takes, or a refused cooperative launch falls back to; MPGPU_HA_PERSIST=0 selects it): bit-exact, and its
    bounded cross-block waits report through the same error flag the persistent tail's do (mp_ha_plan
    checks it after any pipelined launch and fails loudly)."""
    import os
    hs = ha.scenario_batch(12, seed=4) + [ha.driver_searcher(ha.PERPENDICULAR), ha.driver_searcher(ha.PARALLEL)]
    _, p, sc, pc = _setup(ctx)
    os.environ["MPGPU_HA_PERSIST"] = "0"
    try:
        ha.plan_batch(hs, ctx=ctx)
    finally:
        del os.environ["MPGPU_HA_PERSIST"]
    for h in hs:
        ref = oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
        assert h.r.found == ref["found"] and h.r.loop_count == ref["pops"] and h.r.n_nodes == ref["n_nodes"]
        assert np.array_equal(h.r.pop_sequence, ref["pop_seq"])
        assert np.array_equal(h.r.hybrid_astar_states.T, ref["states"])
        assert np.array_equal(h.r.RSpath_final.T, ref["rs_path"])


@pytest.mark.parametrize("max_pops", [1, 7, 40])
def test_max_pops_and_out_of_bounds_start_bitexact(ctx, max_pops):
    """Device-resident search edge cases vs the oracle: the max_pops stop (pop_seq truncated,
    not found), a start outside stbound (Encode 0 -> the start node sits in cell 0), and a start
    on the lattice boundary, in one lockstep batch with ordinary scenes."""
    hs = ha.scenario_batch(6, seed=9)
    hs.append(ha.driver_searcher(ha.PERPENDICULAR, [11.0, 4.0, ha.PI / 2]))   # x > stbound: Encode 0
    hs.append(ha.driver_searcher(ha.PARALLEL, [10.0, 10.0, -ha.PI / 2]))    # corner of the lattice
    _, p, sc, pc = _setup(ctx)
    ha.plan_batch(hs, ctx=ctx, max_pops=max_pops)
    q = ha.params_of(hs[0], max_pops)
    for h in hs:
        ref = oracle.ha_plan(q, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
        assert h.r.loop_count == ref["pops"] <= max_pops
        assert h.r.found == ref["found"] and h.r.n_nodes == ref["n_nodes"]
        assert np.array_equal(h.r.pop_sequence, ref["pop_seq"])
        assert np.array_equal(h.r.hybrid_astar_states.T, ref["states"])
        assert np.array_equal(h.r.RSpath_final.T, ref["rs_path"])


def test_allpath_bitexact(ctx):
    """All 48 Reeds–Shepp candidates (cost + commands) and the findmin winner, vs the oracle."""
    r = np.random.default_rng(7)
    ns = np.r_[r.uniform(-4, 4, (509, 3)) * [1, 1, np.pi / 4],
               [[2.0, 0.0, 0.0], [0.0, 0.0, 0.0], [1e-300, -0.0, 0.0], [3.0, 2.0, np.pi], [-3.0, -2.0, -np.pi]]]
    best, cost, cmds = ha.allpath(ns, ctx=ctx)
    for b in range(len(ns)):
        bo, co, mo = oracle.ha_allpath(ns[b])
        assert best[b] == bo
        assert np.array_equal(cost[b], co, equal_nan=True)  # NaN candidates (e.g. ns = 0) included
        assert np.array_equal(cmds[b], mo, equal_nan=True)
    assert best[len(ns) - 5] == 0 and cost[len(ns) - 5, 0] == 2.0  # straight ahead: LSL, cost d


def test_retrieve_path_batch_bitexact(ctx):
    """retrievePath + cubic_fit (hybrid_astar_utils.jl:100-177) for a planned cfg4-shaped batch in one
    launch (mp_ha_retrieve_path) vs the oracle, bit for bit: actualpath, path_length, tol_length and the 50
    x/y/ψ samples; scenarios without a path retrieve nothing.  (Rmat*path and pinv(A)*B are evaluated
    without FMA, and duplicate arc-length knots take their left value: Julia's BLAS and Interpolations.jl
    are absent, so those two points are parity unpinned vs Julia.)"""
    hs = ha.scenario_batch(48, seed=6)
    ha.plan_batch(hs, ctx=ctx)
    ha.retrieve_batch(hs, ctx=ctx)
    found = 0
    for h in hs:
        if not h.r.found:
            assert h.r.actualpath is None
            continue
        found += 1
        ref = oracle.ha_retrieve(h.s.starting_states, h.r.hybrid_astar_states.T, h.r.RSpath_final.T)
        assert np.array_equal(h.r.actualpath.T, ref["actualpath"])
        assert np.array_equal(h.r.path_length, ref["path_length"])
        assert h.r.tol_length == ref["tol_length"]
        assert np.array_equal(h.r.interp_values, ref["samples"])
        assert np.isfinite(h.r.interp_values).all()
        s = np.linspace(0, h.r.tol_length, 7)
        assert np.isfinite(h.r.x_interp(s)).all() and np.isfinite(h.r.ψ_interp(s)).all()
    assert found > 10


def test_bench_batch_full_size_bitexact(ctx):
    """configs[3] at full size -- the bench's own 256-scenario batch (scenario_batch(256, seed=4)) -- planned
    on the device (mp_ha_plan, the tail shape included) vs 256 oracle plans (threaded: the ctypes calls
    release the GIL): found flags, pop counts, node counts, pop sequences, hybrid_astar_states and
    RSpath_final, bit for bit; then retrievePath + the tracker for every found path vs the oracle."""
    from concurrent.futures import ThreadPoolExecutor

    from motionplanning_amd import tracker

    hs = ha.scenario_batch(256, seed=4)
    ha.plan_batch(hs, ctx=ctx)
    h0 = hs[0]
    p = ha.params_of(h0)
    sc, pc = oracle.ha_neighbor_origin(h0.s.expand_time, h0.s.steer_set, h0.s.gear_set)

    def ref(h):
        return oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)

    with ThreadPoolExecutor(16) as ex:
        refs = list(ex.map(ref, hs))
    assert sum(h.r.loop_count for h in hs) == sum(r["pops"] for r in refs) == 54466
    for h, r in zip(hs, refs):
        assert h.r.found == r["found"] and h.r.loop_count == r["pops"] and h.r.n_nodes == r["n_nodes"]
        assert np.array_equal(h.r.pop_sequence, r["pop_seq"])
        if r["found"]:
            assert np.array_equal(h.r.hybrid_astar_states.T, r["states"])
            assert np.array_equal(h.r.RSpath_final.T, r["rs_path"])
    ha.retrieve_batch(hs, ctx=ctx)
    tracker.track_batch(hs, ctx=ctx)
    tp = tracker.params_of(tracker.settings_for(hs[0]))
    found = [h for h in hs if h.r.found]

    def track_ref(h):
        return oracle.track(tp, h.s.starting_real, h.r.tol_length, h.r.interp_values)

    with ThreadPoolExecutor(16) as ex:
        trs = list(ex.map(track_ref, found))
    for h, t in zip(found, trs):
        tr = h.r.tracking
        assert tr["status"] == tracker.STATUS[t["status"]] and tr["n_steps"] == t["n_steps"]
        assert np.array_equal(tr["final_state"], t["final"]) and tr["err_accumulated"] == t["err_acc"]
    assert len(found) == 169


@pytest.mark.parametrize("shift,cull", [(1e5, 1), (1e7, 0)])
def test_translated_scene_bitexact(ctx, shift, cull):
    """The SAT culls' 1e-6 m rounding margin is proven for coordinates <= 1e6 m (mp_ha_sat_cull_active; the
    library turns the culls off beyond it).  The perpendicular driver scene translated by (shift, shift) --
    walls, stbound, start and goal -- planned on the device vs the oracle's full SAT, bit for bit: at 1e5 m
    with the culls on, at 1e7 m with them off (CollisionDetection/src/utils.jl:37-74)."""
    import ctypes

    from motionplanning_amd.abi import ptr

    st = ha.driver_settings()
    sb = np.array(st["stbound"], float)
    sb[:2] += shift
    sc_ = ha.PERPENDICULAR
    walls = [[w[0] + shift, w[1] + shift] + list(w[2:]) for w in sc_["walls"]]
    start = [sc_["starting_real"][0] + shift, sc_["starting_real"][1] + shift, sc_["starting_real"][2]]
    goal = [sc_["ending_real"][0] + shift, sc_["ending_real"][1] + shift, sc_["ending_real"][2]]
    h = ha.defineHybridAstar(st["vehicle_size"], st["gear_set"], st["steer_set"], st["minR"], st["expand_time"],
                             st["resolutions"], sb, start, goal)
    ha.defineHybridAstarobs_(h, walls)
    p = ha.params_of(h)
    sc, pc = ha.install_primitives(h, ctx)
    W = np.array(h.s.obstacle_list, float)[None]
    a = np.array(h.s.starting_states, float)[None]
    b = np.array(h.s.ending_states, float)[None]
    on = ctypes.c_int32(-1)
    ctx.check(ctx.lib.mp_ha_sat_cull_active(ctx.handle, ctypes.byref(p), 1, ptr(W), ptr(a), ptr(b), ctypes.byref(on)))
    assert on.value == cull
    ha.planHybridAstar_(h, ctx=ctx)
    ref = oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
    assert h.r.found == ref["found"] and h.r.loop_count == ref["pops"] and h.r.n_nodes == ref["n_nodes"]
    assert np.array_equal(h.r.pop_sequence, ref["pop_seq"])
    if ref["found"]:
        assert np.array_equal(h.r.hybrid_astar_states.T, ref["states"])
        assert np.array_equal(h.r.RSpath_final.T, ref["rs_path"])
    assert ref["pops"] > 1


def test_sat_cull_guard_non_finite(ctx):
    """A NaN or infinite coordinate, length or heading anywhere in a call's inputs turns the SAT culls off
    (mp_ha_sat_cull_active 0): std::max would drop a NaN, so the guard tracks finiteness itself."""
    import ctypes

    from motionplanning_amd.abi import ptr

    h = ha.driver_searcher(ha.PERPENDICULAR)
    p = ha.params_of(h)
    ha.install_primitives(h, ctx)
    W0 = np.array(h.s.obstacle_list, float)[None]
    a0 = np.array(h.s.starting_states, float)[None]
    b0 = np.array(h.s.ending_states, float)[None]

    def active(W, a, b):
        on = ctypes.c_int32(-1)
        ctx.check(ctx.lib.mp_ha_sat_cull_active(ctx.handle, ctypes.byref(p), 1, ptr(W), ptr(a), ptr(b),
                                                ctypes.byref(on)))
        return on.value

    assert active(W0, a0, b0) == 1
    for bad in (np.nan, np.inf, -np.inf):
        for where in ("wall_x", "wall_len", "wall_psi", "start_x", "start_psi", "goal_y"):
            W, a, b = W0.copy(), a0.copy(), b0.copy()
            {"wall_x": lambda: W.__setitem__((0, 1, 0), bad), "wall_len": lambda: W.__setitem__((0, 0, 3), bad),
             "wall_psi": lambda: W.__setitem__((0, 2, 2), bad), "start_x": lambda: a.__setitem__((0, 0), bad),
             "start_psi": lambda: a.__setitem__((0, 2), bad), "goal_y": lambda: b.__setitem__((0, 1), bad)}[where]()
            assert active(W, a, b) == 0, (bad, where)


def test_primitive_table_memo(ctx):
    """mp_ha_neighbor_origin keeps the installed table while the settings repeat (plan_batch calls it every
    time): a repeat returns the same table, different settings install their own (each vs the oracle), and a
    plan after a settings change plans with the new table (bit-exact vs the oracle)."""
    import copy

    h, p, sc, pc = _setup(ctx)
    sc2, pc2 = ha.install_primitives(h, ctx)  # memo hit
    assert np.array_equal(sc2, sc) and np.array_equal(pc2, pc)
    h3 = copy.deepcopy(h)
    h3.s.steer_set = h.s.steer_set * 0.5  # other primitives, same shapes
    sc3, pc3 = ha.install_primitives(h3, ctx)
    sco, pco = oracle.ha_neighbor_origin(h3.s.expand_time, h3.s.steer_set, h3.s.gear_set)
    assert np.array_equal(sc3, sco) and np.array_equal(pc3, pco) and not np.array_equal(pc3, pc)
    hs = ha.scenario_batch(4, seed=7)
    ha.plan_batch(hs, ctx=ctx)  # its own settings again: reinstalled, then planned
    h0 = hs[0]
    scb, pcb = oracle.ha_neighbor_origin(h0.s.expand_time, h0.s.steer_set, h0.s.gear_set)
    pb = ha.params_of(h0)
    for h4 in hs:
        ref = oracle.ha_plan(pb, h4.s.starting_states, h4.s.ending_states, np.array(h4.s.obstacle_list), scb, pcb)
        assert h4.r.loop_count == ref["pops"] and np.array_equal(h4.r.pop_sequence, ref["pop_seq"])
