"""Hybrid A* — host-side mirror of PathPlanning/HybridAstar/src/{types,setup,hybrid_astar_utils}.jl
over the libmpgpu C-ABI (mp_ha_*).

``defineHybridAstar`` / ``defineHybridAstarobs_`` / ``planHybridAstar_`` keep the reference's
names and argument meaning.  The search loop runs in the library and is device-resident: per
iteration one fused launch for the whole batch of scenes (RS_connected + the 62-neighbour
FindNewNode expansion) and one bookkeeping launch (Dict / open-list updates, popfirst!),
enqueued without host round trips; ``plan_batch`` runs B scenes in lockstep.
Setup-time lattice arithmetic (regulate_states, Encode bounds) is exact IEEE
(round-half-even, fmod), computed here.
"""
import ctypes
import itertools
import math
import time
from dataclasses import dataclass, field

import numpy as np

from .abi import HAParams, f64, ptr
from .configs import julia_linrange
from .context import default_context

PI = math.pi


def jl_mod(x, y):
    """Julia mod(x, y) for floats (fmod + sign fix)."""
    r = math.fmod(x, y)
    if r == 0.0:
        return math.copysign(r, y)
    if (r > 0.0) != (y > 0.0):
        return r + y
    return r


def modpi(a):
    """modπ, ReedsSheppsUtils.jl:32-46."""
    if -PI <= a <= PI:
        return a
    a = jl_mod(a, 2 * PI)
    if a < -PI:
        a = a + 2 * PI
    elif a > PI:
        a = a - 2 * PI
    return a


def jl_round(x):
    """Julia round(::Float64): ties to even."""
    return float(round(x))


def regulate_states(res, s):
    """regulate_states, hybrid_astar_utils.jl:211-222."""
    x = jl_round(s[0] / res[0]) * res[0]
    y = jl_round(s[1] / res[1]) * res[1]
    psi = jl_round(modpi(s[2]) / res[2]) * res[2]
    return np.array([x, y, psi])


@dataclass
class HybridAstarSettings:
    """types.jl:20-43."""

    vehicle_size: np.ndarray = None
    starting_states: np.ndarray = None
    ending_states: np.ndarray = None
    starting_real: np.ndarray = None
    ending_real: np.ndarray = None
    obstacle_list: list = field(default_factory=list)
    gear_set: np.ndarray = None
    steer_set: np.ndarray = None
    stbound: np.ndarray = None
    resolutions: np.ndarray = None
    num_steer: int = 0
    num_gear: int = 0
    num_neighbors: int = 0
    use_astar: bool = False
    minR: float = 1.0
    expand_time: float = 1.0
    n_col: int = 0


@dataclass
class HybridAstarResult:
    """types.jl:54-63; actualpath / tol_length / x_interp, y_interp, ψ_interp are filled by
    retrievePath (mp_ha_retrieve_path)."""

    found: bool = False
    RSpath_final: np.ndarray = None
    hybrid_astar_states: np.ndarray = None
    planning_time: float = 0.0
    loop_count: int = 0
    n_nodes: int = 0
    pop_sequence: np.ndarray = None
    actualpath: np.ndarray = None
    path_length: np.ndarray = None
    tol_length: float = 0.0
    interp_knots: np.ndarray = None
    interp_values: np.ndarray = None
    x_interp: object = None
    y_interp: object = None
    ψ_interp: object = None
    tracking: dict = None  # main_Tracker.jl's simulation (tracker.track_batch)


@dataclass
class HybridAstarSearcher:
    s: HybridAstarSettings = field(default_factory=HybridAstarSettings)
    r: HybridAstarResult = field(default_factory=HybridAstarResult)


def defineHybridAstar(vehicle_size=(2, 1), gear_set=(1, -1), steer_set=None, minR=1.0, expand_time=1.0,
                      resolutions=(0.2, 0.2, PI / 10), stbound=((-15, 15), (-15, 5), (-PI, PI)),
                      starting_real=(10.0, -5.0, 0.0), ending_real=(-5.0, -5.0, 0.0), use_astar=False):
    """setup.jl:3-53.  use_astar=True (the grid-A* heuristic) is out of scope."""
    if use_astar:
        raise NotImplementedError("use_astar=true (PathPlanning/Astar heuristic) is out of scope")
    steer_set = julia_linrange(-1, 1, 7) if steer_set is None else np.asarray(steer_set, np.float64)
    h = HybridAstarSearcher()
    s = h.s
    s.vehicle_size = np.asarray(vehicle_size, np.float64)
    s.gear_set = np.asarray(gear_set, np.float64)
    s.steer_set = np.asarray(steer_set, np.float64)
    s.num_gear, s.num_steer = len(s.gear_set), len(s.steer_set)
    s.num_neighbors = s.num_gear * s.num_steer
    s.minR, s.expand_time = float(minR), float(expand_time)
    s.resolutions = np.asarray(resolutions, np.float64)
    sb = np.asarray(stbound, np.float64)
    s.stbound = np.c_[regulate_states(s.resolutions, sb[:, 0]), regulate_states(s.resolutions, sb[:, 1])]
    s.starting_real = np.asarray(starting_real, np.float64)
    s.ending_real = np.asarray(ending_real, np.float64)
    s.starting_states = regulate_states(s.resolutions, s.starting_real)
    s.ending_states = regulate_states(s.resolutions, s.ending_real)
    s.n_col = int(math.floor(s.expand_time / 1e-2))
    return h


def defineHybridAstarobs_(h, obstacle_list):
    """defineHybridAstarobs! (setup.jl:56-59): blocks [x, y, ψ, l/2, w/2]."""
    h.s.obstacle_list = [list(map(float, b)) for b in obstacle_list]


def params_of(h, max_pops=5000):
    s = h.s
    p = HAParams()
    p.vehicle_len, p.vehicle_wid = float(s.vehicle_size[0]), float(s.vehicle_size[1])
    p.minR, p.expand_time = s.minR, s.expand_time
    for i in range(3):
        p.res[i] = s.resolutions[i]
    for i in range(3):
        p.stbound[2 * i], p.stbound[2 * i + 1] = s.stbound[i, 0], s.stbound[i, 1]
    p.n_walls = len(s.obstacle_list)
    p.n_prim = s.num_neighbors
    p.n_col = s.n_col
    p.max_pops = max_pops
    return p


def install_primitives(h, ctx=None):
    """neighbor_origin (hybrid_astar_utils.jl:483-503) computed by the library and cached in the context."""
    ctx = ctx or default_context()
    s = h.s
    p = params_of(h)
    sc = np.zeros((p.n_prim, 3))
    pc = np.zeros((p.n_prim, p.n_col, 3))
    ctx.check(ctx.lib.mp_ha_neighbor_origin(ctx.handle, ctypes.byref(p), s.num_steer, ptr(s.steer_set), s.num_gear,
                                            ptr(s.gear_set), ptr(sc), ptr(pc)))
    return sc, pc


def plan_batch(searchers, ctx=None, max_pops=5000):
    """planHybridAstar! for B scenes sharing settings (vehicle, primitives, bounds, resolutions,
    number of walls), each with its own start, goal and walls, in lockstep on the device."""
    ctx = ctx or default_context()
    h0 = searchers[0]
    p = params_of(h0, max_pops)
    # the primitive table (the library keeps it while the settings stay the same; no copies back)
    ctx.check(ctx.lib.mp_ha_neighbor_origin(ctx.handle, ctypes.byref(params_of(h0)), h0.s.num_steer, ptr(h0.s.steer_set),
                                            h0.s.num_gear, ptr(h0.s.gear_set), None, None))
    B = len(searchers)
    start = f64([h.s.starting_states for h in searchers])
    goal = f64([h.s.ending_states for h in searchers])
    if any(len(h.s.obstacle_list) != p.n_walls for h in searchers):
        raise ValueError("plan_batch: every scene needs the same number of walls")
    walls = np.fromiter(itertools.chain.from_iterable(itertools.chain.from_iterable(h.s.obstacle_list for h in searchers)),
                        np.float64, B * p.n_walls * 5).reshape(B, p.n_walls, 5)
    found = np.zeros(B, np.int32)
    pops = np.zeros(B, np.int32)
    n_nodes = np.zeros(B, np.int32)
    n_states = np.zeros(B, np.int32)
    rs_len = np.zeros(B, np.int32)
    # the large outputs live in per-context buffers reused across calls (their pages stay mapped): the library
    # writes every pop_seq entry (-1 past the pops), the first n_states rows of states and rs_len rows of rs_path
    key = (B, max_pops)
    bufs = getattr(ctx, "_ha_plan_bufs", None)
    if bufs is None or bufs[0] != key:
        bufs = (key, np.empty((B, max_pops), np.int64), np.empty((B, max_pops, 3)), np.zeros((B, 501, 3)))
        ctx._ha_plan_bufs = bufs
    _, pop_seq, states, rs_path = bufs
    t0 = time.time()
    ctx.check(ctx.lib.mp_ha_plan(ctx.handle, ctypes.byref(p), B, ptr(start), ptr(goal), ptr(walls), ptr(found),
                                 ptr(pops), ptr(n_nodes), ptr(pop_seq), ptr(n_states), ptr(states), ptr(rs_len),
                                 ptr(rs_path)))
    dt = time.time() - t0
    # one compact copy per output, each scene's result a view of it (nothing aliases the reused buffers)
    ps = pop_seq[:, : max(int(pops.max()), 0)].copy()
    sts = states[:, : max(int(n_states.max()), 0)].copy()
    rsp = rs_path[:, : max(int(rs_len.max()), 0)].copy()
    for b, h in enumerate(searchers):
        r = h.r
        r.found = bool(found[b])
        r.loop_count = int(pops[b])
        r.n_nodes = int(n_nodes[b])
        r.pop_sequence = ps[b, : pops[b]]
        r.hybrid_astar_states = sts[b, : n_states[b]].T
        r.RSpath_final = rsp[b, : rs_len[b]].T
        r.planning_time = dt
    return searchers


def retrieve_batch(searchers, ctx=None):
    """retrievePath (hybrid_astar_utils.jl:129-177, with cubic_fit :100-127) for planned searchers in one
    launch (mp_ha_retrieve_path): fills r.actualpath (3, L), r.path_length, r.tol_length and the
    x/y/ψ_interp interpolants over the 50 arc-length knots LinRange(0, tol_length, 50) (linear, as
    linear_interpolation builds them; evaluated here with numpy on the device-computed knot values)."""
    ctx = ctx or default_context()
    B = len(searchers)
    start = f64([h.s.starting_states for h in searchers])
    ns = np.array([0 if h.r.hybrid_astar_states is None or not h.r.found else h.r.hybrid_astar_states.shape[1]
                   for h in searchers], np.int32)
    stride = max(1, int(ns.max()))
    states = np.zeros((B, stride, 3))
    rs_len = np.zeros(B, np.int32)
    rs = np.zeros((B, 501, 3))
    for b, h in enumerate(searchers):
        if ns[b]:
            states[b, : ns[b]] = h.r.hybrid_astar_states.T
            rs_len[b] = h.r.RSpath_final.shape[1]
            rs[b, : rs_len[b]] = h.r.RSpath_final.T
    tot = int(sum(1 + 100 * (n - 1) + r for n, r in zip(ns, rs_len) if n))
    off = np.zeros(B + 1, np.int64)
    pts, plen = np.zeros((max(tot, 1), 3)), np.zeros(max(tot, 1))
    npts, tol, smp = np.zeros(B, np.int32), np.zeros(B), np.zeros((B, 50, 3))
    ctx.check(ctx.lib.mp_ha_retrieve_path(ctx.handle, B, ptr(start), ptr(ns), ptr(states), stride, ptr(rs_len),
                                          ptr(rs), ptr(off), ptr(pts), ptr(plen), ptr(npts), ptr(tol), ptr(smp)))
    for b, h in enumerate(searchers):
        r = h.r
        if not ns[b]:
            continue
        a, e = int(off[b]), int(off[b + 1])
        r.actualpath = pts[a:e].T.copy()
        r.path_length = plen[a:e].copy()
        r.tol_length = float(tol[b])
        r.interp_knots = configs_linrange(0.0, r.tol_length, 50)
        r.interp_values = smp[b].copy()
        k, v = r.interp_knots, r.interp_values
        r.x_interp = lambda s, k=k, v=v: np.interp(s, k, v[:, 0])
        r.y_interp = lambda s, k=k, v=v: np.interp(s, k, v[:, 1])
        r.ψ_interp = lambda s, k=k, v=v: np.interp(s, k, v[:, 2])
    return searchers


def retrievePath(h, ctx=None):
    """retrievePath(hybrid_astar) (hybrid_astar_utils.jl:129-177) for one planned searcher."""
    retrieve_batch([h], ctx=ctx)
    return None


def configs_linrange(a, b, n):
    from .configs import julia_linrange

    return julia_linrange(a, b, n)


def planHybridAstar_(h, ctx=None, max_pops=5000):
    """planHybridAstar! (hybrid_astar_utils.jl:235-296) for one scene."""
    plan_batch([h], ctx=ctx, max_pops=max_pops)
    return None


def changeBasis(init, term, minR):
    """changeBasis, ReedsSheppsUtils.jl:2-11 (host arithmetic; the device does this inside
    mp_ha_rs_connect / mp_ha_expand with the library's FDLIBM sin/cos)."""
    dx, dy = (term[0] - init[0]) / minR, (term[1] - init[1]) / minR
    c, s = math.cos(init[2]), math.sin(init[2])
    return np.array([dx * c + dy * s, -dx * s + dy * c, term[2] - init[2]])


def allpath(norm_states, ctx=None):
    """allpath (ReedsSheppsUtils.jl:468-511) for B normalised states on the device.
    Returns (best[B] 0-based candidate index, cost[B][48], cmds[B][48][5][3]) with cmds rows
    [distance, gear, steer]; Inf cost (all-zero cmds) where a word is infeasible."""
    ctx = ctx or default_context()
    ns = f64(norm_states).reshape(-1, 3)
    B = ns.shape[0]
    cost = np.zeros((B, 48))
    cmds = np.zeros((B, 48, 5, 3))
    best = np.zeros(B, np.int32)
    ctx.check(ctx.lib.mp_ha_allpath(ctx.handle, B, ptr(ns), ptr(cost), ptr(cmds), ptr(best)))
    return best, cost, cmds


# ----------------------------------------------------- driver scenes
def driver_settings():
    """PathPlanning/HybridAstar/main_hybrid_astar.jl:21-29."""
    vehicle_size = [3, 2]
    max_df = PI / 6
    minR = vehicle_size[0] / math.tan(max_df)
    steer_set = julia_linrange(-1 / minR, 1 / minR, 31)
    return dict(vehicle_size=vehicle_size, gear_set=[1, -1], steer_set=steer_set, minR=minR, expand_time=2.5,
                resolutions=[0.5, 0.5, PI / 12], stbound=[[-5, 10], [0, 10], [-PI, PI]])


PERPENDICULAR = dict(  # main_hybrid_astar.jl:15-17
    starting_real=[7.0, 0.0, PI / 2], ending_real=[0.0, 0.5, PI / 2],
    walls=[[0.0, -1.0, 0.0, 5.5 / 2 + 1.0, 1.0], [-5.5 / 2, 2.7432 / 2, 0.0, 1.0, 2.7432 / 2],
           [5.5 / 2, 2.7432 / 2, 0.0, 1.0, 2.7432 / 2]])
PARALLEL = dict(  # main_hybrid_astar.jl:10-12
    starting_real=[7.0, 0.0, PI / 2], ending_real=[-1.5, 2.0, 0.0],
    walls=[[0.0, -1.0, 0.0, 5.5 / 2 + 1.0, 1.0], [-(5.5 + 3) / 2, 1.0, 0.0, 1.0, 1.0],
           [(5.5 + 3) / 2, 1.0, 0.0, 1.0, 1.0]])


def driver_searcher(scene=PERPENDICULAR, start=None):
    st = driver_settings()
    h = defineHybridAstar(st["vehicle_size"], st["gear_set"], st["steer_set"], st["minR"], st["expand_time"],
                          st["resolutions"], st["stbound"], scene["starting_real"] if start is None else start,
                          scene["ending_real"])
    defineHybridAstarobs_(h, scene["walls"])
    return h


def scenario_batch(n=256, seed=4):
    """n/2 perpendicular + n/2 parallel scenes; start x in {5, 5.5, ..., 9},
    start ψ = π/2 + k·π/12, k in {-2..2}, seeded."""
    r = np.random.default_rng(seed)
    xs = np.arange(5.0, 9.0 + 1e-9, 0.5)
    out = []
    for i in range(n):
        scene = PERPENDICULAR if i < n // 2 else PARALLEL
        x = float(xs[r.integers(len(xs))])
        k = int(r.integers(-2, 3))
        out.append(driver_searcher(scene, [x, 0.0, PI / 2 + k * PI / 12]))
    return out
