"""MPPI planner — host-side mirror of OptimalControl/MPPI/src/{types,setup,MPPIUtils}.jl.

The names, argument meaning and error behaviour follow the reference so a
caller of ``MPPIPlan(mppi)`` can switch over; the hot loop (sample → rollout →
cost → weights → weighted control → final rollout) runs in one HIP launch via
``mp_mppi_plan`` (include/mpgpu.h).  Julia's mutating ``defineMPPIobs!`` /
``defineMPPINominalControl!`` are spelled with a trailing underscore.
"""
import ctypes
import math
import time
from dataclasses import dataclass, field

import numpy as np

from . import configs
from .abi import MP_NOISE_EXTERNAL, MP_NOISE_PHILOX, MP_ERR_NUMERIC, MPPILoopParams, MPPIParams, f64, ptr
from .context import default_context


@dataclass
class MPPIHolder:
    """types.jl:3-8 (one element of TrajectoryCollection)."""

    Trajectory: np.ndarray = None
    Control: np.ndarray = None
    Feasibility: bool = False
    cost: float = 1e6


@dataclass
class MPPISetting:
    """types.jl:10-31."""

    numStates: int = 0
    numControls: int = 0
    X0: np.ndarray = None
    XL: np.ndarray = None
    XU: np.ndarray = None
    CL: np.ndarray = None
    CU: np.ndarray = None
    dt: float = 0.0
    T: float = 0.0
    N: int = 0
    goal: np.ndarray = None
    obstacle_list: list = field(default_factory=list)
    SamplingNumber: int = 0
    FeasibilityCount: int = 1300
    tmax: float = 0.1
    NominalControl: np.ndarray = None
    Σ: np.ndarray = None
    lambda_: float = 0.02
    SlackPenalty: float = 1e5
    # build extensions
    grid: np.ndarray = None
    grid_spec: dict = None
    seed: int = 0
    solve_counter: int = 0


@dataclass
class MPPIPlanner:
    """types.jl:32-34."""

    TrajectoryCollection: list = field(default_factory=list)


@dataclass
class MPPIResult:
    """types.jl:36-44."""

    Traj: np.ndarray = None
    Control: np.ndarray = None
    Feasibility: str = "InFeasible"
    cost: float = 1e6
    time: float = 0.0
    FeasibleTrajCount: int = 0
    RolloutCount: int = 0
    log: dict = None  # build extension: per-replan results of MPPIClosedLoop


@dataclass
class MPPISearcher:
    """types.jl:46-50."""

    s: MPPISetting = field(default_factory=MPPISetting)
    p: MPPIPlanner = field(default_factory=MPPIPlanner)
    r: MPPIResult = field(default_factory=MPPIResult)


def defineMPPI(numStates=0, numControls=0, lambda_=0.25, X0=None, goal=None, SamplingNumber=500, Σ=None, N=15,
               T=3.0, XL=None, XU=None, CL=None, CU=None, seed=0):
    """setup.jl:3-59 — same validation messages as the reference's error() calls."""
    if numControls <= 0:
        raise ValueError(f"Controls ({numControls}) must be > 0")
    if numStates <= 0:
        raise ValueError(f"States ({numStates}) must be > 0")
    X0 = np.full(numStates, np.nan) if X0 is None else np.asarray(X0, np.float64)
    XL = np.full(numStates, np.nan) if XL is None else np.asarray(XL, np.float64)
    XU = np.full(numStates, np.nan) if XU is None else np.asarray(XU, np.float64)
    CL = np.full(numControls, np.nan) if CL is None else np.asarray(CL, np.float64)
    CU = np.full(numControls, np.nan) if CU is None else np.asarray(CU, np.float64)
    if len(X0) != numStates:
        raise ValueError(f"Length of X0 ({len(X0)}) must match number of states ({numStates})")
    if len(XL) != numStates:
        raise ValueError(f"Length of XL ({len(XL)}) must match number of states ({numStates})")
    if len(XU) != numStates:
        raise ValueError(f"Length of XU ({len(XU)}) must match number of states ({numStates})")
    if len(CL) != numControls:
        raise ValueError(f"Length of CL ({len(CL)}) must match number of controls ({numControls})")
    if len(CU) != numControls:
        raise ValueError(f"Length of CU ({len(CU)}) must match number of controls ({numControls})")
    if numStates != 7 or numControls != 2:
        raise ValueError("the bicycle model of vehicledynamics.jl has 7 states and 2 controls")
    m = MPPISearcher()
    s = m.s
    s.goal = np.asarray(goal if goal is not None else [np.nan, np.nan], np.float64)
    s.numStates, s.numControls = numStates, numControls
    s.lambda_ = float(lambda_)
    s.X0, s.XL, s.XU, s.CL, s.CU = X0, XL, XU, CL, CU
    s.T, s.N = float(T), int(N)
    s.dt = s.T / s.N
    s.SamplingNumber = int(SamplingNumber)
    s.NominalControl = np.zeros((s.N, s.numControls))
    s.Σ = np.eye(numControls) if Σ is None else np.asarray(Σ, np.float64).reshape(2, 2)
    s.seed = int(seed)
    return m


def defineMPPIobs_(mppi, obstacle_list):
    """defineMPPIobs! (setup.jl:61-64)."""
    mppi.s.obstacle_list = [list(map(float, o)) for o in obstacle_list]


def defineMPPIgrid_(mppi, grid, spec):
    """Occupancy-grid cost (build extension): uint8 [ny][nx] over spec."""
    mppi.s.grid = np.ascontiguousarray(grid, np.uint8)
    mppi.s.grid_spec = dict(spec)


def defineMPPINominalControl_(mppi, *args):
    """defineMPPINominalControl! (setup.jl:70-80): U, or (U, Σ)."""
    mppi.s.NominalControl = np.asarray(args[0], np.float64).reshape(mppi.s.N, mppi.s.numControls)
    if len(args) > 1:
        mppi.s.Σ = np.asarray(args[1], np.float64).reshape(2, 2)


def ShiftInitialCondition(mppi, X0):
    """MPPIUtils.jl:24-27."""
    mppi.s.X0 = np.asarray(X0, np.float64)


def params_of(mppi, noise_mode):
    s = mppi.s
    return configs.mppi_params(
        K=s.SamplingNumber, H=s.N, T=s.T, lam=s.lambda_, sigma=list(np.asarray(s.Σ).ravel()), XL=s.XL, XU=s.XU,
        CL=s.CL, CU=s.CU, n_obs=len(s.obstacle_list), feasibility_count=s.FeasibilityCount,
        grid=s.grid_spec if s.grid is not None else None, noise_mode=noise_mode, ctrl_cost=1, seed=s.seed,
        offset=s.solve_counter, dt=s.dt)


def mppi_plan_batch(p: MPPIParams, X0, goal, U_nom, obstacles=None, grid=None, noise=None, collect=False,
                    ctx=None):
    """S independent MPPIPlan solves in one launch.  Shapes: X0 (S,7), goal (S,2), U_nom (S,H,2),
    obstacles (S,n_obs,3), grid (S,ny,nx) uint8, noise (S,K,H,2) or None (Philox).
    collect: True = the whole TrajectoryCollection, "costs" = only its costs and feasibility flags
    (the large state / control lists stay on the device), False = none."""
    ctx = ctx or default_context()
    X0 = f64(X0).reshape(-1, 7)
    S, K, H = X0.shape[0], p.K, p.H
    goal = f64(goal, (S, 2))
    U_nom = f64(U_nom, (S, H, 2))
    obstacles = None if obstacles is None or p.n_obs == 0 else f64(obstacles, (S, p.n_obs, 3))
    grid = None if grid is None or p.grid_nx == 0 else np.ascontiguousarray(grid, np.uint8).reshape(
        S, p.grid_ny, p.grid_nx)
    if noise is not None:
        noise = f64(noise, (S, K, H, 2))
        p.noise_mode = MP_NOISE_EXTERNAL
    else:
        p.noise_mode = MP_NOISE_PHILOX
    out = dict(U=np.zeros((S, H, 2)), traj=np.zeros((S, H + 1, 7)), cost=np.zeros(S),
               feasible=np.zeros(S, np.int32), rollout_count=np.zeros(S, np.int32),
               feasible_count=np.zeros(S, np.int32))
    coll = {}
    if collect:
        # device layout: structure of arrays, rollout index fastest (include/mpgpu.h)
        coll = dict(cost=np.zeros((S, K)), feas=np.zeros((S, K), np.uint8))
        if collect != "costs":
            coll.update(traj_soa=np.zeros((S, H + 1, 7, K)), ctrl_soa=np.zeros((S, H, K, 2)))
    st = ctx.lib.mp_mppi_plan(ctx.handle, ctypes.byref(p), S, ptr(X0), ptr(goal), ptr(U_nom), ptr(obstacles),
                              ptr(grid), ptr(noise), ptr(out["U"]), ptr(out["traj"]), ptr(out["cost"]),
                              ptr(out["feasible"]), ptr(out["rollout_count"]), ptr(out["feasible_count"]),
                              ptr(coll.get("traj_soa")), ptr(coll.get("ctrl_soa")), ptr(coll.get("cost")),
                              ptr(coll.get("feas")))
    if collect and collect != "costs":  # reference-shaped views: traj (S, K, H+1, 7), ctrl (S, K, H, 2)
        coll["traj"] = coll["traj_soa"].transpose(0, 3, 1, 2)
        coll["ctrl"] = coll["ctrl_soa"].transpose(0, 2, 1, 3)
    out["nan"] = st == MP_ERR_NUMERIC
    if st != MP_ERR_NUMERIC:
        ctx.check(st)
    out["coll"] = coll
    return out


def mppi_plan_sharded(group, p: MPPIParams, X0, goal, U_nom, obstacles=None, grid=None, noise=None):
    """mp_mppi_plan_sharded: S scenes split over the GPUs of a CommGroup (balanced blocks, Philox counter
    word scene_base + block start) and one RCCL all-gather of the per-scene results.  Same shapes and
    outputs as mppi_plan_batch without the TrajectoryCollection; equal to one mppi_plan_batch over all S
    scenes."""
    X0 = f64(X0).reshape(-1, 7)
    S, K, H = X0.shape[0], p.K, p.H
    goal = f64(goal, (S, 2))
    U_nom = f64(U_nom, (S, H, 2))
    obstacles = None if obstacles is None or p.n_obs == 0 else f64(obstacles, (S, p.n_obs, 3))
    grid = None if grid is None or p.grid_nx == 0 else np.ascontiguousarray(grid, np.uint8).reshape(
        S, p.grid_ny, p.grid_nx)
    if noise is not None:
        noise = f64(noise, (S, K, H, 2))
        p.noise_mode = MP_NOISE_EXTERNAL
    else:
        p.noise_mode = MP_NOISE_PHILOX
    out = dict(U=np.zeros((S, H, 2)), traj=np.zeros((S, H + 1, 7)), cost=np.zeros(S),
               feasible=np.zeros(S, np.int32), rollout_count=np.zeros(S, np.int32),
               feasible_count=np.zeros(S, np.int32))
    st = group.lib.mp_mppi_plan_sharded(group.array, group.n, ctypes.byref(p), S, ptr(X0), ptr(goal), ptr(U_nom),
                                        ptr(obstacles), ptr(grid), ptr(noise), ptr(out["U"]), ptr(out["traj"]),
                                        ptr(out["cost"]), ptr(out["feasible"]), ptr(out["rollout_count"]),
                                        ptr(out["feasible_count"]))
    out["nan"] = st == MP_ERR_NUMERIC
    if st != MP_ERR_NUMERIC:
        group.check(st)
    return out


def MPPIPlan(mppi, noise=None, collect=True, ctx=None):
    """MPPIUtils.jl:169-203.  Mutates mppi.r and mppi.p.TrajectoryCollection.

    noise: optional z ~ N(0, I) of shape (SamplingNumber, N, 2) (the draws the reference
    takes from MvNormal); default is the device Philox stream (seed mppi.s.seed, counter
    advanced per call).  Raises MPGPUError on device failure; a NaN cost sets Feasibility
    to :InFeasible and the cost to NaN like the reference would.
    """
    s = mppi.s
    t1 = time.time()
    p = params_of(mppi, MP_NOISE_EXTERNAL if noise is not None else MP_NOISE_PHILOX)
    obst = np.asarray(s.obstacle_list, np.float64).reshape(1, -1, 3) if s.obstacle_list else None
    grid = s.grid[None] if s.grid is not None else None
    out = mppi_plan_batch(p, s.X0[None], s.goal[None], s.NominalControl[None], obst, grid,
                          None if noise is None else np.asarray(noise)[None], collect=collect, ctx=ctx)
    s.solve_counter += 1
    m = int(out["rollout_count"][0]) - 1
    if collect:
        c = out["coll"]
        mppi.p.TrajectoryCollection = [MPPIHolder(c["traj"][0, i], c["ctrl"][0, i], bool(c["feas"][0, i]),
                                                  float(c["cost"][0, i])) for i in range(m)]
    r = mppi.r
    r.Traj = out["traj"][0]
    r.Control = out["U"][0]
    r.Feasibility = "Feasible" if out["feasible"][0] else "InFeasible"
    r.cost = float(out["cost"][0])
    r.RolloutCount = int(out["rollout_count"][0])
    r.FeasibleTrajCount = int(out["feasible_count"][0])
    r.time = time.time() - t1
    return None


def mppi_closed_loop_batch(p: MPPIParams, X0, goal, U_nom0, hold, update_steps, max_steps, plant_dt, goal_radius,
                           obstacles=None, grid=None, noise=None, logs=True, poll_every=0, ctx=None):
    """S closed loops of MPPI/main.jl:55-83 in lockstep on the device (mp_mppi_closed_loop).
    Shapes: X0 (S,7), goal (S,2), U_nom0 (S,H,2), hold (update_steps,) 0-based rows, noise (R,S,K,H,2)
    or None (Philox, counter word p.offset + replan).  Returns his (S, max_steps+1, 8) with n_rows[s]
    valid rows, n_replans (S,), and per-replan logs U (S,R,H,2), traj (S,R,H+1,7), cost, feasible,
    rollout_count (S,R) valid for r < n_replans[s]."""
    ctx = ctx or default_context()
    X0 = f64(X0).reshape(-1, 7)
    S, K, H = X0.shape[0], p.K, p.H
    R = -(-int(max_steps) // int(update_steps))
    goal = f64(goal, (S, 2))
    U_nom0 = f64(U_nom0, (S, H, 2))
    hold = np.ascontiguousarray(hold, np.int32).reshape(int(update_steps))
    obstacles = None if obstacles is None or p.n_obs == 0 else f64(obstacles, (S, p.n_obs, 3))
    grid = None if grid is None or p.grid_nx == 0 else np.ascontiguousarray(grid, np.uint8).reshape(
        S, p.grid_ny, p.grid_nx)
    if noise is not None:
        noise = f64(noise, (R, S, K, H, 2))
        p.noise_mode = MP_NOISE_EXTERNAL
    else:
        p.noise_mode = MP_NOISE_PHILOX
    lp = MPPILoopParams(update_steps=int(update_steps), max_steps=int(max_steps), plant_dt=float(plant_dt),
                        goal_radius=float(goal_radius), poll_every=int(poll_every))
    out = dict(his=np.zeros((S, max_steps + 1, 8)), n_rows=np.zeros(S, np.int32), n_replans=np.zeros(S, np.int32))
    Rl = max(R, 1)
    lg = {}
    if logs:
        lg = dict(U=np.zeros((S, Rl, H, 2)), traj=np.zeros((S, Rl, H + 1, 7)), cost=np.zeros((S, Rl)),
                  feasible=np.zeros((S, Rl), np.int32), rollout_count=np.zeros((S, Rl), np.int32))
    st = ctx.lib.mp_mppi_closed_loop(ctx.handle, ctypes.byref(p), ctypes.byref(lp), S, ptr(X0), ptr(goal),
                                     ptr(U_nom0), ptr(obstacles), ptr(grid), ptr(hold), ptr(noise), ptr(out["his"]),
                                     ptr(out["n_rows"]), ptr(out["n_replans"]), ptr(lg.get("U")), ptr(lg.get("traj")),
                                     ptr(lg.get("cost")), ptr(lg.get("feasible")), ptr(lg.get("rollout_count")))
    out["nan"] = st == MP_ERR_NUMERIC
    if st != MP_ERR_NUMERIC:
        ctx.check(st)
    out.update(lg)
    return out


def MPPIClosedLoop(mppi, update_time=configs.UPDATE_TIME_REF, δt=configs.PLANT_DT_REF, sim_time=configs.SIM_TIME_REF,
                   goal_radius=configs.GOAL_RADIUS_MPPI, noise=None, ctx=None):
    """The driver loop of OptimalControl/MPPI/main.jl:49-83 for the searcher's scene: replan every
    update_idx plant steps from the current state with NominalControls = the previous r.Control,
    hold the interpolated control, step the 1 kHz Euler plant, stop within goal_radius of the goal.
    Returns states_his as rows [t, states...] (the transpose of the reference's 8×n matrix, i.e.
    the MPPITrajectory.csv layout); mppi.r holds the last plan and mppi.r.log the per-replan
    (Control, Traj, cost, Feasibility, RolloutCount)."""
    s = mppi.s
    t1 = time.time()
    update_idx, hold = configs.mppi_hold_index(s.T, s.N, update_time, δt)
    max_steps = int(math.floor(sim_time / δt))
    p = params_of(mppi, MP_NOISE_EXTERNAL if noise is not None else MP_NOISE_PHILOX)
    obst = np.asarray(s.obstacle_list, np.float64).reshape(1, -1, 3) if s.obstacle_list else None
    grid = s.grid[None] if s.grid is not None else None
    z = None if noise is None else np.asarray(noise, np.float64)[:, None]
    out = mppi_closed_loop_batch(p, s.X0[None], s.goal[None], s.NominalControl[None], hold, update_idx, max_steps,
                                 δt, goal_radius, obst, grid, z, ctx=ctx)
    n, R = int(out["n_rows"][0]), int(out["n_replans"][0])
    s.solve_counter += R
    r = mppi.r
    if R:
        r.Traj = out["traj"][0, R - 1]
        r.Control = out["U"][0, R - 1]
        r.Feasibility = "Feasible" if out["feasible"][0, R - 1] else "InFeasible"
        r.cost = float(out["cost"][0, R - 1])
        r.RolloutCount = int(out["rollout_count"][0, R - 1])
        s.X0 = out["his"][0, (R - 1) * update_idx, 1:].copy()
        s.NominalControl = out["U"][0, R - 1].copy()
    r.log = dict(Control=out["U"][0, :R], Traj=out["traj"][0, :R], cost=out["cost"][0, :R],
                 Feasibility=out["feasible"][0, :R], RolloutCount=out["rollout_count"][0, :R])
    r.time = time.time() - t1
    return out["his"][0, :n]


def TrajectoryRollout(mppi, ctrl_list, ctx=None):
    """MPPIUtils.jl:31-57 for one control list (H, 2): returns (states_his, ctrl_list, constraint, cost)."""
    from .rollout import rollout_batch

    s = mppi.s
    p = params_of(mppi, MP_NOISE_EXTERNAL)
    ctrl = f64(ctrl_list, (1, 1, s.N, 2))
    obst = np.asarray(s.obstacle_list, np.float64).reshape(1, -1, 3) if s.obstacle_list else None
    r = rollout_batch(p, s.X0[None], s.goal[None], ctrl, U_nom=s.NominalControl[None], obstacles=obst,
                      grid=None if s.grid is None else s.grid[None], want_traj=True, ctx=ctx)
    return r["traj"][0, 0], np.asarray(ctrl_list), bool(r["feas"][0, 0]), float(r["cost"][0, 0])


def reference_searcher(K=1500, N=20, T=3.0, obstacles=configs.OBSTACLES_REF, seed=0):
    """The searcher of OptimalControl/MPPI/main.jl:7-30."""
    m = defineMPPI(7, 2, configs.LAMBDA_REF, configs.X0_REF, configs.GOAL_REF, K,
                   np.array(configs.SIGMA_REF).reshape(2, 2), N, T, configs.XL_REF, configs.XU_REF,
                   configs.CL_MPPI, configs.CU_MPPI, seed=seed)
    defineMPPIobs_(m, obstacles)
    return m
