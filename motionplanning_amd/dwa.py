"""Dynamic Window planner on the same rollout kernel — mirror of
OptimalControl/DynamicWindow/src/{types,setup,DWAUtils}.jl,
plus the reference's closed-loop drivers (DynamicWindow/main.jl:139-161,
MPPI/main.jl:238-266) with the 1 kHz Euler plant on the device.
"""
import time
from dataclasses import dataclass, field

import numpy as np

from . import configs
from .rollout import rollout_batch, vehicle_euler


@dataclass
class DWASetting:
    """DynamicWindow/src/types.jl:10-26."""

    numStates: int = 0
    numControls: int = 0
    X0: np.ndarray = None
    XL: np.ndarray = None
    XU: np.ndarray = None
    CL: np.ndarray = None
    CU: np.ndarray = None
    dt: float = 0.0
    T: float = 0.0
    N: int = 20
    goal: np.ndarray = None
    obstacle_list: list = field(default_factory=list)
    SlackPenalty: float = 1e5
    SampleNumber: list = field(default_factory=list)
    ControlSamples: np.ndarray = None


@dataclass
class DWAResult:
    Traj: np.ndarray = None
    Control: np.ndarray = None
    Feasibility: str = "InFeasible"
    cost: float = 1e6
    time: float = 0.0
    best_index: int = -1


@dataclass
class DWASearcher:
    s: DWASetting = field(default_factory=DWASetting)
    r: DWAResult = field(default_factory=DWAResult)


def defineDWA(numStates=0, numControls=0, X0=None, goal=None, SampleNumber=(10, 10), T=3.0, XL=None, XU=None,
              CL=None, CU=None):
    """DynamicWindow/src/setup.jl:3-52 (same validation as the reference)."""
    if numControls <= 0:
        raise ValueError(f"Controls ({numControls}) must be > 0")
    if numStates <= 0:
        raise ValueError(f"States ({numStates}) must be > 0")
    for name, v, n in (("X0", X0, numStates), ("XL", XL, numStates), ("XU", XU, numStates), ("CL", CL, numControls),
                       ("CU", CU, numControls)):
        if v is None or len(v) != n:
            raise ValueError(f"Length of {name} must match number of {'states' if n == numStates else 'controls'} ({n})")
    d = DWASearcher()
    s = d.s
    s.numStates, s.numControls = numStates, numControls
    s.X0, s.goal = np.asarray(X0, np.float64), np.asarray(goal, np.float64)
    s.XL, s.XU = np.asarray(XL, np.float64), np.asarray(XU, np.float64)
    s.CL, s.CU = np.asarray(CL, np.float64), np.asarray(CU, np.float64)
    s.T = float(T)
    s.dt = s.T / s.N
    s.SampleNumber = list(SampleNumber)
    s.ControlSamples = configs.dwa_control_samples(s.CL, s.CU, s.SampleNumber)
    return d


def defineDWAobs_(dwa, obstacle_list):
    dwa.s.obstacle_list = [list(map(float, o)) for o in obstacle_list]


def ShiftInitialCondition(dwa, X0):
    dwa.s.X0 = np.asarray(X0, np.float64)


def DWAPlan(dwa, ctx=None):
    """DWAUtils.jl:141-163: roll out every constant control, keep `minimum` by cost."""
    s = dwa.s
    t1 = time.time()
    p = configs.mppi_params(K=len(s.ControlSamples), H=s.N, T=s.T, XL=s.XL, XU=s.XU, CL=s.CL, CU=s.CU,
                            n_obs=len(s.obstacle_list), obs_penalty=configs.DWA_OBS_PENALTY, ctrl_cost=0,
                            dt=s.dt)
    obst = np.asarray(s.obstacle_list, np.float64).reshape(1, -1, 3) if s.obstacle_list else None
    r = rollout_batch(p, s.X0[None], s.goal[None], s.ControlSamples[None], obstacles=obst, want_argmin=True,
                      ctx=ctx)
    best = int(r["argmin"][0])
    dwa.r.best_index = best
    dwa.r.Control = s.ControlSamples[best].copy()
    dwa.r.cost = float(r["cost"][0, best])
    dwa.r.Feasibility = "Feasible" if r["feas"][0, best] else "InFeasible"
    dwa.r.time = time.time() - t1
    return None


def reference_dwa():
    """The searcher of DynamicWindow/main.jl:7-26."""
    d = defineDWA(7, 2, configs.X0_REF, configs.GOAL_REF, configs.DWA_SAMPLES, 3.0, configs.XL_REF,
                  configs.XU_REF, configs.CL_DWA, configs.CU_DWA)
    defineDWAobs_(d, configs.OBSTACLES_REF)
    return d


def run_dwa_closed_loop(dwa=None, horizon_s=15.0, update_time=0.1, dt=1e-3, goal_radius=7.2, ctx=None):
    """DynamicWindow/main.jl:139-161 — replan every update_time, Euler plant at dt; returns
    states_his (rows [t, x...]) and the chosen control index per replan."""
    dwa = dwa or reference_dwa()
    update_idx = int(np.floor(update_time / dt))
    goal = dwa.s.goal
    state = dwa.s.X0.copy()
    rows = [np.r_[0.0, state]]
    picks = []
    nsteps = int(np.floor(horizon_s / dt))
    t = 1
    while t <= nsteps:
        ShiftInitialCondition(dwa, state)
        DWAPlan(dwa, ctx=ctx)
        picks.append(dwa.r.best_index)
        n = min(update_idx, nsteps - t + 1)
        s, his = vehicle_euler(state, dwa.r.Control, dt, n, ctx=ctx)
        stop = False
        for i in range(n):
            rows.append(np.r_[(t + i) * dt, his[0, i]])
            if (his[0, i, 0] - goal[0]) ** 2 + (his[0, i, 1] - goal[1]) ** 2 <= goal_radius ** 2:
                stop = True
                break
        if stop:
            break
        state = s[0]
        t += n
    return np.array(rows), np.array(picks)
