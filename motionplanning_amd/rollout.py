"""Batched TrajectoryRollout (mp_rollout) and the closed-loop plant (mp_vehicle_euler)."""
import ctypes

import numpy as np

from .abi import MPPIParams, f64, ptr
from .context import default_context


def rollout_batch(p: MPPIParams, X0, goal, ctrl, U_nom=None, obstacles=None, grid=None, want_traj=False,
                  want_argmin=False, ctx=None):
    """TrajectoryRollout (MPPIUtils.jl:31-57 / DWAUtils.jl:16-42) for S scenes x K control lists.

    ctrl: (S, K, H, 2) per-step controls or (S, K, 2) constant controls (DWA).
    Returns dict(cost (S,K), feas (S,K) uint8, traj (S,K,H+1,7) | None, argmin (S,) | None).
    """
    ctx = ctx or default_context()
    X0 = f64(X0).reshape(-1, 7)
    S, H = X0.shape[0], p.H
    ctrl = f64(ctrl)
    const = ctrl.ndim == 3
    K = ctrl.shape[1]
    goal = f64(goal, (S, 2))
    U_nom = None if U_nom is None else f64(U_nom, (S, H, 2))
    obstacles = None if obstacles is None or p.n_obs == 0 else f64(obstacles, (S, p.n_obs, 3))
    grid = None if grid is None or p.grid_nx == 0 else np.ascontiguousarray(grid, np.uint8)
    cost = np.zeros((S, K))
    feas = np.zeros((S, K), np.uint8)
    traj = np.zeros((S, K, H + 1, 7)) if want_traj else None
    am = np.zeros(S, np.int32) if want_argmin else None
    ctx.check(ctx.lib.mp_rollout(ctx.handle, ctypes.byref(p), S, K, ptr(X0), ptr(goal), ptr(ctrl), 0 if const else 2,
                                 ptr(U_nom), ptr(obstacles), ptr(grid), ptr(traj), ptr(cost), ptr(feas), ptr(am)))
    return dict(cost=cost, feas=feas, traj=traj, argmin=am)


def vehicle_euler(states, ctrl, dt, nsteps, want_his=True, ctx=None):
    """Closed-loop plant (MPPI/main.jl:259-261): n vehicles, control held for nsteps Euler steps."""
    ctx = ctx or default_context()
    s = np.array(states, np.float64).reshape(-1, 7)
    c = f64(ctrl).reshape(-1, 2)
    n = s.shape[0]
    his = np.zeros((n, nsteps, 7)) if want_his else None
    ctx.check(ctx.lib.mp_vehicle_euler(ctx.handle, n, ptr(s), ptr(c), float(dt), int(nsteps), ptr(his)))
    return s, his
