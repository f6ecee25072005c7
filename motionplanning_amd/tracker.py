"""The Hybrid A* -> tracker hand-off and the path-tracker closed loop on the device
(PathPlanning/HybridAstar/main_Tracker.jl:42-137, src/tracker_utils.jl:1-43) through mp_ha_track.

The reference runs the tracker as a script over one planned `hybrid_astar`; here `track_batch`
takes any number of planned + retrieved searchers (`hybrid_astar.plan_batch` then
`hybrid_astar.retrieve_batch`) and tracks all of them in one launch, one wavefront each.
"""
import ctypes
import math
from dataclasses import dataclass

import numpy as np

from .abi import MP_TRACK_DONE, MP_TRACK_EMPTY, MP_TRACK_MAXSTEP, MP_TRACK_NOPATH, TrackParams, f64, ptr
from .context import default_context

STATUS = {MP_TRACK_DONE: "done", MP_TRACK_MAXSTEP: "max_steps", MP_TRACK_NOPATH: "no path",
          MP_TRACK_EMPTY: "empty window"}


@dataclass
class TrackerSettings:
    """main_Tracker.jl:42-72 (veh_param = [veh_length, veh_width, max_sa], :50-53)."""

    n_ref: int = 1000              # refined_length = LinRange(0, tol_length, 1000) (:42)
    look_ahead_dist: float = 1.0   # (:57)
    p_gain: float = 10.0           # (:58)
    i_gain: float = 0.1            # (:59)
    dt_sim: float = 1e-3           # (:67)
    veh_length: float = 3.0        # vehicle_size[1] (main_hybrid_astar.jl:21)
    max_sa: float = math.pi / 6 + 0.1  # max_δf + 0.1 (:52, main_hybrid_astar.jl:22)
    max_steps: int = 200_000       # safety cap (the reference loops until the last point is closest)


def params_of(st: TrackerSettings, his_stride=0):
    p = TrackParams()
    p.n_ref = st.n_ref
    p.max_steps = st.max_steps
    p.dt_sim = st.dt_sim
    p.look_ahead = st.look_ahead_dist
    p.p_gain = st.p_gain
    p.i_gain = st.i_gain
    p.veh_len = st.veh_length
    p.max_sa = st.max_sa
    p.his_stride = his_stride
    return p


def settings_for(h, **kw):
    """Tracker settings for a planned searcher: veh_length = vehicle_size[1] (main_Tracker.jl:50)."""
    st = TrackerSettings(**kw)
    if "veh_length" not in kw:
        st.veh_length = float(h.s.vehicle_size[0])
    return st


def track_batch(searchers, ctx=None, settings=None, his_stride=0, his_cap=0):
    """Track every planned searcher's reference path from its starting_real (main_Tracker.jl:63-122).

    Needs `retrieve_batch` first (r.tol_length, r.interp_values).  Fills r.tracking =
    dict(status, n_steps, states_his (rows, 3), final_state, err_accumulated, x_ref/y_ref/ψ_ref).
    Without `settings`, each searcher is tracked with its own vehicle length (veh_param[1] =
    vehicle_size[1], main_Tracker.jl:50): the batch is split into one launch per distinct length."""
    ctx = ctx or default_context()
    if settings is not None:
        return _track_group(searchers, ctx, settings, his_stride, his_cap)
    groups = {}
    for h in searchers:
        groups.setdefault(float(h.s.vehicle_size[0]), []).append(h)
    for hs in groups.values():
        _track_group(hs, ctx, settings_for(hs[0]), his_stride, his_cap)
    return searchers


def _track_group(searchers, ctx, st, his_stride, his_cap):
    B = len(searchers)
    start = f64([h.s.starting_real for h in searchers])
    tol = np.array([h.r.tol_length if h.r.found and h.r.interp_values is not None else 0.0 for h in searchers])
    ns = 50
    smp = np.zeros((B, ns, 3))
    for b, h in enumerate(searchers):
        if tol[b] > 0:
            smp[b] = h.r.interp_values
    p = params_of(st, his_stride if his_cap else 0)
    n_steps = np.zeros(B, np.int32)
    status = np.zeros(B, np.int32)
    fin = np.zeros((B, 3))
    ea = np.zeros(B)
    ref = np.zeros((B, st.n_ref, 3))
    his = np.zeros((B, his_cap, 3)) if his_cap else None
    ctx.check(ctx.lib.mp_ha_track(ctx.handle, ctypes.byref(p), B, ptr(start), ptr(tol), ptr(smp), ns, ptr(n_steps),
                                  ptr(status), ptr(fin), ptr(ea), ptr(ref), ptr(his), his_cap))
    for b, h in enumerate(searchers):
        n = int(n_steps[b])
        rows = 0
        if his_cap:
            rows = 1 if n == 0 else min(his_cap, (n - 1) // his_stride + 1)
        h.r.tracking = dict(status=STATUS[int(status[b])], n_steps=n, final_state=fin[b].copy(),
                            err_accumulated=float(ea[b]), x_ref=ref[b, :, 0].copy(), y_ref=ref[b, :, 1].copy(),
                            ψ_ref=ref[b, :, 2].copy(),
                            states_his=his[b, :rows].T.copy() if his_cap else None)
    return searchers
