"""Tracker oracle (oracle/or_track.c): the Hybrid A* -> tracker hand-off and the tracker loop of
PathPlanning/HybridAstar/main_Tracker.jl:42-137 (src/tracker_utils.jl:1-43).

main_Tracker.jl writes no artifact, so the loop has no reference output to pin (parity unpinned vs
Julia; GPU-vs-oracle is bit-exact in tests/test_gpu_track.py).  Here the C restatement is checked
against an independent line-by-line Python restatement of the script (same FDLIBM libm through the
oracle's exported math), and against answers derivable from the text (a straight path is tracked
with zero cross-track error; the loop stops when the closest point is the last one).
"""
import math

import numpy as np
import pytest

import oracle
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd import tracker
from motionplanning_amd.configs import julia_linrange


def _planned(scene):
    h = ha.driver_searcher(scene)
    p = ha.params_of(h)
    sc, pc = oracle.ha_neighbor_origin(h.s.expand_time, h.s.steer_set, h.s.gear_set)
    r = oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
    assert r["found"]
    ret = oracle.ha_retrieve(h.s.starting_states, r["states"], r["rs_path"])
    return h, ret


def _params(n_ref=1000, max_steps=200_000, his_stride=0, veh_len=3.0):
    return tracker.params_of(tracker.TrackerSettings(n_ref=n_ref, max_steps=max_steps, veh_length=veh_len),
                             his_stride)


def _py_track(p, start, tol, samples, max_steps):
    """main_Tracker.jl:42-122 restated line by line in Python (scalar floats; FDLIBM via the oracle)."""
    cos, sin, tan, atan = (lambda x, f=f: oracle.m(f, x) for f in ("cos", "sin", "tan", "atan"))
    n, ns = p.n_ref, samples.shape[0]
    refined = julia_linrange(0.0, tol, n)

    def interp(s, q):  # linear_interpolation(LinRange(0, tol, ns), samples[:, q])(s)
        c = ((ns - 1) * (s - 0.0)) / (tol - 0.0) + 1.0
        f = math.floor(c)
        if c == ns:
            f -= 1
        f = min(max(f, 1), ns - 1)
        d = c - f
        return (1 - d) * samples[f - 1, q] + d * samples[f, q]

    ref = np.array([[interp(s, q) for q in range(3)] for s in refined])

    def argmin_abs(c):  # argmin(abs.(refined_length .- c)) = argmin(abs.(LinRange(0 - c, tol - c, n)))
        vals = [abs(v) for v in julia_linrange(0.0 - c, tol - c, n)]
        return int(np.argmin(vals))  # first minimum

    def findclosest(px, py, lo, hi):
        d = [(ref[i, 0] - px) ** 2 + (ref[i, 1] - py) ** 2 for i in range(lo, hi + 1)]
        return int(np.argmin(d)) + lo

    cur = [float(v) for v in start]
    least = least_look = 0
    eacc = 0.0
    sim = 0
    his = [list(cur)]
    while True:
        sim += 1
        if sim > max_steps:
            return "max_steps", sim, cur, eacc, his, ref
        maximum_idx = argmin_abs(sim * p.dt_sim + p.look_ahead)
        idx = findclosest(cur[0], cur[1], least, maximum_idx)
        if idx == n - 1:
            return "done", sim, cur, eacc, his, ref
        least = max(idx, argmin_abs(sim * p.dt_sim))
        rc, rn = ref[idx], ref[idx + 1]
        den = (refined[idx + 1] - refined[idx] + 1e-4) / 1
        dref = [(rn[q] - rc[q]) / den for q in range(3)]
        # inverseKinematic
        if abs(cos(rc[2])) >= math.sqrt(2) / 2:
            ux = dref[0] / cos(rc[2])
        else:
            ux = dref[1] / sin(rc[2])
        sa = atan((dref[2] / ux) * p.veh_len) if abs(ux) >= 0.01 else 0.0
        look = [p.look_ahead * cos(cur[2]), p.look_ahead * sin(cur[2])]
        look = [cur[0] + look[0], cur[1] + look[1]] if ux > 0 else [cur[0] - look[0], cur[1] - look[1]]
        maximum_look_idx = argmin_abs(sim * p.dt_sim + p.look_ahead * 2)
        look_idx = findclosest(look[0], look[1], least_look, maximum_look_idx)
        least_look = max(look_idx, argmin_abs(sim * p.dt_sim + p.look_ahead))
        vec1 = [cos(ref[look_idx, 2]), sin(ref[look_idx, 2])]
        vec2 = [look[0] - ref[look_idx, 0], look[1] - ref[look_idx, 1]]
        err = vec1[0] * vec2[1] - vec1[1] * vec2[0]
        eacc = eacc + err * p.dt_sim
        sa = sa + p.p_gain * (-err) + p.i_gain * (-eacc)
        sa = min(max(sa, -p.max_sa), p.max_sa)
        k = [ux * cos(cur[2]), ux * sin(cur[2]), ux / p.veh_len * tan(sa)]
        cur = [cur[q] + k[q] * p.dt_sim for q in range(3)]
        his.append(list(cur))


@pytest.mark.parametrize("scene", ["perpendicular", "parallel"])
def test_oracle_matches_python_restatement(scene):
    """The first 400 simulation steps of the driver scenes: C oracle == Python restatement, bit for bit."""
    h, ret = _planned(ha.PERPENDICULAR if scene == "perpendicular" else ha.PARALLEL)
    steps = 400
    p = _params(max_steps=steps, his_stride=1, veh_len=float(h.s.vehicle_size[0]))
    got = oracle.track(p, h.s.starting_real, ret["tol_length"], ret["samples"], his_cap=steps + 1)
    status, sim, cur, eacc, his, ref = _py_track(p, h.s.starting_real, ret["tol_length"], ret["samples"], steps)
    assert np.array_equal(got["ref"], ref)
    assert got["status"] == tracker.MP_TRACK_MAXSTEP and status == "max_steps"
    assert got["n_steps"] == sim == steps + 1
    assert np.array_equal(got["his"], np.array(his))
    assert np.array_equal(got["final"], np.array(cur)) and got["err_acc"] == eacc


@pytest.mark.parametrize("scene", ["perpendicular", "parallel"])
def test_oracle_tracks_driver_scene_to_the_end(scene):
    """The whole loop: it ends when the closest point is the last one (main_Tracker.jl:84), after about
    tol_length / (1 m/s) of simulated time, with the vehicle near the end of the reference path."""
    h, ret = _planned(ha.PERPENDICULAR if scene == "perpendicular" else ha.PARALLEL)
    p = _params(his_stride=100)
    got = oracle.track(p, h.s.starting_real, ret["tol_length"], ret["samples"], his_cap=5000)
    assert got["status"] == tracker.MP_TRACK_DONE
    tol = ret["tol_length"]
    assert tol / p.dt_sim * 0.9 < got["n_steps"] < tol / p.dt_sim + 3 * p.look_ahead / p.dt_sim
    end = got["ref"][-1]
    assert math.hypot(got["final"][0] - end[0], got["final"][1] - end[1]) < 0.5
    assert np.isfinite(got["his"]).all() and got["his"].shape[0] == (got["n_steps"] - 1) // 100 + 1


def test_straight_path_zero_cross_track_error():
    """A straight reference along +x from the start: every look-ahead point is on the path, err = 0,
    the steering stays 0 and y, ψ stay exactly 0."""
    tol = 7.0
    s = julia_linrange(0.0, tol, 50)
    samples = np.c_[s, np.zeros(50), np.zeros(50)]
    p = _params(his_stride=1)
    got = oracle.track(p, [0.0, 0.0, 0.0], tol, samples, his_cap=20000)
    assert got["status"] == tracker.MP_TRACK_DONE and got["err_acc"] == 0.0
    assert (got["his"][:, 1] == 0).all() and (got["his"][:, 2] == 0).all()
    assert np.all(np.diff(got["his"][:, 0]) > 0)


def test_reference_endpoints_and_no_path():
    """x/y/ψ_ref starts at the first knot value exactly; a scenario without a path does not run."""
    h, ret = _planned(ha.PERPENDICULAR)
    ref = oracle.track_reference(ret["tol_length"], ret["samples"], 1000)
    assert np.array_equal(ref[0], ret["samples"][0])
    assert np.allclose(ref[-1], ret["samples"][-1], rtol=0, atol=1e-12)
    got = oracle.track(_params(his_stride=5), h.s.starting_real, 0.0, ret["samples"], his_cap=3)
    assert got["status"] == tracker.MP_TRACK_NOPATH and got["n_steps"] == 0
    assert np.array_equal(got["his"], np.array([h.s.starting_real]))


def test_time_argmin_window_guard():
    """The device's 8-candidate window for argmin(abs.(refined_length .- c)) (tracker.hip argmin_time_lane)
    equals the full scan whenever its guard s > 4E holds: random tol, n_ref and c, the window logic restated
    in numpy with the same float64 operations (lerp (1-t)a + tb, t = j/(n-1))."""
    r = np.random.default_rng(11)
    eps = 2.220446049250313e-16
    checked = 0
    for _ in range(3000):
        n = int(r.choice([2, 3, 37, 50, 1000, 2048]))
        tol = float(10 ** r.uniform(-4, 2.5))
        c = float(r.uniform(0, tol + 3)) if r.random() < 0.9 else float(r.choice([0.0, tol, tol / 2]))
        t = np.arange(n, dtype=np.float64) / float(n - 1)
        a, b = 0.0 - c, tol - c
        v = np.abs((1 - t) * a + t * b)
        full = int(np.argmin(v))
        E = 8 * eps * (abs(c) + abs(tol - c) + abs(tol - c) + tol)
        if not tol / (n - 1) > 4 * E:
            continue
        g = min(max(np.rint(c * ((n - 1) / tol)), 0.0), n - 1.0)
        js = np.clip(int(g) - 3 + np.arange(8), 0, n - 1)
        win = int(js[np.argmin(v[js])])
        assert win == full, (n, tol, c)
        checked += 1
    assert checked > 2500
