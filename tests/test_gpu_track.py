"""GPU parity of the Hybrid A* -> tracker hand-off and the tracker loop (mp_ha_track,
PathPlanning/HybridAstar/main_Tracker.jl:42-137) against the oracle (oracle/or_track.c), bit for bit:
reference points, step counts, statuses, final states, accumulated errors and states_his rows.
(main_Tracker.jl writes no artifact: parity unpinned vs Julia, see tests/test_oracle_track.py.)"""
import ctypes

import numpy as np
import pytest

import oracle
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd import tracker
from motionplanning_amd.abi import MPGPUError, ptr
from motionplanning_amd.configs import julia_linrange

pytestmark = pytest.mark.gpu


def _run(ctx, p, start, tol, samples, his_cap):
    B = len(tol)
    start = np.ascontiguousarray(start, np.float64)
    tol = np.ascontiguousarray(tol, np.float64)
    samples = np.ascontiguousarray(samples, np.float64)
    out = dict(n=np.zeros(B, np.int32), st=np.zeros(B, np.int32), fin=np.zeros((B, 3)), ea=np.zeros(B),
               ref=np.zeros((B, p.n_ref, 3)), his=np.zeros((B, his_cap, 3)) if his_cap else None)
    ctx.check(ctx.lib.mp_ha_track(ctx.handle, ctypes.byref(p), B, ptr(start), ptr(tol), ptr(samples),
                                  samples.shape[1], ptr(out["n"]), ptr(out["st"]), ptr(out["fin"]), ptr(out["ea"]),
                                  ptr(out["ref"]), ptr(out["his"]), his_cap))
    return out


def _check(p, out, start, tol, samples, his_cap):
    for b in range(len(tol)):
        r = oracle.track(p, start[b], tol[b], samples[b], his_cap=his_cap)
        assert out["st"][b] == r["status"], b
        assert out["n"][b] == r["n_steps"], b
        assert np.array_equal(out["fin"][b], r["final"]), b
        assert out["ea"][b] == r["err_acc"], b
        if r["status"] != tracker.MP_TRACK_NOPATH:
            assert np.array_equal(out["ref"][b], r["ref"]), b
        if his_cap:
            rows = r["his"].shape[0]
            assert np.array_equal(out["his"][b, :rows], r["his"]), b


def test_track_planned_batch_bitexact(ctx):
    """Plan (mp_ha_plan) -> retrieve (mp_ha_retrieve_path) -> track (mp_ha_track) for both driver scenes and
    a cfg4-shaped batch; scenarios without a path report MP_TRACK_NOPATH."""
    hs = [ha.driver_searcher(ha.PERPENDICULAR), ha.driver_searcher(ha.PARALLEL)] + ha.scenario_batch(22, seed=9)
    ha.plan_batch(hs, ctx=ctx)
    ha.retrieve_batch(hs, ctx=ctx)
    tracker.track_batch(hs, ctx=ctx, his_stride=50, his_cap=2000)
    st = tracker.settings_for(hs[0])
    p = tracker.params_of(st, 50)
    done = 0
    for h in hs:
        tr = h.r.tracking
        if not h.r.found:
            assert tr["status"] == "no path" and tr["n_steps"] == 0
            continue
        r = oracle.track(p, h.s.starting_real, h.r.tol_length, h.r.interp_values, his_cap=2000)
        assert tr["status"] == tracker.STATUS[r["status"]]
        assert tr["n_steps"] == r["n_steps"]
        assert np.array_equal(tr["final_state"], r["final"]) and tr["err_accumulated"] == r["err_acc"]
        assert np.array_equal(np.c_[tr["x_ref"], tr["y_ref"], tr["ψ_ref"]], r["ref"])
        assert np.array_equal(tr["states_his"].T, r["his"])
        done += tr["status"] == "done"
    assert done >= 10


def test_track_edges_bitexact(ctx):
    """n_ref 2 / 37 / 2048, a max_steps stop, a no-path row, a tiny path whose time argmins take the
    whole-wave fallback (the window guard fails), and a states_his buffer shorter than the run."""
    h = ha.driver_searcher(ha.PERPENDICULAR)
    ha.plan_batch([h], ctx=ctx)
    ha.retrieve_batch([h], ctx=ctx)
    s_line = julia_linrange(0.0, 1e-11, 50)
    line = np.c_[s_line, np.zeros(50), np.zeros(50)]
    start = np.array([h.s.starting_real, h.s.starting_real, [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]])
    tol = np.array([h.r.tol_length, 0.0, 1e-11, 4.0])
    s4 = julia_linrange(0.0, 4.0, 50)
    curve = np.c_[s4, 0.1 * s4 ** 2, np.arctan(0.2 * s4)]
    samples = np.stack([h.r.interp_values, h.r.interp_values, line, curve])
    for n_ref, max_steps, his_cap in ((1000, 200_000, 7), (2, 5000, 50), (37, 3000, 400), (2048, 1500, 2000)):
        p = tracker.params_of(tracker.TrackerSettings(n_ref=n_ref, max_steps=max_steps), 3)
        out = _run(ctx, p, start, tol, samples, his_cap)
        _check(p, out, start, tol, samples, his_cap)
        assert out["st"][1] == tracker.MP_TRACK_NOPATH
    assert out["st"][0] == tracker.MP_TRACK_MAXSTEP


def test_track_argument_checks(ctx):
    p = tracker.params_of(tracker.TrackerSettings(n_ref=4096), 0)
    z = np.zeros((1, 50, 3))
    with pytest.raises(MPGPUError):
        _run(ctx, p, np.zeros((1, 3)), np.ones(1), z, 0)
    p = tracker.params_of(tracker.TrackerSettings(), 0)  # states_his without a stride
    with pytest.raises(MPGPUError):
        _run(ctx, p, np.zeros((1, 3)), np.ones(1), z, 4)
