"""GPU parity at the edges: degenerate and ragged sizes, NaN and signed-zero inputs, and the C-ABI's
argument validation (the reference's `error()` checks, MPPI/src/setup.jl:19-38).

Tolerances as tests/test_gpu_mppi.py (rollouts bit-exact, MPPICtrl rtol 1e-9); NaN compares equal to
NaN (numpy assert_array_equal), signed zeros are compared bit for bit.
"""
import ctypes

import numpy as np
import pytest

import oracle
from motionplanning_amd import configs
from motionplanning_amd.abi import MP_ERR_INVALID, MPGPUError, MPPILoopParams, ptr
from motionplanning_amd.mppi import mppi_closed_loop_batch, mppi_plan_batch

from test_gpu_mppi import _check_plan

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.int64)


@pytest.mark.parametrize("K,H", [(1, 1), (1, 2), (3, 1), (129, 7)])
def test_plan_degenerate_and_ragged_sizes(ctx, K, H):
    """K = 1 (a single rollout: weight 1), H = 1 (terminal step only after one RK2 step), K one past a
    block of 128 lane pairs, odd H."""
    p = configs.mppi_params(K=K, H=H, T=0.15 * H, n_obs=3)
    r = np.random.default_rng(K * 100 + H)
    z = r.standard_normal((K, H, 2))
    un = r.uniform(-0.2, 0.2, (H, 2))
    X0, goal = np.array(configs.X0_REF), np.array(configs.GOAL_REF)
    obs = np.array(configs.OBSTACLES_REF)
    gpu = mppi_plan_batch(p, X0[None], goal[None], un[None], obs[None], None, z[None], collect=True, ctx=ctx)
    ref = oracle.mppi_plan(p, X0, goal, un, obs, None, z, collect=True)
    _check_plan(gpu, ref)
    if K == 1:  # one rollout, weight exp(0)/exp(0) = 1: MPPICtrl is its control list exactly
        assert np.array_equal(gpu["U"][0], gpu["coll"]["ctrl"][0, 0])


def test_plan_circles_and_grid_together(ctx):
    """Both obstacle representations in one scene (circle costs then the grid cost, MPPIUtils.jl:120-132
    order), a FeasibilityCount prefix inside the first block, S = 3 scenes."""
    spec = configs.grid_spec()
    grid = configs.rasterize_circles([[60.0, 0.0, 4.0], [20.0, 3.0, 2.0]], spec)
    p = configs.mppi_params(K=700, H=30, T=4.5, n_obs=5, grid=spec, feasibility_count=40)
    r = np.random.default_rng(8)
    S = 3
    X0 = np.tile(configs.X0_REF, (S, 1))
    X0[:, 0] = [0.0, 12.0, 45.0]
    goal = np.tile(configs.GOAL_REF, (S, 1))
    un = r.uniform(-0.1, 0.1, (S, 30, 2))
    obs = np.tile(np.array(configs.OBSTACLES_CFG1), (S, 1, 1))
    z = r.standard_normal((S, 700, 30, 2))
    G = np.tile(grid, (S, 1, 1))
    gpu = mppi_plan_batch(p, X0, goal, un, obs, G, z, collect=True, ctx=ctx)
    for s in range(S):
        ref = oracle.mppi_plan(p, X0[s], goal[s], un[s], obs[s], grid, z[s], collect=True)
        _check_plan(gpu, ref, s)


def test_nan_noise_propagates_like_julia(ctx):
    """A NaN draw stays NaN through PushInBounds (Julia's max/min propagate NaN; C fmax/fmin would clamp
    it to CL): that rollout's control and cost are NaN, findmin takes NaN as ρ, so every weight and
    MPPICtrl are NaN; the call reports MP_ERR_NUMERIC with every output written."""
    p = configs.mppi_params(K=200, H=10, T=1.5, n_obs=3)
    r = np.random.default_rng(3)
    z = r.standard_normal((200, 10, 2))
    z[37, 4, 1] = np.nan
    X0, goal, un = np.array(configs.X0_REF), np.array(configs.GOAL_REF), np.zeros((10, 2))
    obs = np.array(configs.OBSTACLES_REF)
    gpu = mppi_plan_batch(p, X0[None], goal[None], un[None], obs[None], None, z[None], collect=True, ctx=ctx)
    ref = oracle.mppi_plan(p, X0, goal, un, obs, None, z, collect=True)
    assert gpu["nan"] and ref["nan"]
    assert np.isnan(ref["coll"]["ctrl"][37, 4, 1]) and np.isnan(ref["coll"]["cost"][37])
    np.testing.assert_array_equal(gpu["coll"]["ctrl"][0], ref["coll"]["ctrl"])
    np.testing.assert_array_equal(gpu["coll"]["cost"][0], ref["coll"]["cost"])
    np.testing.assert_array_equal(gpu["coll"]["traj"][0], ref["coll"]["traj"])
    assert np.isnan(ref["U"]).all() and np.isnan(gpu["U"][0]).all()
    assert int(gpu["rollout_count"][0]) == ref["rollout_count"]


def test_signed_zero_clamp_like_julia(ctx):
    """With CL = 0.0 a sample of -0.0 is clamped to +0.0 (Julia: max(-0.0, 0.0) == 0.0): the device's
    v_max_f64 ordering of signed zeros against the oracle's mpj_jmax, bit for bit."""
    p = configs.mppi_params(K=64, H=4, T=0.6, n_obs=0, CL=[-0.5, 0.0], CU=[0.5, 2.5])
    z = np.random.default_rng(4).standard_normal((64, 4, 2))
    z[:8, :, :] = -0.0  # n = L z = -0.0 for both components
    un = np.full((4, 2), -0.0)
    X0, goal = np.array(configs.X0_REF), np.array(configs.GOAL_REF)
    gpu = mppi_plan_batch(p, X0[None], goal[None], un[None], None, None, z[None], collect=True, ctx=ctx)
    ref = oracle.mppi_plan(p, X0, goal, un, None, None, z, collect=True)
    assert bits(ref["coll"]["ctrl"][0, 0, 1]) == bits(0.0)  # Julia semantics in the oracle
    assert bits(ref["coll"]["ctrl"][0, 0, 0]) == bits(-0.0)  # inside [CL, CU]: unchanged
    assert np.array_equal(bits(gpu["coll"]["ctrl"][0]), bits(ref["coll"]["ctrl"]))
    assert np.array_equal(bits(gpu["coll"]["cost"][0]), bits(ref["coll"]["cost"]))


def _raw_plan(ctx, p, S=1, noise=True):
    K, H = p.K, p.H
    X0 = np.tile(configs.X0_REF, (S, 1))
    goal = np.tile(configs.GOAL_REF, (S, 1))
    un = np.zeros((S, max(H, 1), 2))
    z = np.zeros((S, max(K, 1), max(H, 1), 2)) if noise else None
    o = [np.zeros(n) for n in (S * max(H, 1) * 2, S * (max(H, 1) + 1) * 7, S)] + [np.zeros(S, np.int32)] * 3
    return ctx.lib.mp_mppi_plan(ctx.handle, ctypes.byref(p), S, ptr(X0), ptr(goal), ptr(un), None, None, ptr(z),
                                *[ptr(a) for a in o], None, None, None, None)


def test_abi_rejects_bad_arguments(ctx):
    """Every entry point validates before launching and leaves a message (mp_last_error), the
    reference's error() style; the context stays usable afterwards."""
    cases = [
        (dict(K=0, H=20, n_obs=0), True, "SamplingNumber"),
        (dict(K=16, H=0, n_obs=0, dt=0.15), True, "horizon"),
        (dict(K=16, H=5, n_obs=0, sigma=[-1.0, 0.0, 0.0, 0.1]), True, "positive definite"),
        (dict(K=16, H=5, n_obs=0), False, "noise"),
        (dict(K=16, H=5, n_obs=2), True, "obstacles"),  # obstacles NULL with n_obs > 0
    ]
    for kw, noise, word in cases:
        st = _raw_plan(ctx, configs.mppi_params(**kw), noise=noise)
        assert st == MP_ERR_INVALID, kw
        assert word in ctx.lib.mp_last_error(ctx.handle).decode(), kw
    # closed loop: a hold row outside [0, H)
    p = configs.mppi_params(K=16, H=5, n_obs=0)
    with pytest.raises(MPGPUError, match="hold_idx"):
        mppi_closed_loop_batch(p, np.array(configs.X0_REF)[None], np.array(configs.GOAL_REF)[None],
                               np.zeros((1, 5, 2)), np.full(10, 5, np.int32), 10, 20, 1e-3, 6.0, ctx=ctx)
    lp = MPPILoopParams(update_steps=0, max_steps=10, plant_dt=1e-3, goal_radius=1.0)
    st = ctx.lib.mp_mppi_closed_loop(ctx.handle, ctypes.byref(p), ctypes.byref(lp), 1, *([None] * 15))
    assert st == MP_ERR_INVALID
    # the context still works
    p = configs.mppi_params(K=16, H=5, n_obs=0)
    z = np.zeros((1, 16, 5, 2))
    out = mppi_plan_batch(p, np.array(configs.X0_REF)[None], np.array(configs.GOAL_REF)[None],
                          np.zeros((1, 5, 2)), None, None, z, ctx=ctx)
    assert np.isfinite(out["cost"]).all()
