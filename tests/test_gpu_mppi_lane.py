"""GPU parity of the one-rollout-per-lane plan kernel (LPR 1, dyn_lane).

The launch picks it by itself when S*K >= 131072 (16 scenes x 8192); MPGPU_LPR=1 forces it
here so the parity cases of test_gpu_mppi.py (same tolerances: rollouts, trajectories, flags
and counts bit-exact vs the oracle) run through it at oracle-friendly sizes."""
import os

import numpy as np
import pytest

import oracle
from motionplanning_amd import configs
from motionplanning_amd.abi import MP_NOISE_PHILOX
from motionplanning_amd.mppi import mppi_plan_batch

import test_gpu_mppi as base
from test_gpu_mppi import _check_plan

pytestmark = pytest.mark.gpu


@pytest.fixture
def lane(ctx):
    os.environ["MPGPU_LPR"] = "1"
    yield ctx
    del os.environ["MPGPU_LPR"]


def test_lane_cfg1(lane):
    base.test_cfg1_external_noise(lane)


def test_lane_nonzero_nominal(lane):
    base.test_reference_defaults_nonzero_nominal(lane)


@pytest.mark.parametrize("fc", [0, 300])
def test_lane_feasibility_prefix(lane, fc):
    base.test_feasibility_count_prefix(lane, fc)
    base.test_philox_feasibility_prefix(lane, fc)


def test_lane_multi_scene(lane):
    base.test_multi_scene(lane)


def test_lane_grid_philox_vs_pair(ctx):
    """cfg2 (grid, K=8192, H=50) x 2 scenes, device noise: LPR 1 and LPR 2 give identical
    TrajectoryCollections, costs and counts (bit-exact); MPPICtrl and the final rollout within the
    combine tolerance (the block partition differs: 256 vs 128 rollouts); scene 0 matches the oracle."""
    c = configs.cfg2(noise_mode=MP_NOISE_PHILOX, seed=3)
    p = c["params"]
    S = 2
    X0 = np.tile(c["X0"], (S, 1))
    X0[1, 1] = 0.3
    args = (p, X0, np.tile(c["goal"], (S, 1)), np.zeros((S, p.H, 2)), None, np.stack([c["grid"]] * S), None)
    outs = {}
    for lpr in ("1", "2"):
        os.environ["MPGPU_LPR"] = lpr
        try:
            outs[lpr] = mppi_plan_batch(*args, collect=True, ctx=ctx)
        finally:
            del os.environ["MPGPU_LPR"]
    for k in ("feasible", "rollout_count", "feasible_count"):
        assert np.array_equal(outs["1"][k], outs["2"][k]), k
    for k in ("U", "traj", "cost"):
        np.testing.assert_allclose(outs["1"][k], outs["2"][k], rtol=1e-9, atol=1e-12, err_msg=k)
    for k in ("traj_soa", "ctrl_soa", "cost", "feas"):
        assert np.array_equal(outs["1"]["coll"][k], outs["2"]["coll"][k]), k
    ref = oracle.mppi_plan(p, X0[0], c["goal"], np.zeros((p.H, 2)), None, c["grid"], None, collect=True)
    _check_plan(outs["1"], ref, 0)
