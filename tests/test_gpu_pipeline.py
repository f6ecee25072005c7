"""GPU: the deferred final rollout (mp_mppi_params.final_stream = 1).

The final TrajectoryRollout(MPPICtrl) (MPPIUtils.jl:192-198) then runs on the context's side
stream from a device snapshot of its inputs, overlapping the next call's rollouts.  Its
outputs must be BIT-IDENTICAL to the in-kernel tail (final_stream = 0): same rollout_pair,
same inputs.  The pipelined test overwrites the input buffers right after each call (in
context-stream order) to prove the side stream reads the snapshot, not the live inputs.
"""
import ctypes

import numpy as np
import pytest
import torch

from motionplanning_amd import configs
from motionplanning_amd.abi import MP_NOISE_PHILOX, ptr
from motionplanning_amd.mppi import mppi_plan_batch

pytestmark = pytest.mark.gpu

KEYS = ("U", "traj", "cost", "feasible", "rollout_count", "feasible_count")


def _scenes(S, H, n_obs, seed):
    r = np.random.default_rng(seed)
    X0 = np.tile(configs.X0_REF, (S, 1))
    X0[:, 1] = r.uniform(-0.5, 0.5, S)
    goal = np.tile(configs.GOAL_REF, (S, 1))
    un = r.uniform(-0.1, 0.1, (S, H, 2))
    obs = np.stack([np.array(configs.OBSTACLES_CFG1)[:n_obs] + [[r.uniform(-1, 1), 0, 0]] for _ in range(S)])
    return X0, goal, un, obs


@pytest.mark.parametrize("nx", [100, 300])  # 300x300 grid: snapshot too big for LDS, read from HBM
def test_final_stream_host_api_bitexact(ctx, nx):
    spec = configs.grid_spec(nx=nx, ny=nx)
    grid = configs.rasterize_circles(configs.OBSTACLES_CFG1, spec)
    p = configs.mppi_params(K=1000, H=30, T=4.5, n_obs=3, grid=spec, noise_mode=MP_NOISE_PHILOX, seed=9)
    S = 3
    X0, goal, un, obs = _scenes(S, 30, 3, 4)
    G = np.stack([grid] * S)
    outs = []
    for fs in (0, 1):
        p.final_stream = fs
        outs.append(mppi_plan_batch(p, X0, goal, un, obs, G, None, collect=True, ctx=ctx))
    for k in KEYS:
        assert np.array_equal(outs[0][k], outs[1][k]), k
    assert np.array_equal(outs[0]["coll"]["traj_soa"], outs[1]["coll"]["traj_soa"])


def test_final_stream_pipelined_dev(ctx):
    dev = torch.device("cuda", 0)
    stream = torch.cuda.ExternalStream(ctx.stream, device=dev)
    c = configs.cfg2(noise_mode=MP_NOISE_PHILOX, seed=77)
    p = c["params"]
    S, K, H, calls = 3, p.K, p.H, 4
    rng = np.random.default_rng(8)
    X0s = [np.tile(c["X0"], (S, 1)) + np.c_[np.zeros((S, 1)), rng.uniform(-0.5, 0.5, (S, 1)), np.zeros((S, 5))]
           for _ in range(calls)]
    uns = [rng.uniform(-0.1, 0.1, (S, H, 2)) for _ in range(calls)]
    G = np.stack([c["grid"]] * S)
    goal = np.tile(c["goal"], (S, 1))
    # reference: synchronous host calls with the in-kernel tail
    refs = []
    p.final_stream = 0
    for i in range(calls):
        p.offset = i
        refs.append(mppi_plan_batch(p, X0s[i], goal, uns[i], None, G, None, ctx=ctx))
    with torch.cuda.stream(stream):
        dX0 = torch.zeros((S, 7), dtype=torch.float64, device=dev)
        dun = torch.zeros((S, H, 2), dtype=torch.float64, device=dev)
        dgoal = torch.as_tensor(goal, device=dev)
        dgrid = torch.as_tensor(G, device=dev)
        outs = [dict(U=torch.empty((S, H, 2), dtype=torch.float64, device=dev),
                     traj=torch.empty((S, H + 1, 7), dtype=torch.float64, device=dev),
                     cost=torch.empty(S, dtype=torch.float64, device=dev),
                     feasible=torch.empty(S, dtype=torch.int32, device=dev),
                     rollout_count=torch.empty(S, dtype=torch.int32, device=dev),
                     feasible_count=torch.empty(S, dtype=torch.int32, device=dev)) for _ in range(calls)]
        torch.cuda.synchronize()
        p.final_stream = 1
        for i in range(calls):
            dX0.copy_(torch.as_tensor(X0s[i]), non_blocking=False)  # ordered on the context stream
            dun.copy_(torch.as_tensor(uns[i]))
            p.offset = i
            o = outs[i]
            ctx.check(ctx.lib.mp_mppi_plan_dev(
                ctx.handle, ctypes.byref(p), S, ptr(dX0), ptr(dgoal), ptr(dun), None, ptr(dgrid), None, ptr(o["U"]),
                ptr(o["traj"]), ptr(o["cost"]), ptr(o["feasible"]), ptr(o["rollout_count"]),
                ptr(o["feasible_count"]), None, None, None, None))
            dX0.fill_(1e3)  # clobber the live inputs before the side stream can have read them
            dun.fill_(5.0)
        ctx.check(ctx.lib.mp_ctx_join(ctx.handle))
        torch.cuda.synchronize()
    ctx.synchronize()
    for i in range(calls):
        for k in KEYS:
            assert np.array_equal(outs[i][k].cpu().numpy(), refs[i][k]), (i, k)
