"""World-size-2 run of the sharded paths on the GPU: two gloo ranks, both on cuda:0 (the one-GPU box's
rehearsal of the N-rank job), each calling libmpgpu for its own shard -- MPPI scenes (Philox streams
keyed by the global scene id), Hybrid A* scenarios (+ the tracker hand-off) and iLQR instances, uneven
shards -- then the all-gather.  Unlike tests/test_distributed.py (CPU, device call replaced by the
oracle), the device path itself runs here in two processes; every gathered output must equal the
single-process oracle on the whole batch, bit for bit (MPPICtrl within the plan's rtol 1e-9)."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from motionplanning_amd import distributed as D
from motionplanning_amd import hybrid_astar as ha

import test_distributed as T

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, outdir):
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, X0, goal, unom, obs = T._mppi_inputs()
        m = D.mppi_plan_sharded(p, X0, goal, unom, obstacles=obs)
        hs = ha.scenario_batch(T.N_HA, seed=4)
        h = D.hybrid_astar_sharded(hs)
        from motionplanning_amd import tracker

        t = D.track_sharded(hs, settings=tracker.TrackerSettings(max_steps=T.TRACK_STEPS))
        pi, X, U = T._ilqr_inputs()
        Xs, Us, J, it = D.ilqr_solve_sharded(pi, X, U)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **{f"m_{k}": v for k, v in m.items()},
                 **{f"h_{k}": v for k, v in h.items()},
                 **{f"t_{k}": v for k, v in t.items()}, i_X=Xs, i_U=Us, i_J=J, i_it=it)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_world2_device_shards_match_oracle(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, T._port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = (np.load(tmp_path / f"r{r}.npz") for r in range(world))
    for k in r0.files:
        assert np.array_equal(r0[k], r1[k]), k
    p, X0, goal, unom, obs = T._mppi_inputs()
    ref = T._oracle_mppi(p, X0, goal, unom, obs, None)
    for k, v in ref.items():
        if k == "U":
            np.testing.assert_allclose(r0["m_U"], v, rtol=1e-9, atol=1e-12)
        elif k in ("traj", "cost"):
            np.testing.assert_allclose(r0[f"m_{k}"], v, rtol=1e-9, atol=1e-12)
        else:
            assert np.array_equal(r0[f"m_{k}"], v), k
    hs = ha.scenario_batch(T.N_HA, seed=4)
    T._ha_oracle_planner(hs)
    assert np.array_equal(r0["h_found"], [h.r.found for h in hs])
    assert np.array_equal(r0["h_pops"], [h.r.loop_count for h in hs])
    assert np.array_equal(r0["h_n_nodes"], [h.r.n_nodes for h in hs])
    T._track_oracle_runner(hs)
    from motionplanning_amd import tracker

    inv = {v: k for k, v in tracker.STATUS.items()}
    assert np.array_equal(r0["t_status"], [inv[h.r.tracking["status"]] for h in hs])
    assert np.array_equal(r0["t_n_steps"], [h.r.tracking["n_steps"] for h in hs])
    pi, X, U = T._ilqr_inputs()
    Xs, Us, J, it = T._ilqr_oracle_planner(pi, X, U)
    assert np.array_equal(r0["i_X"], Xs) and np.array_equal(r0["i_U"], Us)
    assert np.array_equal(r0["i_J"], J) and np.array_equal(r0["i_it"], it)
