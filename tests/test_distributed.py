"""World-size-2 gloo tests of the sharded paths (motionplanning_amd/distributed.py) on CPU.

The device call is replaced by the CPU oracle (``planner=``) so the sharding, the
scene_base Philox bookkeeping, uneven shards and the final all-gather run here without a
GPU; results must equal a single-process oracle run on the whole batch, bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from motionplanning_amd import configs
from motionplanning_amd import distributed as D
from motionplanning_amd import hybrid_astar as ha
from motionplanning_amd import ilqr
from motionplanning_amd.abi import MP_NOISE_PHILOX

S_MPPI, N_HA, B_ILQR = 5, 5, 5  # odd counts: uneven shards (3 + 2)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mppi_inputs():
    c = configs.cfg1()
    p = c["params"]
    p.noise_mode = MP_NOISE_PHILOX
    p.seed = 99
    X0 = np.tile(c["X0"], (S_MPPI, 1))
    X0[:, 1] = np.linspace(-1.0, 1.0, S_MPPI)
    goal = np.tile(c["goal"], (S_MPPI, 1))
    unom = np.zeros((S_MPPI, p.H, 2))
    obs = np.tile(c["obstacles"], (S_MPPI, 1, 1))
    return p, X0, goal, unom, obs


def _oracle_mppi(q, X0, goal, unom, obs, grid):
    rs = [oracle.mppi_plan(q, X0[i], goal[i], unom[i], obs[i], None, None, scene=i) for i in range(len(X0))]
    return dict(U=np.stack([r["U"] for r in rs]), traj=np.stack([r["traj"] for r in rs]),
                cost=np.array([r["cost"] for r in rs]), feasible=np.array([r["feasible"] for r in rs], np.int32),
                rollout_count=np.array([r["rollout_count"] for r in rs], np.int32),
                feasible_count=np.array([r["feasible_count"] for r in rs], np.int32))


def _ha_oracle_planner(hs):
    h0 = hs[0]
    p = ha.params_of(h0)
    sc, pc = oracle.ha_neighbor_origin(h0.s.expand_time, h0.s.steer_set, h0.s.gear_set)
    for h in hs:
        r = oracle.ha_plan(p, h.s.starting_states, h.s.ending_states, np.array(h.s.obstacle_list), sc, pc)
        h.r.found, h.r.loop_count, h.r.n_nodes = r["found"], r["pops"], r["n_nodes"]
        h.r.RSpath_final = r["rs_path"].T
        h.r.hybrid_astar_states = r["states"].T


TRACK_STEPS = 2000


def _track_oracle_runner(hs):
    from motionplanning_amd import tracker

    p = tracker.params_of(tracker.TrackerSettings(max_steps=TRACK_STEPS))
    for h in hs:
        tol, smp = 0.0, np.zeros((50, 3))
        if h.r.found:
            ret = oracle.ha_retrieve(h.s.starting_states, h.r.hybrid_astar_states.T, h.r.RSpath_final.T)
            tol, smp = ret["tol_length"], ret["samples"]
        t = oracle.track(p, h.s.starting_real, tol, smp)
        h.r.tracking = dict(status=tracker.STATUS[t["status"]], n_steps=t["n_steps"])


def _ilqr_inputs():
    p = ilqr.params(N=20)
    r = np.random.default_rng(3)
    x0 = np.c_[r.uniform(-1, 1, B_ILQR), 3.6 + r.uniform(-1, 1, B_ILQR), 5 + r.uniform(-1, 1, B_ILQR),
               r.uniform(-0.2, 0.2, B_ILQR)]
    U = ilqr.initial_controls(B_ILQR, p.N)
    X = np.zeros((B_ILQR, p.N, 4))
    for b in range(B_ILQR):
        X[b], _ = oracle.ilqr_rollout(p, x0[b], U[b])
    return p, X, U


def _ilqr_oracle_planner(p, X, U):
    out = [oracle.ilqr_solve(p, X[b], U[b]) for b in range(len(X))]
    return (np.stack([o[0] for o in out]), np.stack([o[1] for o in out]), np.array([o[2] for o in out]),
            np.array([o[3] for o in out], np.int32))


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, X0, goal, unom, obs = _mppi_inputs()
        m = D.mppi_plan_sharded(p, X0, goal, unom, obstacles=obs, planner=_oracle_mppi)
        hs = ha.scenario_batch(N_HA, seed=4)
        h = D.hybrid_astar_sharded(hs, planner=_ha_oracle_planner)
        t = D.track_sharded(hs, runner=_track_oracle_runner)
        pi, X, U = _ilqr_inputs()
        Xs, Us, J, it = D.ilqr_solve_sharded(pi, X, U, planner=_ilqr_oracle_planner)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **{f"m_{k}": v for k, v in m.items()},
                 **{f"h_{k}": v for k, v in h.items()},
                 **{f"t_{k}": v for k, v in t.items()}, i_X=Xs, i_U=Us, i_J=J, i_it=it)
    finally:
        dist.destroy_process_group()


def test_shard_bounds():
    for n in range(0, 20):
        for w in (1, 2, 3, 8):
            blocks = [D.shard_bounds(n, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


def test_shard_indices_partition():
    """Both splits partition 0..n-1 with the same shard sizes; the strided one gives every rank of the
    configs[3] batch (128 perpendicular scenes, then 128 parallel) the same mix of the two."""
    for n in range(0, 20):
        for w in (1, 2, 3, 8):
            for strided in (False, True):
                parts = [D.shard_indices(n, r, w, strided) for r in range(w)]
                assert sorted(np.concatenate(parts).tolist()) == list(range(n))
                assert [len(q) for q in parts] == [b - a for a, b in (D.shard_bounds(n, r, w) for r in range(w))]
    for r in range(8):
        idx = D.shard_indices(256, r, 8, strided=True)
        assert (idx < 128).sum() == 16 and (idx >= 128).sum() == 16


def test_params_copy_is_deep():
    p = configs.cfg1()["params"]
    q = D._params_copy(p)
    q.scene_base = 7
    assert p.scene_base == 0 and q.K == p.K and q.dt == p.dt


@pytest.mark.timeout(300)
def test_world2_gloo_matches_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    r0, r1 = (np.load(tmp_path / f"r{r}.npz") for r in range(world))
    for k in r0.files:  # every rank holds the same gathered arrays
        assert np.array_equal(r0[k], r1[k]), k
    # single-process oracle on the whole batch
    p, X0, goal, unom, obs = _mppi_inputs()
    ref = _oracle_mppi(p, X0, goal, unom, obs, None)
    for k, v in ref.items():
        assert np.array_equal(r0[f"m_{k}"], v), k
    assert len(set(map(tuple, r0["m_U"].reshape(S_MPPI, -1)))) == S_MPPI  # distinct streams per scene
    hs = ha.scenario_batch(N_HA, seed=4)
    _ha_oracle_planner(hs)
    assert np.array_equal(r0["h_found"], [h.r.found for h in hs])
    assert np.array_equal(r0["h_pops"], [h.r.loop_count for h in hs])
    assert np.array_equal(r0["h_n_nodes"], [h.r.n_nodes for h in hs])
    _track_oracle_runner(hs)  # the tracker hand-off of the planned shards, gathered
    from motionplanning_amd import tracker

    inv = {v: k for k, v in tracker.STATUS.items()}
    assert np.array_equal(r0["t_status"], [inv[h.r.tracking["status"]] for h in hs])
    assert np.array_equal(r0["t_n_steps"], [h.r.tracking["n_steps"] for h in hs])
    pi, X, U = _ilqr_inputs()
    Xs, Us, J, it = _ilqr_oracle_planner(pi, X, U)
    assert np.array_equal(r0["i_X"], Xs) and np.array_equal(r0["i_U"], Us)
    assert np.array_equal(r0["i_J"], J) and np.array_equal(r0["i_it"], it)
