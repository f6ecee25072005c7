"""Scene / scenario / instance sharding across GPUs.

One process per GPU (``torch.distributed.run``), ``torch.distributed`` over RCCL — backend
"nccl" is RCCL on ROCm, its all-gather rides the xGMI links — and "gloo" for the CPU tests.
Every path here is independent per unit, so the data path has no collective; each helper
does exactly one all-gather at the end, the exchange step the north star names:

* multi-ego MPPI (configs[4]): scenes [a, b) per rank, one ``mp_mppi_plan`` launch for
  the rank's block with ``scene_base = a`` (the Philox counter word), so every scene draws
  the stream it would draw on one GPU; then an all-gather of the optimal controls
  (S×H×2 f64 — 6.4 KB per rank at 8 scenes × H=50) plus the per-scene scalars;
* Hybrid A* (configs[3]): a contiguous block of scenarios per rank (``HA_STRIDED``), each rank runs its
  own lockstep search (``mp_ha_plan``); all-gather of the outcome (found, pops, nodes, RS length) back
  into batch order;
* iLQR (configs[2]): instances [a, b) per rank (replicas of the solver); all-gather of
  J and the iteration counts.

Results are independent of the world size (the gloo tests check that against the
single-process oracle).  ``planner=`` lets the tests substitute the CPU oracle for the
device call; the default is always the libmpgpu entry point.
"""
import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Join the process group torch.distributed.run set up (RANK/WORLD_SIZE/MASTER_*).
    Returns (rank, world, local_rank); (0, 1, 0) when not launched distributed."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n, rank, world):
    """Balanced contiguous block [a, b) of n units for `rank` (the first n % world ranks
    take one extra)."""
    base, rem = divmod(n, world)
    a = rank * base + min(rank, rem)
    return a, a + base + (1 if rank < rem else 0)


# Hybrid A*'s split.  Round 4 defaulted to strided (every rank the same mix of perpendicular and parallel
# scenes); every one-GPU world-8 projection since measured the contiguous split ahead (round 5: 1.29-1.35x vs
# 1.12-1.25x, profiles/r05*_ha_*; the strided shard that draws the 729-pop scenario also draws more long
# searches), so round 5 returns to contiguous blocks.
HA_STRIDED = False


def shard_indices(n, rank, world, strided=False):
    """The units of `rank`: the contiguous block shard_bounds gives, or (strided) every world-th unit
    from `rank` on.  Both give rank r the same number of units (the first n % world ranks one extra)."""
    if strided:
        return np.arange(rank, n, world)
    a, b = shard_bounds(n, rank, world)
    return np.arange(a, b)


def all_gather_rows(local, n_total, device=None, strided=False):
    """Every rank's leading-axis rows (its shard_indices) gathered back into n_total rows in unit
    order.  Blocks are padded to the largest shard so one fixed-size collective suffices
    (all_gather_into_tensor on RCCL; all_gather on gloo)."""
    rank, world = _world()
    arr = np.ascontiguousarray(local)
    if world == 1:
        return arr.copy()
    rows = shard_bounds(n_total, 0, world)[1]  # largest shard
    tail = arr.shape[1:]
    dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                             if dist.get_backend() == "nccl" else torch.device("cpu"))
    t = torch.zeros((rows,) + tail, dtype=torch.from_numpy(arr[:0]).dtype, device=dev)
    if arr.shape[0]:
        t[: arr.shape[0]] = torch.from_numpy(arr).to(dev)
    if dist.get_backend() == "nccl":
        out = torch.empty((world * rows,) + tail, dtype=t.dtype, device=dev)
        dist.all_gather_into_tensor(out, t)
        parts = list(out.view((world, rows) + tail))
    else:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
    out = np.empty((n_total,) + tail, dtype=arr.dtype)
    for r in range(world):
        idx = shard_indices(n_total, r, world, strided)
        out[idx] = parts[r][: len(idx)].cpu().numpy()
    return out


def _params_copy(p):
    q = type(p)()
    ctypes.pointer(q)[0] = p
    return q


# ------------------------------------------------------------------- MPPI
def mppi_plan_sharded(p, X0, goal, U_nom, obstacles=None, grid=None, planner=None, ctx=None):
    """Multi-ego MPPIPlan: S scenes (replicated inputs) split across ranks; returns the
    gathered dict of mppi_plan_batch outputs for all S scenes on every rank."""
    from . import mppi

    rank, world = _world()
    X0 = np.asarray(X0, np.float64).reshape(-1, 7)
    S = X0.shape[0]
    a, b = shard_bounds(S, rank, world)
    q = _params_copy(p)
    q.scene_base = p.scene_base + a
    sl = slice(a, b)
    if b > a:
        args = (q, X0[sl], np.asarray(goal)[sl], np.asarray(U_nom)[sl],
                None if obstacles is None else np.asarray(obstacles)[sl], None if grid is None else np.asarray(grid)[sl])
        res = planner(*args) if planner is not None else mppi.mppi_plan_batch(*args, ctx=ctx)
    else:
        H = p.H
        res = dict(U=np.zeros((0, H, 2)), traj=np.zeros((0, H + 1, 7)), cost=np.zeros(0),
                   feasible=np.zeros(0, np.int32), rollout_count=np.zeros(0, np.int32),
                   feasible_count=np.zeros(0, np.int32))
    return {k: all_gather_rows(res[k], S) for k in ("U", "traj", "cost", "feasible", "rollout_count",
                                                   "feasible_count")}


# -------------------------------------------------------------- Hybrid A*
def hybrid_astar_sharded(searchers, planner=None, ctx=None, max_pops=5000):
    """planHybridAstar! over a batch of scenarios split across ranks (lockstep search per
    rank).  The rank's own searchers get their full results; every rank returns the gathered
    outcome arrays {found, pops, n_nodes, rs_len} for the whole batch."""
    from . import hybrid_astar as ha

    rank, world = _world()
    n = len(searchers)
    mine = [searchers[i] for i in shard_indices(n, rank, world, strided=HA_STRIDED)]
    if mine:
        (planner or (lambda hs: ha.plan_batch(hs, ctx=ctx, max_pops=max_pops)))(mine)
    out = np.array([[int(h.r.found), h.r.loop_count, h.r.n_nodes, h.r.RSpath_final.shape[1]] for h in mine],
                   np.int64).reshape(-1, 4)
    g = all_gather_rows(out, n, strided=HA_STRIDED)
    return dict(found=g[:, 0].astype(bool), pops=g[:, 1], n_nodes=g[:, 2], rs_len=g[:, 3])


def track_sharded(searchers, ctx=None, settings=None, runner=None):
    """retrievePath + the main_Tracker.jl loop for this rank's shard of a planned batch (the same
    split as hybrid_astar_sharded, so each rank tracks what it planned).  Every rank returns
    the gathered {status, n_steps} for the whole batch.  `runner(mine)` replaces the device calls
    (the gloo tests run the oracle there)."""
    from . import hybrid_astar as ha
    from . import tracker

    rank, world = _world()
    n = len(searchers)
    mine = [searchers[i] for i in shard_indices(n, rank, world, strided=HA_STRIDED)]
    if mine and runner is not None:
        runner(mine)
    elif mine:
        ha.retrieve_batch(mine, ctx=ctx)
        tracker.track_batch(mine, ctx=ctx, settings=settings)
    inv = {v: k for k, v in tracker.STATUS.items()}
    out = np.array([[inv[h.r.tracking["status"]], h.r.tracking["n_steps"]] for h in mine], np.int64).reshape(-1, 2)
    g = all_gather_rows(out, n, strided=HA_STRIDED)
    return dict(status=g[:, 0], n_steps=g[:, 1])


# ------------------------------------------------------------------ iLQR
def ilqr_solve_sharded(p, X, U, planner=None, ctx=None):
    """ilqr_solve over B instances split across ranks; returns gathered (X, U, J, iters)."""
    from . import ilqr

    rank, world = _world()
    X = np.asarray(X, np.float64).reshape(-1, p.N, 4)
    B = X.shape[0]
    a, b = shard_bounds(B, rank, world)
    if b > a:
        Xs, Us, J, it = (planner or (lambda p_, X_, U_: ilqr.ilqr_solve(p_, X_, U_, ctx=ctx)[:4]))(
            p, X[a:b], np.asarray(U, np.float64).reshape(B, p.N, 2)[a:b])
    else:
        Xs, Us, J, it = np.zeros((0, p.N, 4)), np.zeros((0, p.N, 2)), np.zeros(0), np.zeros(0, np.int32)
    return (all_gather_rows(Xs, B), all_gather_rows(Us, B), all_gather_rows(np.asarray(J, np.float64), B),
            all_gather_rows(np.asarray(it, np.int32), B))
