"""One process per GPU on one node, without an external launcher.

``python bench.py --gpus N`` (the driver's command) must run N ranks even when nothing set
``WORLD_SIZE``: the parent process, before it makes any GPU call, starts N fresh child
processes of the same command with the rendezvous environment ``torch.distributed.run``
would have given them (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``,
``MASTER_ADDR`` = 127.0.0.1, ``MASTER_PORT``), waits for all of them and exits with the
first non-zero status.  The children are started as subprocesses (never ``exec``), so the
parent never touches the GPU.
"""
import os
import socket
import subprocess
import sys
import time


def free_port():
    """A TCP port on 127.0.0.1 that was free a moment ago (the rendezvous store binds it)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    """The environment of local rank `rank` of a `world`-rank single-node job."""
    env = dict(os.environ if base is None else base)
    env.update({
        "RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
        "MASTER_PORT": str(port),
    })
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    return env


def spawn_local(world, cmd, port=None, timeout=None, poll_s=0.2):
    """Run `cmd` (argv list) as `world` local ranks and wait.  Returns the exit status: 0 when every
    rank succeeded, else the first failing rank's status (the others are terminated, so a rank that
    dies does not leave its peers blocked in a collective)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    port = port or free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(r, world, port)) for r in range(world)]
    t0 = time.monotonic()
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                status = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                status = 124
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return status


def relaunch_if_needed(n_gpus, argv=None):
    """When this process was not started as a rank (no WORLD_SIZE) and `n_gpus` > 1, run this same
    script as `n_gpus` ranks and return their exit status; else return None (the caller is a rank)."""
    if n_gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    argv = sys.argv if argv is None else argv
    return spawn_local(n_gpus, [sys.executable, "-u"] + list(argv))
