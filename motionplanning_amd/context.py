"""Device context: one libmpgpu mp_ctx per (process, GPU)."""
import atexit
import ctypes
import threading
import weakref

from .abi import MP_OK, MPGPUError, load_library

_local = threading.local()


class Context:
    """Owns an mp_ctx (device, HIP stream, cached workspaces).  Not thread-safe."""

    def __init__(self, device=0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        st = self.lib.mp_ctx_create(int(device), ctypes.byref(h))
        if st != MP_OK:
            raise MPGPUError(st, self.lib.mp_last_error(None).decode())
        self.handle = h
        self.device = device
        _live.add(self)

    def check(self, st):
        if st != MP_OK:
            raise MPGPUError(st, self.lib.mp_last_error(self.handle).decode())
        return st

    def synchronize(self):
        self.check(self.lib.mp_ctx_synchronize(self.handle))

    def trim(self, keep_bytes=0):
        """Free cached device workspaces larger than keep_bytes (0: all) — mp_ctx_trim."""
        self.check(self.lib.mp_ctx_trim(self.handle, int(keep_bytes)))

    def set_workspace_limit(self, nbytes):
        """Cap any single device workspace at nbytes (0: no cap) — mp_ctx_set_workspace_limit."""
        self.check(self.lib.mp_ctx_set_workspace_limit(self.handle, int(nbytes)))

    @property
    def stream(self):
        return self.lib.mp_ctx_stream(self.handle)

    def close(self):
        """mp_ctx_destroy.  A context still joined to a communicator is refused (MPGPUError): close the
        CommGroup (mp_comm_destroy) first; the handle then stays valid."""
        if getattr(self, "handle", None):
            st = self.lib.mp_ctx_destroy(self.handle)
            if st != MP_OK:
                raise MPGPUError(st, self.lib.mp_last_error(self.handle).decode())
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CommGroup:
    """One host process driving several GPUs: a Context per device joined into one RCCL communicator
    (mp_comm_init, ncclCommInitAll) — the single-process multi-GPU path of include/mpgpu.h that a Julia
    host uses (torch.distributed's one-process-per-GPU path is motionplanning_amd/distributed.py)."""

    def __init__(self, devices):
        self.ctxs = [Context(d) for d in devices]
        self.lib = self.ctxs[0].lib
        self.n = len(self.ctxs)
        self.array = (ctypes.c_void_p * self.n)(*[c.handle.value for c in self.ctxs])
        st = self.lib.mp_comm_init(self.array, self.n)
        if st != MP_OK:
            raise MPGPUError(st, self.lib.mp_last_error(self.ctxs[0].handle).decode())
        self.live = True

    def check(self, st):
        if st != MP_OK:
            raise MPGPUError(st, self.lib.mp_last_error(self.ctxs[0].handle).decode())
        return st

    def close(self):
        if getattr(self, "live", False):
            self.lib.mp_comm_destroy(self.array, self.n)
            self.live = False
        for c in getattr(self, "ctxs", []):
            c.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_live = weakref.WeakSet()


@atexit.register
def _close_all():
    """Destroy every context still open at interpreter exit (synchronised, workspaces and streams released)
    while the HIP runtime is still up, instead of leaving them to garbage collection after it."""
    for c in list(_live):
        try:
            c.close()
        except Exception:
            pass


def default_context(device=None):
    """Per-thread default context on `device` (default: LOCAL_RANK or 0)."""
    import os

    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    ctxs = getattr(_local, "ctxs", None)
    if ctxs is None:
        ctxs = _local.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]
