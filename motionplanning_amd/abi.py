"""ctypes mirror of include/mpgpu.h and the loader for libmpgpu.so.

This is the Python side of the drop-in boundary: the same entry points the
Julia wrapper (julia/MPGPU.jl) binds with `ccall`.  The shared library is built
in-tree by ``__graft_entry__.build()`` (``motionplanning_amd/lib/libmpgpu.so``).
There is no fallback: if the library is missing or fails to load, every
planner call raises ``MPGPUError`` (no silent CPU path).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmpgpu.so")
LIB_PATH = os.environ.get("MPGPU_LIB") or LIB_PATH  # alternate builds (A/B experiments)

MP_OK = 0
MP_ERR_INVALID = 1
MP_ERR_HIP = 2
MP_ERR_NOMEM = 3
MP_ERR_NUMERIC = 4
MP_ERR_UNSUPPORTED = 5

MP_NOISE_EXTERNAL = 0
MP_NOISE_PHILOX = 1

MP_ILQR_OPTIMALCONTROL = 0
MP_ILQR_PARKING = 1

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int32_p = ctypes.POINTER(ctypes.c_int32)
c_int64_p = ctypes.POINTER(ctypes.c_int64)
c_uint8_p = ctypes.POINTER(ctypes.c_uint8)


class MPGPUError(RuntimeError):
    """Non-zero status from libmpgpu (message from mp_last_error)."""

    def __init__(self, status, msg):
        super().__init__(f"libmpgpu status {status}: {msg}")
        self.status = status


class MPPIParams(ctypes.Structure):
    """mp_mppi_params (include/mpgpu.h) — fields mirror MPPISetting, MPPI/src/types.jl:10-31."""

    _fields_ = [
        ("K", ctypes.c_int32),
        ("H", ctypes.c_int32),
        ("feasibility_count", ctypes.c_int32),
        ("n_obs", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("lambda_", ctypes.c_double),
        ("sigma", ctypes.c_double * 4),
        ("XL", ctypes.c_double * 7),
        ("XU", ctypes.c_double * 7),
        ("CL", ctypes.c_double * 2),
        ("CU", ctypes.c_double * 2),
        ("slack_penalty", ctypes.c_double),
        ("obs_penalty", ctypes.c_double),
        ("grid_nx", ctypes.c_int32),
        ("grid_ny", ctypes.c_int32),
        ("grid_x0", ctypes.c_double),
        ("grid_y0", ctypes.c_double),
        ("grid_dx", ctypes.c_double),
        ("grid_dy", ctypes.c_double),
        ("noise_mode", ctypes.c_int32),
        ("ctrl_cost", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("offset", ctypes.c_uint64),
        ("scene_base", ctypes.c_int32),
        ("final_stream", ctypes.c_int32),
        ("calls_in_flight", ctypes.c_int32),
    ]


class MPPILoopParams(ctypes.Structure):
    """mp_mppi_loop_params (include/mpgpu.h) — the closed-loop settings of MPPI/main.jl:14-19,55,80."""

    _fields_ = [
        ("update_steps", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("plant_dt", ctypes.c_double),
        ("goal_radius", ctypes.c_double),
        ("poll_every", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class ILQRParams(ctypes.Structure):
    """mp_ilqr_params (include/mpgpu.h) — OptimalControl/ILQR/ILQR.jl:12-18 settings."""

    _fields_ = [
        ("N", ctypes.c_int32),
        ("variant", ctypes.c_int32),
        ("dT", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("alpha_floor", ctypes.c_double),
        ("tol", ctypes.c_double),
        ("max_iter", ctypes.c_int32),
        ("max_ls", ctypes.c_int32),
    ]


class HAParams(ctypes.Structure):
    """mp_ha_params (include/mpgpu.h) — HybridAstarSettings, HybridAstar/src/types.jl:20-43."""

    _fields_ = [
        ("vehicle_len", ctypes.c_double),
        ("vehicle_wid", ctypes.c_double),
        ("minR", ctypes.c_double),
        ("expand_time", ctypes.c_double),
        ("res", ctypes.c_double * 3),
        ("stbound", ctypes.c_double * 6),
        ("n_walls", ctypes.c_int32),
        ("n_prim", ctypes.c_int32),
        ("n_col", ctypes.c_int32),
        ("max_pops", ctypes.c_int32),
    ]


class TrackParams(ctypes.Structure):
    """mp_track_params (include/mpgpu.h) — the tracker settings of HybridAstar/main_Tracker.jl:42-72."""

    _fields_ = [
        ("n_ref", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("dt_sim", ctypes.c_double),
        ("look_ahead", ctypes.c_double),
        ("p_gain", ctypes.c_double),
        ("i_gain", ctypes.c_double),
        ("veh_len", ctypes.c_double),
        ("max_sa", ctypes.c_double),
        ("his_stride", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


MP_TRACK_DONE = 0
MP_TRACK_MAXSTEP = 1
MP_TRACK_NOPATH = 2
MP_TRACK_EMPTY = 3

# (name, restype, argtypes) for every symbol declared in include/mpgpu.h
_V = ctypes.c_void_p
_I = ctypes.c_int32
SIGNATURES = {
    "mp_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_V)]),
    "mp_ctx_destroy": (ctypes.c_int, [_V]),
    "mp_last_error": (ctypes.c_char_p, [_V]),
    "mp_version": (ctypes.c_char_p, []),
    "mp_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mp_ctx_synchronize": (ctypes.c_int, [_V]),
    "mp_ctx_join": (ctypes.c_int, [_V]),
    "mp_ctx_stream": (_V, [_V]),
    "mp_ctx_kernel_timing": (ctypes.c_int, [_V, ctypes.c_int]),
    "mp_ctx_kernel_ms": (ctypes.c_int, [_V, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)]),
    "mp_ctx_trim": (ctypes.c_int, [_V, ctypes.c_size_t]),
    "mp_ctx_set_workspace_limit": (ctypes.c_int, [_V, ctypes.c_size_t]),
    "mp_mppi_plan": (ctypes.c_int, [_V, ctypes.POINTER(MPPIParams), _I] + [_V] * 16),
    "mp_mppi_plan_dev": (ctypes.c_int, [_V, ctypes.POINTER(MPPIParams), _I] + [_V] * 16),
    "mp_rollout": (ctypes.c_int, [_V, ctypes.POINTER(MPPIParams), _I, _I, _V, _V, _V, ctypes.c_int64]
                   + [_V] * 7),
    "mp_vehicle_euler": (ctypes.c_int, [_V, _I, _V, _V, ctypes.c_double, _I, _V]),
    "mp_mppi_closed_loop": (ctypes.c_int, [_V, ctypes.POINTER(MPPIParams), ctypes.POINTER(MPPILoopParams), _I]
                            + [_V] * 15),
    "mp_ilqr_rollout": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I, _V, _V, _V, _V]),
    "mp_ilqr_backward": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I, _V, _V, _V, _V]),
    "mp_ilqr_forward": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I] + [_V] * 8),
    "mp_ilqr_backward_dev": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I, _V, _V, _V, _V]),
    "mp_ilqr_forward_dev": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I] + [_V] * 8),
    "mp_ilqr_solve": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I, _V, _V, _V, _V]),
    "mp_ilqr_solve_dev": (ctypes.c_int, [_V, ctypes.POINTER(ILQRParams), _I, _V, _V, _V, _V]),
    "mp_ha_set_primitives": (ctypes.c_int, [_V, ctypes.POINTER(HAParams), _V, _V]),
    "mp_ha_neighbor_origin": (ctypes.c_int, [_V, ctypes.POINTER(HAParams), _I, _V, _I, _V, _V, _V]),
    "mp_ha_expand": (ctypes.c_int, [_V, ctypes.POINTER(HAParams), _I] + [_V] * 7),
    "mp_ha_rs_connect": (ctypes.c_int, [_V, ctypes.POINTER(HAParams), _I] + [_V] * 6),
    "mp_ha_allpath": (ctypes.c_int, [_V, _I, _V, _V, _V, _V]),
    "mp_ha_sat_cull_active": (ctypes.c_int, [_V, ctypes.POINTER(HAParams), _I, _V, _V, _V, _V]),
    "mp_ha_plan": (ctypes.c_int, [_V, ctypes.POINTER(HAParams), _I] + [_V] * 11),
    "mp_ha_retrieve_path": (ctypes.c_int, [_V, _I, _V, _V, _V, _I] + [_V] * 8),
    "mp_ha_track": (ctypes.c_int, [_V, ctypes.POINTER(TrackParams), _I, _V, _V, _V, _I] + [_V] * 6 + [_I]),
    "mp_math_eval": (ctypes.c_int, [_V, _I, ctypes.c_int64, _V, _V, _V]),
    "mp_comm_init": (ctypes.c_int, [_V, _I]),
    "mp_comm_destroy": (ctypes.c_int, [_V, _I]),
    "mp_comm_allgather_dev": (ctypes.c_int, [_V, _I, _V, _V, ctypes.c_size_t]),
    "mp_mppi_plan_sharded": (ctypes.c_int, [_V, _I, ctypes.POINTER(MPPIParams), _I] + [_V] * 12),
}

_lib = None


def load_library(path=LIB_PATH):
    """Load libmpgpu.so (raises MPGPUError when absent — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MPGPUError(-1, f"{path} not built; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def ptr(a):
    """Raw data pointer of a C-contiguous numpy array (None passes NULL)."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if hasattr(a, "data_ptr"):  # torch tensor (device pointers for *_dev calls)
        return a.data_ptr()
    assert a.flags["C_CONTIGUOUS"], "arrays must be C-contiguous"
    return a.ctypes.data


def f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a
