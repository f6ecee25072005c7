"""ORACLE — test infrastructure only.

ctypes access to the OpenBLAS that numpy ships (0.3.29, DYNAMIC_ARCH; SkylakeX kernels on this
host) through its Fortran interface -- dgemm_64_ / dgemv_64_ / ddot_64_, the ILP64 entry points
Julia's LinearAlgebra.BLAS ccalls.  It is the ground truth that pins oracle/or_blas.h (the rounding
of the reference's BLAS-dispatched products) in tests/test_oracle_blas.py and the Julia-dispatch
products of tools/ilqr_ulp_sources.py / tools/blas_replay.py.  Never used by the product.
"""
import ctypes
import glob
import os

import numpy as np

_lib = None
_i64 = ctypes.c_int64
_dp = ctypes.POINTER(ctypes.c_double)


def lib():
    """The numpy-bundled libscipy_openblas64_ (None when this numpy links another BLAS)."""
    global _lib
    if _lib is None:
        d = os.path.join(os.path.dirname(np.__file__), os.pardir, "numpy.libs")
        cands = sorted(glob.glob(os.path.join(d, "libscipy_openblas64_*.so")))
        if not cands:
            return None
        _lib = ctypes.CDLL(cands[0])
        _lib.scipy_ddot_64_.restype = ctypes.c_double
        f = _lib.scipy_openblas_get_config64_
        f.restype = ctypes.c_char_p
    return _lib


def config():
    L = lib()
    return None if L is None else L.scipy_openblas_get_config64_().decode()


def _p(a):
    return a.ctypes.data_as(_dp)


def _r(v):
    return ctypes.byref(_i64(v))


def gemm(A, B, ta=False, tb=False):
    """BLAS.gemm!('T'/'N', 'T'/'N', 1.0, A, B, 0.0, C) exactly as Julia calls it: op(A) * op(B),
    A and B given untransposed (column-major copies are made, the values are the same)."""
    A = np.asfortranarray(A, np.float64)
    B = np.asfortranarray(B, np.float64)
    if A.ndim == 1:
        A = A.reshape(-1, 1, order="F")
    if B.ndim == 1:
        B = B.reshape(-1, 1, order="F")
    m = A.shape[1] if ta else A.shape[0]
    k = A.shape[0] if ta else A.shape[1]
    n = B.shape[0] if tb else B.shape[1]
    assert (B.shape[1] if tb else B.shape[0]) == k
    C = np.zeros((m, n), order="F")
    one, zero = ctypes.c_double(1.0), ctypes.c_double(0.0)
    lib().scipy_dgemm_64_(ctypes.c_char_p(b"T" if ta else b"N"), ctypes.c_char_p(b"T" if tb else b"N"),
                          _r(m), _r(n), _r(k), ctypes.byref(one), _p(A), _r(A.shape[0]), _p(B), _r(B.shape[0]),
                          ctypes.byref(zero), _p(C), _r(m), ctypes.c_size_t(1), ctypes.c_size_t(1))
    return np.ascontiguousarray(C)


def gemv(A, x, t=False):
    """BLAS.gemv!('T'/'N', 1.0, A, x, 0.0, y): op(A) * x for a matrix A and a vector x."""
    A = np.asfortranarray(A, np.float64)
    x = np.ascontiguousarray(x, np.float64).ravel()
    m, n = A.shape
    assert len(x) == (m if t else n)
    y = np.zeros(n if t else m)
    one, zero = ctypes.c_double(1.0), ctypes.c_double(0.0)
    lib().scipy_dgemv_64_(ctypes.c_char_p(b"T" if t else b"N"), _r(m), _r(n), ctypes.byref(one), _p(A), _r(m),
                          _p(x), _r(1), ctypes.byref(zero), _p(y), _r(1), ctypes.c_size_t(1))
    return y


def dot(x, y):
    """BLAS.dot(x, y) (LinearAlgebra.dot of two Float64 vectors)."""
    x = np.ascontiguousarray(x, np.float64).ravel()
    y = np.ascontiguousarray(y, np.float64).ravel()
    return lib().scipy_ddot_64_(_r(len(x)), _p(x), _r(1), _p(y), _r(1))
