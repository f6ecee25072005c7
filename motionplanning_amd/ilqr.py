"""Batched iLQR — host-side mirror of the OptimalControl/ILQR script (ILQR.jl:11-88) and its
PathPlanning/Parking_ILQR variant, over the libmpgpu C-ABI (mp_ilqr_*).

The reference has no function surface (it is a script); this module names its steps:
initial roll out (ILQR.jl:31-37) -> ``ilqr_rollout``; one backward Riccati sweep
(:46-67) -> ``ilqr_backward``; one forward trial (:72-80) -> ``ilqr_forward``; the
whole loop (:39-88) -> ``ilqr_solve``.  Arrays are C-order (B, N, 4) / (B, N, 2).
"""
import ctypes

import numpy as np

from .abi import MP_ERR_NUMERIC, MP_ILQR_OPTIMALCONTROL, MP_ILQR_PARKING, ILQRParams, f64, ptr
from .context import default_context

X0_REF = [0.0, 3.6, 5.0, 0.0]  # ILQR.jl:12
U_INIT_REF = [-2.6, 0.01]  # ILQR.jl:33


def params(N=20, variant=MP_ILQR_OPTIMALCONTROL, dT=0.05, eps=1e-3, alpha_floor=None, tol=1e-6, max_iter=1000,
           max_ls=200):
    """ILQR.jl:15-16 defaults; the Parking variant floors the line search at 1e-3 (Parking_ILQR/ILQR.jl:83-85)."""
    p = ILQRParams()
    p.N, p.variant, p.dT, p.eps, p.tol = N, variant, dT, eps, tol
    p.alpha_floor = (1e-3 if variant == MP_ILQR_PARKING else 0.0) if alpha_floor is None else alpha_floor
    p.max_iter, p.max_ls = max_iter, max_ls
    return p


def initial_controls(B, N, u=U_INIT_REF):
    U = np.zeros((B, N, 2))
    U[:, : N - 1] = u
    return U


def cfg3_instances(B=4096, N=100, seed=3):
    """BASELINE configs[2] / SURVEY §8d cfg3 initial states x0 = [U(-1,1), 3.6+U(-1,1), 5+U(-1,1),
    U(-0.2,0.2)] (instance 0 = ILQR.jl:12's x0) and the ILQR.jl:33 initial guess."""
    r = np.random.default_rng(seed)
    x0 = np.c_[r.uniform(-1, 1, B), 3.6 + r.uniform(-1, 1, B), 5 + r.uniform(-1, 1, B), r.uniform(-0.2, 0.2, B)]
    x0[0] = X0_REF
    return x0, initial_controls(B, N)


def ilqr_rollout(p, x0, U, ctx=None):
    ctx = ctx or default_context()
    x0 = f64(x0).reshape(-1, 4)
    B = x0.shape[0]
    U = f64(U, (B, p.N, 2))
    X = np.zeros((B, p.N, 4))
    J = np.zeros(B)
    ctx.check(ctx.lib.mp_ilqr_rollout(ctx.handle, ctypes.byref(p), B, ptr(x0), ptr(U), ptr(X), ptr(J)))
    return X, J


def ilqr_backward(p, X, U, ctx=None):
    ctx = ctx or default_context()
    X = f64(X).reshape(-1, p.N, 4)
    B = X.shape[0]
    U = f64(U, (B, p.N, 2))
    k = np.zeros((B, p.N - 1, 2))
    K = np.zeros((B, p.N - 1, 4, 2))  # Julia 2x4 column-major per knot
    ctx.check(ctx.lib.mp_ilqr_backward(ctx.handle, ctypes.byref(p), B, ptr(X), ptr(U), ptr(k), ptr(K)))
    return k, K


def ilqr_forward(p, X, U, k, K, alpha, ctx=None):
    ctx = ctx or default_context()
    X = f64(X).reshape(-1, p.N, 4)
    B = X.shape[0]
    U, k, K = f64(U, (B, p.N, 2)), f64(k, (B, p.N - 1, 2)), f64(K, (B, p.N - 1, 4, 2))
    alpha = f64(np.broadcast_to(alpha, (B,)))
    Xn, Un, Jn = np.zeros_like(X), np.zeros_like(U), np.zeros(B)
    ctx.check(ctx.lib.mp_ilqr_forward(ctx.handle, ctypes.byref(p), B, ptr(X), ptr(U), ptr(k), ptr(K), ptr(alpha),
                                      ptr(Xn), ptr(Un), ptr(Jn)))
    return Xn, Un, Jn


def ilqr_solve(p, X, U, ctx=None, strict=False):
    """The ILQR.jl loop for every instance; returns (X, U, J, iters, ok)."""
    ctx = ctx or default_context()
    X = np.array(X, np.float64).reshape(-1, p.N, 4)
    B = X.shape[0]
    U = np.array(U, np.float64).reshape(B, p.N, 2)
    J = np.zeros(B)
    it = np.zeros(B, np.int32)
    st = ctx.lib.mp_ilqr_solve(ctx.handle, ctypes.byref(p), B, ptr(X), ptr(U), ptr(J), ptr(it))
    if st != MP_ERR_NUMERIC or strict:
        ctx.check(st)
    return X, U, J, it, st == 0


def ilqr_solve_dev(p, X, U, J, iters, ctx=None, strict=False):
    """ilqr_solve on device buffers (torch tensors in HBM: X (B, N, 4) and U (B, N, 2) f64 solved in place,
    J (B,) f64 and iters (B,) int32 written); returns ok (False: some instance hit max_iter / max_ls)."""
    ctx = ctx or default_context()
    B = X.shape[0]
    assert X.shape == (B, p.N, 4) and U.shape == (B, p.N, 2) and J.shape == (B,) and iters.shape == (B,)
    st = ctx.lib.mp_ilqr_solve_dev(ctx.handle, ctypes.byref(p), B, ptr(X), ptr(U), ptr(J), ptr(iters))
    if st != MP_ERR_NUMERIC or strict:
        ctx.check(st)
    return st == 0
