"""iLQR oracle (oracle/or_ilqr.c) checks.  Parity vs Julia is UNPINNED (no reference artifact,
SURVEY §8c); these tests pin the restatement against independent pure-Python restatements
of GetMatrix.jl / Dynamics.jl / Cost.jl / ILQR.jl (small N, loops; tools/ilqr_ulp_sources.py) and
the script's convergence behaviour."""
import math

import numpy as np
import pytest

import oracle
from motionplanning_amd import ilqr

LA, LB = 1.56, 1.64


def _dyn(s, u):
    x, y, ux, psi = s
    ax, d = u
    b = math.atan(LA / (LA + LB) * math.tan(d))
    return np.array([ux * math.cos(psi + b), ux * math.sin(psi + b), ax, ux * math.cos(b) * math.tan(d) / (LA + LB)])


def _rk4(s, u, dT):
    k1 = _dyn(s, u); k2 = _dyn(s + dT / 2 * k1, u); k3 = _dyn(s + dT / 2 * k2, u); k4 = _dyn(s + dT * k3, u)
    return 1 / 6 * (k1 + 2 * k2 + 2 * k3 + k4) * dT + s


def _sig(st, mn, mx):
    def e(v):
        try:
            return math.exp(v)
        except OverflowError:
            return math.inf
    return 100 * (1 / (1 + e(-10 * (st - mx))) + 1 / (1 + e(10 * (st - mn))))


def _stage(s, u):
    return 10 * u[0] ** 2 + 10 * u[1] ** 2 + 0.01 * s[2] ** 2 + _sig(u[1], -math.pi / 6, math.pi / 6) + _sig(u[0], -2, 2)


def _term(s, u=None):
    return 1000 * (s[0] ** 2 + s[1] ** 2 + 0.1 * s[2] ** 2 + s[3] ** 2)


def _calc(s, u, f, e=1e-3):
    n, m = 4, 2
    E, F = np.eye(n) * e, np.eye(m) * e
    lx = np.array([(f(s + E[i], u) - f(s - E[i], u)) / (2 * e) for i in range(n)])
    lu = np.array([(f(s, u + F[j]) - f(s, u - F[j])) / (2 * e) for j in range(m)])
    lxx = np.zeros((n, n))
    for i in range(n):
        for j in range(n):
            if i == j:
                lxx[i, j] = (1 / (12 * e ** 2)) * (-f(s + 2 * E[i], u) + 16 * f(s + E[i], u) - 30 * f(s, u)
                                                   + 16 * f(s - E[i], u) - f(s - 2 * E[i], u))
            else:
                lxx[i, j] = (1 / (4 * e ** 2)) * (f(s + E[i] + E[j], u) + f(s - E[i] - E[j], u)
                                                  - f(s + E[i] - E[j], u) - f(s - E[i] + E[j], u))
    luu = np.zeros((m, m))
    for i in range(m):
        for j in range(m):
            if i == j:
                luu[i, j] = (1 / (12 * e ** 2)) * (-f(s, u + 2 * F[i]) + 16 * f(s, u + F[i]) - 30 * f(s, u)
                                                   + 16 * f(s, u - F[i]) - f(s, u - 2 * F[i]))
            else:
                luu[i, j] = (1 / (4 * e ** 2)) * (f(s, u + F[i] + F[j]) + f(s, u - F[i] - F[j])
                                                  - f(s, u + F[i] - F[j]) - f(s, u - F[i] + F[j]))
    lux = np.array([[(1 / (4 * e ** 2)) * (f(s + E[j], u + F[i]) + f(s - E[j], u - F[i]) - f(s - E[j], u + F[i])
                                           - f(s + E[j], u - F[i])) for j in range(n)] for i in range(m)])
    return lx, lu, lxx, luu, lux


def _lin(s, u, dT, e=1e-3):
    A = np.zeros((4, 4)); B = np.zeros((4, 2))
    for i in range(4):
        d = np.zeros(4); d[i] = e
        A[:, i] = (_rk4(s + d, u, dT) - _rk4(s - d, u, dT)) / (2 * e)
    for j in range(2):
        d = np.zeros(2); d[j] = e
        B[:, j] = (_rk4(s, u + d, dT) - _rk4(s, u - d, dT)) / (2 * e)
    return A, B


def _setup(N=20):
    p = ilqr.params(N=N)
    U = ilqr.initial_controls(1, N)[0]
    X, J = oracle.ilqr_rollout(p, np.array(ilqr.X0_REF), U)
    return p, X, U, J


def test_rollout_matches_python():
    p, X, U, J = _setup()
    Xp = [np.array(ilqr.X0_REF)]
    for i in range(p.N - 1):
        Xp.append(_rk4(Xp[-1], U[i], p.dT))
    np.testing.assert_allclose(X, np.array(Xp), rtol=1e-13, atol=1e-13)
    Jp = sum(_stage(Xp[i], U[i]) for i in range(p.N - 1)) + _term(Xp[-1])
    assert abs(J - Jp) <= 1e-9 * abs(Jp)


def _model(**kw):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import ilqr_ulp_sources
    return ilqr_ulp_sources.Model(**kw)


@pytest.mark.skipif(__import__("oracle.openblas").openblas.lib() is None, reason="numpy without its OpenBLAS")
def test_backward_matches_independent_restatement():
    """k, K of the first sweep (ILQR.jl:46-67) vs tools/ilqr_ulp_sources.py, an independent Python
    restatement (Julia's `states .+ Δ` perturbations, matrix-shaped lx/Vx, its own loops): bit for bit
    with the oracle's rounding sources -- every product through numpy's OpenBLAS called as Julia calls it
    (oracle/openblas.py) against the oracle's default or_blas.h, and the sequential sums against
    or_blas = 0 -- and within 1e-10 with glibc trig/exp and numpy's own matmul choices."""
    p, X, U, _ = _setup()
    k, K = oracle.ilqr_backward(p, X, U)
    kk, KK = _model().backward(X, U, p.dT)
    assert np.array_equal(k, kk[:, :, 0]) and np.array_equal(K, np.swapaxes(KK, 1, 2))
    with oracle.blas_mode(0):
        k0, K0 = oracle.ilqr_backward(p, X, U)
    kk, KK = _model(prod="seq").backward(X, U, p.dT)
    assert np.array_equal(k0, kk[:, :, 0]) and np.array_equal(K0, np.swapaxes(KK, 1, 2))
    assert not np.array_equal(k0, k)  # the conventions differ in the last bits
    kk, KK = _model(trig="libm", exp="libm", prod="blas").backward(X, U, p.dT)
    np.testing.assert_allclose(k, kk[:, :, 0], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(K, np.swapaxes(KK, 1, 2), rtol=1e-10, atol=1e-12)


@pytest.mark.skipif(__import__("oracle.openblas").openblas.lib() is None, reason="numpy without its OpenBLAS")
def test_solve_converges():
    """ILQR.jl loop at N = 20: the oracle == the independent restatement bit for bit (12 passes,
    J = 10093.685266152588 with the products rounded as Julia's OpenBLAS dispatch rounds them,
    10093.673801764775 with sequential sums).  The pass count is a property of Julia's pinv composition:
    with it, every choice of trig / exp (Julia-libm or glibc) and products (sequential, numpy's matmul or
    Julia's dispatch) converges in 12 passes to J in [10093.65, 10093.69]; only numpy's pinv (BLAS-composed,
    rcond 1e-15) together with numpy's matmul products gives the 13 passes / J = 10086.6 of the SURVEY's
    probe (tools/ilqr_ulp_sources.py)."""
    p, X0, U0, J0 = _setup()
    X, U, J, iters, flags = oracle.ilqr_solve(p, X0, U0)
    assert flags == 0 and iters == 13 and J == 10093.685266152588
    it, Jm, _ = _model().solve()
    assert it == iters and Jm == J
    with oracle.blas_mode(0):
        _, _, J, iters, flags = oracle.ilqr_solve(p, X0, U0)
    assert flags == 0 and iters == 13 and J == 10093.673801764775
    it, Jm, _ = _model(prod="seq").solve()
    assert it == iters and Jm == J
    for kw in (dict(trig="libm", exp="libm", prod="blas"), dict(exp="fdlibm", prod="blas"), dict(trig="libm")):
        it, Jm, _ = _model(**kw).solve()
        assert it == 13 and 10093.65 < Jm < 10093.69, kw
    it, Jm, _ = _model(pinv="numpy", prod="blas").solve()
    assert it == 14 and 10086.6 < Jm < 10086.7


def test_parking_variant_runs():
    """PathPlanning/Parking_ILQR: N=30, cost weights of Cost.jl:21/:33, alpha floor 1e-3 (ILQR.jl:83-85)."""
    p = ilqr.params(N=30, variant=ilqr.MP_ILQR_PARKING, max_iter=50)
    U = ilqr.initial_controls(1, 30)[0]
    X, J0 = oracle.ilqr_rollout(p, np.array(ilqr.X0_REF), U)
    X, U, J, iters, flags = oracle.ilqr_solve(p, X, U)
    # the alpha floor accepts a worse trial (reference behaviour), so J need not decrease
    assert np.isfinite(J) and np.isfinite(X).all()
    assert flags in (0, 2)  # the script oscillates; max_iter may end it
    del J0


def _fixpoint(U, k, cap):
    """ilqr.hip trial_fixpoint restated: least m in [0, cap] with U + 2^-m k == U bit for bit for every
    control entry (cap + 1 if none)."""
    u, kk = U[:-1].reshape(-1), k.reshape(-1)
    for m in range(cap + 1):
        if np.array_equal((u + np.ldexp(1.0, -m) * kk).view(np.int64), u.view(np.int64)):
            return m
    return cap + 1


def test_trial_fixpoint_trials_are_identical():
    """The line-search cutoff of ilqr.hip (trial_fixpoint): every trial m >= m* is bit-identical to trial m*
    (controls, states and cost), so the device never evaluates one beyond m*.  Checked on the oracle's
    forward trial along real solves of configs[2] instances, OptimalControl (stalling instances reach
    max_ls there) and Parking; plus the sandwich on random entries, signed zeros and subnormals included."""
    cases = 0
    for variant, N in ((ilqr.MP_ILQR_OPTIMALCONTROL, 100), (ilqr.MP_ILQR_PARKING, 30)):
        p = ilqr.params(N=N, variant=variant, max_iter=60)
        x0, U0 = ilqr.cfg3_instances(12, N, seed=5)
        for b in range(12):
            X, J = oracle.ilqr_rollout(p, x0[b], U0[b])
            U = U0[b].copy()
            for _ in range(6):
                k, K = oracle.ilqr_backward(p, X, U)
                ms = _fixpoint(U, k, 199)
                assert 0 < ms < 200
                ref = oracle.ilqr_forward(p, X, U, k, K, np.ldexp(1.0, -ms))
                for m in (ms + 1, ms + 7, 199):
                    got = oracle.ilqr_forward(p, X, U, k, K, np.ldexp(1.0, -m))
                    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]) and got[2] == ref[2]
                cases += 1
                a, Jn = 1.0, J
                while True:  # the reference's halving loop, to move on to the next iterate
                    Xn, Un, Jn = oracle.ilqr_forward(p, X, U, k, K, a)
                    a /= 2
                    if Jn < J or a < 2.0 ** -199:
                        break
                X, U, J = Xn, Un, Jn
    assert cases == 144
    # the monotone sandwich on raw entries: fixed at m* => fixed at every m > m* (bits)
    r = np.random.default_rng(2)
    u = np.concatenate([r.standard_normal(4000) * 10.0 ** r.integers(-300, 300, 4000), [0.0, -0.0, 5e-324, -5e-324]])
    kk = np.concatenate([r.standard_normal(4000) * 10.0 ** r.integers(-300, 300, 4000), [-0.0, 0.0, 1.0, 0.0]])
    for m0 in range(0, 1100, 7):
        t0 = (u + np.ldexp(1.0, -m0) * kk).view(np.int64) == u.view(np.int64)
        for m in (m0 + 1, m0 + 13, m0 + 200):
            assert not np.any(t0 & ((u + np.ldexp(1.0, -m) * kk).view(np.int64) != u.view(np.int64)))
