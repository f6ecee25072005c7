"""Which rounding source decides the iLQR script's converged result?  

A pure-Python restatement of OptimalControl/ILQR/ILQR.jl:39-88 at N = 20 whose every rounding source
can be swapped independently:

  trig   jl     the oracle's Julia-libm restatements (mp_jlmath.h: tan, atan, sin/cos)
         libm   glibc via Python's math module
  exp    julia  Julia >= 1.6's table-driven exp (mp_jlmath.h mpj_exp, muladd fused)
         fdlibm FDLIBM e_exp.c (the round-1/2 oracle)
         libm   glibc
  pinv   lapack LinearAlgebra.pinv: isdiag branch, else gesdd's 2x2 path (oracle or_svd2) composed as
                Vt' * (Diagonal(Sinv) * U') with matmul2x2 (no FMA)
         closed the round-1/2 closed-form 2x2 SVD (atan2 + sincos)
         numpy  np.linalg.pinv (BLAS composition, rcond 1e-15)
  prod   seq    every matrix product as a left-to-right sum of rounded products (the oracle)
         blas   numpy's OpenBLAS for the same shapes (FMA kernels; the gemm->gemv forward for n = 1)
         julia  numpy's OpenBLAS called as Julia calls it (oracle/openblas.py: dgemm_64_ with Julia's
                trans flags for every matrix product -- lx/lu/Vx are n x 1 matrices -- and dgemv_64_
                'N' for Klist * (xtilde .- xn)); = the C oracle with or_blas = 1 bit for bit
  pert   plus   Julia's `states .+ Δ` (untouched entries get + 0.0: -0.0 -> +0.0)
         copy   the perturbed entry only (round-1/2 oracle; -0.0 survives)

Run:  python tools/ilqr_ulp_sources.py      (prints one row per configuration; ~1 s each)
Test infrastructure only: imports oracle/ as the source of the restated libm functions.
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

LA, LB = 1.56, 1.64


class Model:
    def __init__(self, trig="jl", exp="julia", pinv="lapack", prod="julia", pert="plus"):
        self.cfg = dict(trig=trig, exp=exp, pinv=pinv, prod=prod, pert=pert)
        L = oracle.lib()
        if trig == "jl":
            self.tan, self.atan, self.sin, self.cos = L.or_m_tan, L.or_m_atan, L.or_m_sin, L.or_m_cos
        else:
            self.tan, self.atan, self.sin, self.cos = math.tan, math.atan, math.sin, math.cos
        if exp == "julia":
            self.exp = L.or_m_exp
        elif exp == "fdlibm":
            self.exp = L.or_m_exp_fdlibm
        else:
            self.exp = lambda v: math.exp(v) if v < 709.78 else math.inf
        self.pinv = {"lapack": oracle.pinv2, "closed": oracle.pinv2_closed,
                     "numpy": lambda M: np.linalg.pinv(M)}[pinv]
        self.prod = prod
        self.pert = pert

    # ---------------------------------------------------------------- products
    def mm(self, A, B, ta=False):
        """op(A) * B; ta: A' * B (Julia's A' * B)."""
        if self.prod == "julia":
            from oracle import openblas
            return openblas.gemm(A, B, ta=ta)
        A = np.asarray(A, np.float64)
        B = np.asarray(B, np.float64)
        if ta:
            A = A.T
        if self.prod == "blas":
            return np.asfortranarray(A) @ np.asfortranarray(B)
        m, k = A.shape
        n = B.shape[1]
        C = np.zeros((m, n))
        for i in range(m):
            for j in range(n):
                acc = A[i, 0] * B[0, j]
                for t in range(1, k):
                    acc = acc + A[i, t] * B[t, j]
                C[i, j] = acc
        return C

    # ---------------------------------------------------------------- Dynamics.jl / Cost.jl
    def dyn(self, s, u):
        ux, psi, ax, d = s[2], s[3], u[0], u[1]
        td = self.tan(d)
        b = self.atan(LA / (LA + LB) * td)
        return np.array([ux * self.cos(psi + b), ux * self.sin(psi + b), ax, ux * self.cos(b) * td / (LA + LB)])

    def rk4(self, s, u, dT):
        k1 = self.dyn(s, u)
        k2 = self.dyn(s + dT / 2 * k1, u)
        k3 = self.dyn(s + dT / 2 * k2, u)
        k4 = self.dyn(s + dT * k3, u)
        return 1 / 6 * (((k1 + 2 * k2) + 2 * k3) + k4) * dT + s

    def sig(self, st, mn, mx):
        return 100 * (1 / (1 + self.exp(-10 * (st - mx))) + 1 / (1 + self.exp(10 * (st - mn))))

    def stage(self, s, u):
        return (((10 * (u[0] * u[0]) + 10 * (u[1] * u[1])) + 0.01 * (s[2] * s[2])) + self.sig(u[1], -math.pi / 6, math.pi / 6)
                ) + self.sig(u[0], -2, 2)

    @staticmethod
    def term(s, u=None):
        return 1000 * (((s[0] * s[0] + s[1] * s[1]) + 0.1 * (s[2] * s[2])) + 1 * (s[3] * s[3]))

    def total(self, X, U):
        J = 0.0
        for i in range(len(X) - 1):
            J = J + self.stage(X[i], U[i])
        return J + self.term(X[-1])

    # ---------------------------------------------------------------- GetMatrix.jl
    def shift(self, v, terms):
        """v .+ Δa .- Δb ... : Julia adds every (mostly zero) entry; the 'copy' model touches only the
        perturbed entries."""
        out = np.array(v, np.float64)
        for sgn, idx, mag in terms:
            if self.pert == "plus":
                d = np.zeros_like(out)
                d[idx] = mag
                out = out + d if sgn > 0 else out - d
            else:
                out[idx] = out[idx] + mag if sgn > 0 else out[idx] - mag
        return out

    def calc(self, s, u, f, e=1e-3):
        n, m = 4, 2
        sh = self.shift
        c12, c4 = 1 / (12 * (e * e)), 1 / (4 * (e * e))
        lx = np.array([(f(sh(s, [(1, i, e)]), u) - f(sh(s, [(-1, i, e)]), u)) / (2 * e) for i in range(n)])
        lu = np.array([(f(s, sh(u, [(1, j, e)])) - f(s, sh(u, [(-1, j, e)]))) / (2 * e) for j in range(m)])
        lxx = np.zeros((n, n))
        for i in range(n):
            for j in range(n):
                if i == j:
                    lxx[i, j] = c12 * ((((-f(sh(s, [(1, i, 2 * e)]), u) + 16 * f(sh(s, [(1, i, e)]), u)) - 30 * f(s, u))
                                        + 16 * f(sh(s, [(-1, i, e)]), u)) - f(sh(s, [(-1, i, 2 * e)]), u))
                else:
                    lxx[i, j] = c4 * (((f(sh(s, [(1, i, e), (1, j, e)]), u) + f(sh(s, [(-1, i, e), (-1, j, e)]), u))
                                       - f(sh(s, [(1, i, e), (-1, j, e)]), u)) - f(sh(s, [(-1, i, e), (1, j, e)]), u))
        luu = np.zeros((m, m))
        for i in range(m):
            for j in range(m):
                if i == j:
                    luu[i, j] = c12 * ((((-f(s, sh(u, [(1, i, 2 * e)])) + 16 * f(s, sh(u, [(1, i, e)]))) - 30 * f(s, u))
                                        + 16 * f(s, sh(u, [(-1, i, e)]))) - f(s, sh(u, [(-1, i, 2 * e)])))
                else:
                    luu[i, j] = c4 * (((f(s, sh(u, [(1, i, e), (1, j, e)])) + f(s, sh(u, [(-1, i, e), (-1, j, e)])))
                                       - f(s, sh(u, [(1, i, e), (-1, j, e)]))) - f(s, sh(u, [(-1, i, e), (1, j, e)])))
        lux = np.zeros((m, n))
        for i in range(m):
            for j in range(n):
                lux[i, j] = c4 * (((f(sh(s, [(1, j, e)]), sh(u, [(1, i, e)])) + f(sh(s, [(-1, j, e)]), sh(u, [(-1, i, e)])))
                                   - f(sh(s, [(-1, j, e)]), sh(u, [(1, i, e)]))) - f(sh(s, [(1, j, e)]), sh(u, [(-1, i, e)])))
        return lx.reshape(n, 1), lu.reshape(m, 1), lxx, luu, lux

    def lin(self, s, u, dT, e=1e-3):
        A = np.zeros((4, 4))
        B = np.zeros((4, 2))
        for i in range(4):
            A[:, i] = (self.rk4(self.shift(s, [(1, i, e)]), u, dT) - self.rk4(self.shift(s, [(-1, i, e)]), u, dT)) / (2 * e)
        for j in range(2):
            B[:, j] = (self.rk4(s, self.shift(u, [(1, j, e)]), dT) - self.rk4(s, self.shift(u, [(-1, j, e)]), dT)) / (2 * e)
        return A, B

    # ---------------------------------------------------------------- ILQR.jl:46-67
    def backward(self, X, U, dT):
        N = len(X)
        Vx, _, Vxx, _, _ = self.calc(X[-1], np.zeros(2), self.term)
        k = np.zeros((N - 1, 2, 1))
        K = np.zeros((N - 1, 2, 4))
        mm = self.mm
        for j in range(N - 2, -1, -1):
            fx, fu = self.lin(X[j], U[j], dT)
            lx, lu, lxx, luu, lux = self.calc(X[j], U[j], self.stage)
            Qx = lx + mm(fx, Vx, ta=True)
            Qu = lu + mm(fu, Vx, ta=True)
            Qxx = lxx + mm(mm(fx, Vxx, ta=True), fx)
            Quu = luu + mm(mm(fu, Vxx, ta=True), fu)
            Qux = lux + mm(mm(fu, Vxx, ta=True), fx)
            P = -np.asarray(self.pinv(Quu))
            kk = mm(P, Qu)
            KK = mm(P, Qux)
            k[j], K[j] = kk, KK
            Vx = Qx - mm(KK, mm(Quu, kk), ta=True)
            Vxx = Qxx - mm(mm(KK, Quu, ta=True), KK)
        return k, K

    def forward(self, X, U, k, K, alpha, dT):
        N = len(X)
        Xn = X.copy()
        Un = np.zeros_like(U)
        for i in range(N - 1):
            dx = (Xn[i] - X[i]).reshape(4, 1)
            if self.prod == "julia":  # Klist[:, :, i] * (xtilde .- xn): a matrix times a Vector -> dgemv
                from oracle import openblas
                Kdx = openblas.gemv(K[i], dx[:, 0])
            else:
                Kdx = self.mm(K[i], dx)[:, 0]
            u = (U[i] + alpha * k[i][:, 0]) + Kdx
            Un[i] = u
            Xn[i + 1] = self.rk4(Xn[i], u, dT)
        return Xn, Un, self.total(Xn, Un)

    def solve(self, N=20, dT=0.05, max_iter=60):
        X = np.zeros((N, 4))
        X[0] = [0.0, 3.6, 5.0, 0.0]
        U = np.zeros((N, 2))
        U[: N - 1] = [-2.6, 0.01]
        for i in range(N - 1):
            X[i + 1] = self.rk4(X[i], U[i], dT)
        J = self.total(X, U)
        Jn, it, trials = J, 1, []
        while abs((Jn - J) / J) > 1e-6 or it == 1:
            if it > max_iter:
                break
            J = Jn
            k, K = self.backward(X, U, dT)
            a, ls = 1.0, 0
            while Jn >= J:
                Xn, Un, Jn = self.forward(X, U, k, K, a, dT)
                a /= 2
                ls += 1
            trials.append(ls)
            X, U = Xn, Un
            it += 1
        return it, Jn, trials


CONFIGS = [
    ("round-2 oracle (jl trig, fdlibm exp, closed pinv, seq, copy)", dict(exp="fdlibm", pinv="closed", pert="copy",
                                                                        prod="seq")),
    ("round-3..5 oracle (jl trig, julia exp, lapack pinv, seq, plus)", dict(prod="seq")),
    ("round-6 oracle (products as Julia's OpenBLAS dispatch rounds them)", dict()),
    ("  swap pinv -> closed", dict(pinv="closed")),
    ("  swap pinv -> numpy", dict(pinv="numpy")),
    ("  swap exp -> fdlibm", dict(exp="fdlibm")),
    ("  swap exp -> glibc", dict(exp="libm")),
    ("  swap trig -> glibc", dict(trig="libm")),
    ("  swap prod -> numpy's @ (OpenBLAS, numpy's own gemm/gemv choice)", dict(prod="blas")),
    ("  swap prod -> sequential", dict(prod="seq")),
    ("  swap pert -> copy", dict(pert="copy")),
    ("numpy restatement (glibc trig+exp, numpy pinv, OpenBLAS, plus)", dict(trig="libm", exp="libm", pinv="numpy",
                                                                          prod="blas")),
]


def main():
    print("| configuration | passes (iter at exit) | J | line-search trials per pass |")
    print("|---|---|---|---|")
    for name, kw in CONFIGS:
        it, J, trials = Model(**kw).solve()
        print("| %s | %d | %.10f | %s |" % (name, it - 1, J, ",".join(map(str, trials))))




def factorial():
    """Full factorial over the four sources that differ between the oracle and the numpy restatement."""
    import itertools
    print("| trig | exp | pinv | prod | passes | J | trials |")
    print("|---|---|---|---|---|---|---|")
    for trig, exp, pinv, prod in itertools.product(("jl", "libm"), ("julia", "libm"), ("lapack", "numpy"),
                                                   ("seq", "blas", "julia")):
        it, J, trials = Model(trig=trig, exp=exp, pinv=pinv, prod=prod).solve()
        print("| %s | %s | %s | %s | %d | %.10f | %s |" % (trig, exp, pinv, prod, it - 1, J, ",".join(map(str, trials))))


if __name__ == "__main__":
    main()
    print()
    factorial()
