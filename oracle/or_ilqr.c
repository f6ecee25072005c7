/*
 * ORACLE — test infrastructure only.  CPU restatement of the iLQR sibling:
 * OptimalControl/ILQR/{Dynamics,Cost,GetMatrix,ILQR}.jl and the cost/line-search
 * variant PathPlanning/Parking_ILQR (all files).  Scalar C, fp64, reference evaluation order.
 *
 * Parity status: there is no reference-produced artifact for this path
 * ("parity unpinned" against Julia).  Anchors: the script's own
 * constants, and the restatement-derived convergence value quoted in SURVEY §8a
 * B7 (14 iterations, J ≈ 10086.597 at N = 20), checked in tests/test_oracle_ilqr.py.
 *
 * Layouts: X[N][4] (StatesList 4×N), U[N][2] (CtrlsList 2×N), k[N-1][2] (klist),
 * Kg[N-1][4][2] (Klist 2×4×(N-1), Julia column-major: element (r,c) at [c][r]).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mp_jlmath.h"
#include "../include/mpgpu.h"
#include "or_blas.h"

/* Dynamics.jl:1-16 ; state [x, y, ux, ψ], control [ax, δ] */
static void dyn(const double* s, const double* u, double* d) {
  const double la = 1.56, lb = 1.64;
  double ux = s[2], psi = s[3], ax = u[0], dl = u[1];
  double tdl = mpj_tan(dl);
  double beta = mpj_atan(la / (la + lb) * tdl);
  double sb, cb;
  mpj_sincos(psi + beta, &sb, &cb);
  d[0] = ux * cb;
  d[1] = ux * sb;
  d[2] = ax;
  d[3] = ux * mpj_cos(beta) * tdl / (la + lb);
}

/* RK4Integration, Dynamics.jl:18-28 */
void or_ilqr_rk4(const double* s, const double* u, double dT, double* o) {
  double k1[4], k2[4], k3[4], k4[4], x2[4], x3[4], x4[4];
  dyn(s, u, k1);
  for (int i = 0; i < 4; i++) x2[i] = s[i] + dT / 2 * k1[i];
  dyn(x2, u, k2);
  for (int i = 0; i < 4; i++) x3[i] = s[i] + dT / 2 * k2[i];
  dyn(x3, u, k3);
  for (int i = 0; i < 4; i++) x4[i] = s[i] + dT * k3[i];
  dyn(x4, u, k4);
  for (int i = 0; i < 4; i++) o[i] = 1.0 / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]) * dT + s[i];
}

/* sigmoid_boundary, Cost.jl:42-49 */
static double sigmoid_boundary(double st, double mn, double mx) {
  const double slope = 10, mag = 100;
  double c1 = 1 / (1 + mpj_exp(-slope * (st - mx)));
  double c2 = 1 / (1 + mpj_exp(slope * (st - mn)));
  return mag * (c1 + c2);
}

/* StageCost, Cost.jl:10-27 (variant 1: PathPlanning/Parking_ILQR/Cost.jl:21) */
double or_ilqr_stage(int variant, const double* s, const double* u) {
  double x = s[0], y = s[1], ux = s[2], psi = s[3], ax = u[0], dl = u[1];
  double db = sigmoid_boundary(dl, -MPJ_PI / 6, MPJ_PI / 6);
  double ab = sigmoid_boundary(ax, -2, 2);
  if (variant == MP_ILQR_PARKING)
    return 0.01 * (ax * ax) + 0.01 * (dl * dl) + 10 * (y * y) + 0.5 * (x * x) + 100 * (psi * psi) +
           0.01 * (ux * ux) + db + ab;
  return 10 * (ax * ax) + 10 * (dl * dl) + 0.01 * (ux * ux) + db + ab;
}

/* TerminalCost, Cost.jl:29-40 */
double or_ilqr_terminal(int variant, const double* s) {
  double x = s[0], y = s[1], ux = s[2], psi = s[3];
  double w = variant == MP_ILQR_PARKING ? 10 : 1000;
  return w * (((x - 0.0) * (x - 0.0) + (y - 0.0) * (y - 0.0)) + 0.1 * ((ux - 0.0) * (ux - 0.0)) +
              1 * ((psi - 0.0) * (psi - 0.0)));
}

/* TotalCost, Cost.jl:1-8 */
double or_ilqr_total(int variant, int N, const double* X, const double* U) {
  double J = 0.0;
  for (int i = 0; i < N - 1; i++) J = J + or_ilqr_stage(variant, X + 4 * i, U + 2 * i);
  return J + or_ilqr_terminal(variant, X + 4 * (N - 1));
}

typedef struct { int variant; int terminal; } costsel;
static double cfun(costsel c, const double* s, const double* u) {
  return c.terminal ? or_ilqr_terminal(c.variant, s) : or_ilqr_stage(c.variant, s, u);
}

/* CalculateMatrix, GetMatrix.jl:3-68 (ϵ = eps): lx[4], lu[2], lxx[4][4], luu[2][2], lux[2][4] */
static void calc_matrix(costsel cs, const double* s, const double* u, double e, double* lx, double* lu,
                        double* lxx, double* luu, double* lux) {
  double sp[4], sm[4], up[2], um[2], t1[4], t2[4], t3[4], t4[4], v1[2], v2[2], v3[2], v4[2];
  const double c12 = 1 / (12 * (e * e)), c4 = 1 / (4 * (e * e));
  for (int i = 0; i < 4; i++) {
    memcpy(sp, s, 32); memcpy(sm, s, 32);
    sp[i] = s[i] + e; sm[i] = s[i] - e;
    lx[i] = (cfun(cs, sp, u) - cfun(cs, sm, u)) / (2 * e);
  }
  for (int j = 0; j < 2; j++) {
    memcpy(up, u, 16); memcpy(um, u, 16);
    up[j] = u[j] + e; um[j] = u[j] - e;
    lu[j] = (cfun(cs, s, up) - cfun(cs, s, um)) / (2 * e);
  }
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      if (i == j) {
        memcpy(t1, s, 32); memcpy(t2, s, 32); memcpy(t3, s, 32); memcpy(t4, s, 32);
        t1[i] = s[i] + 2 * e; t2[i] = s[i] + e; t3[i] = s[i] - e; t4[i] = s[i] - 2 * e;
        lxx[4 * i + j] = c12 * (-cfun(cs, t1, u) + 16 * cfun(cs, t2, u) - 30 * cfun(cs, s, u) +
                                16 * cfun(cs, t3, u) - cfun(cs, t4, u));
      } else {
        /* states .+ Δi .+ Δj etc.: element i gets ±ϵ, element j gets ±ϵ */
        memcpy(t1, s, 32); memcpy(t2, s, 32); memcpy(t3, s, 32); memcpy(t4, s, 32);
        t1[i] = s[i] + e; t1[j] = s[j] + e;
        t2[i] = s[i] - e; t2[j] = s[j] - e;
        t3[i] = s[i] + e; t3[j] = s[j] - e;
        t4[i] = s[i] - e; t4[j] = s[j] + e;
        lxx[4 * i + j] = c4 * (cfun(cs, t1, u) + cfun(cs, t2, u) - cfun(cs, t3, u) - cfun(cs, t4, u));
      }
    }
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) {
      if (i == j) {
        memcpy(v1, u, 16); memcpy(v2, u, 16); memcpy(v3, u, 16); memcpy(v4, u, 16);
        v1[i] = u[i] + 2 * e; v2[i] = u[i] + e; v3[i] = u[i] - e; v4[i] = u[i] - 2 * e;
        luu[2 * i + j] = c12 * (-cfun(cs, s, v1) + 16 * cfun(cs, s, v2) - 30 * cfun(cs, s, u) +
                                16 * cfun(cs, s, v3) - cfun(cs, s, v4));
      } else {
        memcpy(v1, u, 16); memcpy(v2, u, 16); memcpy(v3, u, 16); memcpy(v4, u, 16);
        v1[i] = u[i] + e; v1[j] = u[j] + e;
        v2[i] = u[i] - e; v2[j] = u[j] - e;
        v3[i] = u[i] + e; v3[j] = u[j] - e;
        v4[i] = u[i] - e; v4[j] = u[j] + e;
        luu[2 * i + j] = c4 * (cfun(cs, s, v1) + cfun(cs, s, v2) - cfun(cs, s, v3) - cfun(cs, s, v4));
      }
    }
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 4; j++) {
      memcpy(sp, s, 32); memcpy(sm, s, 32); memcpy(up, u, 16); memcpy(um, u, 16);
      sp[j] = s[j] + e; sm[j] = s[j] - e; up[i] = u[i] + e; um[i] = u[i] - e;
      lux[4 * i + j] = c4 * (cfun(cs, sp, up) + cfun(cs, sm, um) - cfun(cs, sm, up) - cfun(cs, sp, um));
    }
}

/* LocallyLinearizeDynamics, GetMatrix.jl:70-91: A[4][4], B[4][2] (row-major) */
static void linearize(const double* s, const double* u, double dT, double e, double* A, double* B) {
  double sp[4], sm[4], up[2], um[2], fp[4], fm[4];
  for (int i = 0; i < 4; i++) {
    memcpy(sp, s, 32); memcpy(sm, s, 32);
    sp[i] = s[i] + e; sm[i] = s[i] - e;
    or_ilqr_rk4(sp, u, dT, fp);
    or_ilqr_rk4(sm, u, dT, fm);
    for (int r = 0; r < 4; r++) A[4 * r + i] = (fp[r] - fm[r]) / (2 * e);
  }
  for (int j = 0; j < 2; j++) {
    memcpy(up, u, 16); memcpy(um, u, 16);
    up[j] = u[j] + e; um[j] = u[j] - e;
    or_ilqr_rk4(s, up, dT, fp);
    or_ilqr_rk4(s, um, dT, fm);
    for (int r = 0; r < 4; r++) B[2 * r + j] = (fp[r] - fm[r]) / (2 * e);
  }
}

/* pinv of a 2x2: Julia's LinearAlgebra.pinv through LAPACK dgesdd (mp_jlmath.h mpj_pinv2). */
void or_pinv2(const double* M, double* P) { mpj_pinv2(M, P); }
void or_pinv2_batch(int n, const double* M, double* P) {
  for (int i = 0; i < n; i++) mpj_pinv2(M + 4 * i, P + 4 * i);
}
/* the device sweep's straight-line variant (mpj_pinv2_fast); rare[i] = 1 where it defers to mpj_pinv2 */
void or_pinv2_fast_batch(int n, const double* M, double* P, int* rare) {
  for (int i = 0; i < n; i++) {
    rare[i] = 0;
    mpj_pinv2_fast(M + 4 * i, P + 4 * i, rare + i);
  }
}
void or_svd2_batch(int n, const double* A, double* U, double* S, double* VT) {
  for (int i = 0; i < n; i++) mpj_svd2(A + 4 * i, U + 4 * i, S + 2 * i, VT + 4 * i);
}

/* The round-1/2 closed-form 2x2 SVD pinv (M = R(φ) diag(sx, sy) R(θ)), kept only for
 * tools/ilqr_ulp_sources.py's rounding-source table. */
void or_pinv2_closed(const double* M, double* P) {
  double E = (M[0] + M[3]) / 2, F = (M[0] - M[3]) / 2, G = (M[2] + M[1]) / 2, H = (M[2] - M[1]) / 2;
  double Q = sqrt(E * E + H * H), R = sqrt(F * F + G * G);
  double sx = Q + R, sy = Q - R;
  double a1 = mpj_atan2(G, F), a2 = mpj_atan2(H, E);
  double th = (a2 - a1) / 2, ph = (a2 + a1) / 2;
  double st, ct, sp, cp;
  mpj_sincos(th, &st, &ct);
  mpj_sincos(ph, &sp, &cp);
  double smax = fabs(sx) > fabs(sy) ? fabs(sx) : fabs(sy);
  double tol = 4.440892098500626e-16 * smax;
  double i1 = fabs(sx) > tol ? 1.0 / sx : 0.0;
  double i2 = fabs(sy) > tol ? 1.0 / sy : 0.0;
  P[0] = ct * i1 * cp - st * i2 * sp;
  P[1] = ct * i1 * sp + st * i2 * cp;
  P[2] = -st * i1 * cp - ct * i2 * sp;
  P[3] = -st * i1 * sp + ct * i2 * cp;
}

/* ILQR.jl:46-67, one backward sweep.  Returns 0. */
int or_ilqr_backward(const mp_ilqr_params* p, const double* X, const double* U, double* kout, double* Kout) {
  const int N = p->N;
  const double e = p->eps;
  double Vx[4], Vxx[16], lx[4], lu[2], lxx[16], luu[4], lux[8], A[16], B[8];
  {
    costsel ct = {p->variant, 1};
    double zu[2] = {0.0, 0.0}, lu1[2], luu1[4], lux1[8];
    calc_matrix(ct, X + 4 * (N - 1), zu, e, Vx, lu1, Vxx, luu1, lux1);
  }
  costsel cs = {p->variant, 0};
  for (int j = N - 2; j >= 0; j--) {
    const double* xc = X + 4 * j;
    const double* uc = U + 2 * j;
    linearize(xc, uc, p->dT, e, A, B);
    calc_matrix(cs, xc, uc, e, lx, lu, lxx, luu, lux);
    double Qx[4], Qu[2], Qxx[16], Quu[4], Qux[8], T44[16], T24[8], P[4];
    /* Every product is BLAS dgemm in Julia (lx, lu, Vx are n x 1 matrices, GetMatrix.jl:6-7), with the
     * association of Julia's 3-argument `*` (LinearAlgebra._tri_matmul: equal costs -> (A*B)*C, and
     * K'*(Quu*k) for Vx); or_blas.h blk4 / blk2 round them as OpenBLAS does. */
    for (int i = 0; i < 4; i++) Qx[i] = lx[i] + blk4(A + i, 4, Vx, 1);      /* Qx = lx + fx' * Vx */
    for (int i = 0; i < 2; i++) Qu[i] = lu[i] + blk4(B + i, 2, Vx, 1);      /* Qu = lu + fu' * Vx */
    for (int i = 0; i < 4; i++)                                             /* T44 = fx' * Vxx */
      for (int c = 0; c < 4; c++) T44[4 * i + c] = blk4(A + i, 4, Vxx + c, 4);
    for (int i = 0; i < 4; i++)                                             /* Qxx = lxx + (fx' Vxx) fx */
      for (int c = 0; c < 4; c++) Qxx[4 * i + c] = lxx[4 * i + c] + blk4(T44 + 4 * i, 1, A + c, 4);
    for (int i = 0; i < 2; i++)                                             /* T24 = fu' * Vxx */
      for (int c = 0; c < 4; c++) T24[4 * i + c] = blk4(B + i, 2, Vxx + c, 4);
    for (int i = 0; i < 2; i++)                                             /* Quu = luu + (fu' Vxx) fu */
      for (int c = 0; c < 2; c++) Quu[2 * i + c] = luu[2 * i + c] + blk4(T24 + 4 * i, 1, B + c, 2);
    for (int i = 0; i < 2; i++)                                             /* Qux = lux + (fu' Vxx) fx */
      for (int c = 0; c < 4; c++) Qux[4 * i + c] = lux[4 * i + c] + blk4(T24 + 4 * i, 1, A + c, 4);
    or_pinv2(Quu, P);
    double kk[2], KK[8];
    /* k = -pinv(Quu) * Qu, K = -pinv(Quu) * Qux: dgemm with K = 2 (2x1 and 2x4 right operands) */
    for (int i = 0; i < 2; i++) kk[i] = blk2(-P[2 * i + 0], Qu[0], -P[2 * i + 1], Qu[1]);
    for (int i = 0; i < 2; i++)
      for (int c = 0; c < 4; c++) KK[4 * i + c] = blk2(-P[2 * i + 0], Qux[0 * 4 + c], -P[2 * i + 1], Qux[1 * 4 + c]);
    for (int i = 0; i < 2; i++) kout[2 * j + i] = kk[i];
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 4; c++) Kout[8 * j + 2 * c + r] = KK[4 * r + c];
    /* Vx = Qx - K' * (Quu * k)   (Julia's 3-arg * picks A*(B*C) here) */
    double qk[2];
    for (int i = 0; i < 2; i++) qk[i] = blk2(Quu[2 * i + 0], kk[0], Quu[2 * i + 1], kk[1]);
    for (int i = 0; i < 4; i++) Vx[i] = Qx[i] - blk2(KK[0 * 4 + i], qk[0], KK[1 * 4 + i], qk[1]);
    /* Vxx = Qxx - (K' * Quu) * K */
    double KQ[8];
    for (int i = 0; i < 4; i++)
      for (int c = 0; c < 2; c++) KQ[2 * i + c] = blk2(KK[0 * 4 + i], Quu[0 * 2 + c], KK[1 * 4 + i], Quu[1 * 2 + c]);
    for (int i = 0; i < 4; i++)
      for (int c = 0; c < 4; c++) Vxx[4 * i + c] = Qxx[4 * i + c] - blk2(KQ[2 * i + 0], KK[0 * 4 + c], KQ[2 * i + 1], KK[1 * 4 + c]);
  }
  return 0;
}

/* ILQR.jl:72-80, one forward trial at step size alpha; returns J_new. */
double or_ilqr_forward(const mp_ilqr_params* p, const double* X, const double* U, const double* k,
                       const double* Kg, double alpha, double* Xn, double* Un) {
  const int N = p->N;
  memcpy(Xn, X, 32);
  for (int i = 0; i < N - 1; i++) {
    double dx[4], u[2];
    for (int r = 0; r < 4; r++) dx[r] = Xn[4 * i + r] - X[4 * i + r];
    for (int r = 0; r < 2; r++) /* Klist[:, :, i] * (xtilde .- xn): BLAS dgemv 'N' 2x4 (or_blas.h) */
      u[r] = (U[2 * i + r] + alpha * k[2 * i + r]) + blv_n24(Kg + 8 * i + r, 2, dx);
    Un[2 * i] = u[0];
    Un[2 * i + 1] = u[1];
    or_ilqr_rk4(Xn + 4 * i, u, p->dT, Xn + 4 * (i + 1));
  }
  Un[2 * (N - 1)] = 0.0;
  Un[2 * (N - 1) + 1] = 0.0;
  return or_ilqr_total(p->variant, N, Xn, Un);
}

/* Initial guess roll out (ILQR.jl:31-37): X[0] = x0, X[i+1] = RK4(X[i], U[i]); returns TotalCost. */
double or_ilqr_rollout(const mp_ilqr_params* p, const double* x0, const double* U, double* X) {
  memcpy(X, x0, 32);
  for (int i = 0; i < p->N - 1; i++) or_ilqr_rk4(X + 4 * i, U + 2 * i, p->dT, X + 4 * (i + 1));
  return or_ilqr_total(p->variant, p->N, X, U);
}

/* The script loop ILQR.jl:39-88.  X/U: in initial guess (X from or_ilqr_rollout), out solution.
 * Returns status flags: 1 = max_ls reached (reference would loop forever), 2 = max_iter reached. */
int or_ilqr_solve(const mp_ilqr_params* p, double* X, double* U, double* Jout, int32_t* iters) {
  const int N = p->N;
  double* k = calloc((size_t)(N - 1) * 2, sizeof(double));
  double* Kg = calloc((size_t)(N - 1) * 8, sizeof(double));
  double* Xn = malloc(sizeof(double) * 4 * N);
  double* Un = calloc((size_t)2 * N, sizeof(double));
  double J = or_ilqr_total(p->variant, N, X, U);
  double Jn = J;
  int iter = 1, flags = 0;
  while (fabs((Jn - J) / J) > p->tol || iter == 1) {
    if (iter > p->max_iter) { flags |= 2; break; }
    J = Jn;
    or_ilqr_backward(p, X, U, k, Kg);
    double alpha = 1.0;
    int ls = 0;
    while (Jn >= J) {
      Jn = or_ilqr_forward(p, X, U, k, Kg, alpha, Xn, Un);
      alpha = alpha / 2;
      ls++;
      if (p->alpha_floor > 0 && alpha <= p->alpha_floor) break;
      if (ls >= p->max_ls) { flags |= 1; break; }
    }
    memcpy(X, Xn, sizeof(double) * 4 * N);
    memcpy(U, Un, sizeof(double) * 2 * N);
    iter++;
  }
  *Jout = Jn;
  *iters = iter;
  free(k); free(Kg); free(Xn); free(Un);
  return flags;
}
