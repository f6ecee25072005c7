// ilqr.hip — batched iLQR (OptimalControl/ILQR/{Dynamics,Cost,GetMatrix,ILQR}.jl and
// the PathPlanning/Parking_ILQR variant) for gfx950 + C-ABI entry points.
//
// Per outer iteration (ILQR.jl:44-88) for B instances:
//   ilqr_deriv_kernel     one thread per (instance, knot j): LocallyLinearizeDynamics
//                         (12 RK4) and CalculateMatrix (130 StageCost evaluations) by
//                         finite differences.  Control-only sub-expressions (tan δ, β,
//                         cos β, the two sigmoid barriers) are evaluated once per distinct
//                         perturbed control and reused: the same function of the same bits,
//                         so every derivative is bit-identical to the scalar restatement.
//                         405,504 independent threads at configs[2] (B=4096, N=100).
//   ilqr_backward_kernel  one thread per instance: the Riccati sweep j = N-2..0 (ILQR.jl:46-67).
//   ilqr_search_kernel    one thread per instance: halving line search + accept (ILQR.jl:70-86).
// The host loops until every instance has met |ΔJ/J| <= tol.
#include "../../include/mp_jlmath.h"
#include "runtime.hpp"

namespace {

constexpr int ND = 58;  // derivative record: A16 B8 lx4 lu2 lxx16 luu4 lux8

struct IlqrDev {
  int N, variant, max_iter, max_ls;
  double dT, eps, alpha_floor, tol;
};

struct UPre {  // control-only part of Dynamics (Dynamics.jl:8-12)
  double tdl, beta, cb;
};

__device__ __forceinline__ UPre upre(double dl) {
  const double la = 1.56, lb = 1.64;
  UPre q;
  q.tdl = mpj_tan(dl);
  q.beta = mpj_atan(la / (la + lb) * q.tdl);
  q.cb = mpj_cos(q.beta);
  return q;
}

// Dynamics.jl:1-16
__device__ __forceinline__ void dyn(const double* s, double ax, const UPre& q, double* d) {
  const double la = 1.56, lb = 1.64;
  double sb, cbb;
  mpj_sincos(s[3] + q.beta, &sb, &cbb);
  d[0] = s[2] * cbb;
  d[1] = s[2] * sb;
  d[2] = ax;
  d[3] = s[2] * q.cb * q.tdl / (la + lb);
}

// RK4Integration, Dynamics.jl:18-28
__device__ __forceinline__ void rk4(const double* s, double ax, const UPre& q, double dT, double* o) {
  double k1[4], k2[4], k3[4], k4[4], x2[4], x3[4], x4[4];
  dyn(s, ax, q, k1);
#pragma unroll
  for (int i = 0; i < 4; i++) x2[i] = s[i] + dT / 2 * k1[i];
  dyn(x2, ax, q, k2);
#pragma unroll
  for (int i = 0; i < 4; i++) x3[i] = s[i] + dT / 2 * k2[i];
  dyn(x3, ax, q, k3);
#pragma unroll
  for (int i = 0; i < 4; i++) x4[i] = s[i] + dT * k3[i];
  dyn(x4, ax, q, k4);
#pragma unroll
  for (int i = 0; i < 4; i++) o[i] = 1.0 / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]) * dT + s[i];
}

// sigmoid_boundary, Cost.jl:42-49
__device__ __forceinline__ double sigmoid_boundary(double st, double mn, double mx) {
  const double slope = 10, mag = 100;
  const double c1 = 1 / (1 + mpj_exp(-slope * (st - mx)));
  const double c2 = 1 / (1 + mpj_exp(slope * (st - mn)));
  return mag * (c1 + c2);
}
__device__ __forceinline__ double sig_d(double dl) { return sigmoid_boundary(dl, -MPJ_PI / 6, MPJ_PI / 6); }
__device__ __forceinline__ double sig_a(double ax) { return sigmoid_boundary(ax, -2, 2); }

// StageCost (Cost.jl:10-27 / Parking_ILQR/Cost.jl:21) with the barrier terms supplied
__device__ __forceinline__ double stage_pre(int variant, const double* s, double ax, double dl, double sd,
                                            double sa) {
  const double x = s[0], y = s[1], ux = s[2], psi = s[3];
  if (variant == MP_ILQR_PARKING)
    return 0.01 * (ax * ax) + 0.01 * (dl * dl) + 10 * (y * y) + 0.5 * (x * x) + 100 * (psi * psi) +
           0.01 * (ux * ux) + sd + sa;
  return 10 * (ax * ax) + 10 * (dl * dl) + 0.01 * (ux * ux) + sd + sa;
}
__device__ __forceinline__ double stage(int variant, const double* s, const double* u) {
  return stage_pre(variant, s, u[0], u[1], sig_d(u[1]), sig_a(u[0]));
}
// TerminalCost, Cost.jl:29-40
__device__ __forceinline__ double terminal(int variant, const double* s) {
  const double x = s[0], y = s[1], ux = s[2], psi = s[3];
  const double w = variant == MP_ILQR_PARKING ? 10 : 1000;
  return w * (((x - 0.0) * (x - 0.0) + (y - 0.0) * (y - 0.0)) + 0.1 * ((ux - 0.0) * (ux - 0.0)) +
              1 * ((psi - 0.0) * (psi - 0.0)));
}

__device__ double total_cost(int variant, int N, const double* X, const double* U) {
  double J = 0.0;
  for (int i = 0; i < N - 1; i++) J = J + stage(variant, X + 4 * i, U + 2 * i);
  return J + terminal(variant, X + 4 * (N - 1));
}

// Cost evaluation at (s, u + du) where du components are offsets from {-2e,-e,0,e,2e};
// sigmoid values cached per offset index (0..4 = -2e..2e).
struct SigCache {
  double a[5], d[5];  // perturbed control values
  double sa[5], sd[5];
};

__device__ __forceinline__ double cst(int variant, const double* s, const SigCache& C, int ia, int id) {
  return stage_pre(variant, s, C.a[ia], C.d[id], C.sd[id], C.sa[ia]);
}

// LocallyLinearizeDynamics + CalculateMatrix for one knot (GetMatrix.jl:3-91)
__device__ void knot_derivs(const IlqrDev& P, const double* s, const double* u, double* out) {
  const double e = P.eps;
  double* A = out;       // [4][4] row-major
  double* Bm = out + 16; // [4][2]
  double* lx = out + 24;
  double* lu = out + 28;
  double* lxx = out + 30;
  double* luu = out + 46;
  double* lux = out + 50;
  // ---- dynamics Jacobians
  const UPre q0 = upre(u[1]);
  double sp[4], sm[4], fp[4], fm[4];
  for (int i = 0; i < 4; i++) {
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[i] = s[i] + e;
    sm[i] = s[i] - e;
    rk4(sp, u[0], q0, P.dT, fp);
    rk4(sm, u[0], q0, P.dT, fm);
    for (int r = 0; r < 4; r++) A[4 * r + i] = (fp[r] - fm[r]) / (2 * e);
  }
  {  // ax perturbation leaves the δ-only terms unchanged
    rk4(s, u[0] + e, q0, P.dT, fp);
    rk4(s, u[0] - e, q0, P.dT, fm);
    for (int r = 0; r < 4; r++) Bm[2 * r + 0] = (fp[r] - fm[r]) / (2 * e);
    const UPre qp = upre(u[1] + e), qm = upre(u[1] - e);
    rk4(s, u[0], qp, P.dT, fp);
    rk4(s, u[0], qm, P.dT, fm);
    for (int r = 0; r < 4; r++) Bm[2 * r + 1] = (fp[r] - fm[r]) / (2 * e);
  }
  // ---- cost derivatives
  SigCache C;
  C.a[0] = u[0] - 2 * e; C.a[1] = u[0] - e; C.a[2] = u[0]; C.a[3] = u[0] + e; C.a[4] = u[0] + 2 * e;
  C.d[0] = u[1] - 2 * e; C.d[1] = u[1] - e; C.d[2] = u[1]; C.d[3] = u[1] + e; C.d[4] = u[1] + 2 * e;
#pragma unroll
  for (int t = 0; t < 5; t++) {
    C.sa[t] = sig_a(C.a[t]);
    C.sd[t] = sig_d(C.d[t]);
  }
  const int V = P.variant;
  const double c12 = 1 / (12 * (e * e)), c4 = 1 / (4 * (e * e));
  const double c0 = cst(V, s, C, 2, 2);
  for (int i = 0; i < 4; i++) {
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[i] = s[i] + e;
    sm[i] = s[i] - e;
    lx[i] = (cst(V, sp, C, 2, 2) - cst(V, sm, C, 2, 2)) / (2 * e);
  }
  lu[0] = (cst(V, s, C, 3, 2) - cst(V, s, C, 1, 2)) / (2 * e);
  lu[1] = (cst(V, s, C, 2, 3) - cst(V, s, C, 2, 1)) / (2 * e);
  double t1[4], t2[4], t3[4], t4[4];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      for (int r = 0; r < 4; r++) { t1[r] = s[r]; t2[r] = s[r]; t3[r] = s[r]; t4[r] = s[r]; }
      if (i == j) {
        t1[i] = s[i] + 2 * e; t2[i] = s[i] + e; t3[i] = s[i] - e; t4[i] = s[i] - 2 * e;
        lxx[4 * i + j] = c12 * (-cst(V, t1, C, 2, 2) + 16 * cst(V, t2, C, 2, 2) - 30 * c0 +
                                16 * cst(V, t3, C, 2, 2) - cst(V, t4, C, 2, 2));
      } else {
        t1[i] = s[i] + e; t1[j] = s[j] + e;
        t2[i] = s[i] - e; t2[j] = s[j] - e;
        t3[i] = s[i] + e; t3[j] = s[j] - e;
        t4[i] = s[i] - e; t4[j] = s[j] + e;
        lxx[4 * i + j] = c4 * (cst(V, t1, C, 2, 2) + cst(V, t2, C, 2, 2) - cst(V, t3, C, 2, 2) - cst(V, t4, C, 2, 2));
      }
    }
  // luu: index 0 = ax, 1 = δ
  luu[0] = c12 * (-cst(V, s, C, 4, 2) + 16 * cst(V, s, C, 3, 2) - 30 * c0 + 16 * cst(V, s, C, 1, 2) - cst(V, s, C, 0, 2));
  luu[3] = c12 * (-cst(V, s, C, 2, 4) + 16 * cst(V, s, C, 2, 3) - 30 * c0 + 16 * cst(V, s, C, 2, 1) - cst(V, s, C, 2, 0));
  // (i=0,j=1): v1 = (+e,+e), v2 = (-e,-e), v3 = (a+e, d-e), v4 = (a-e, d+e)
  luu[1] = c4 * (cst(V, s, C, 3, 3) + cst(V, s, C, 1, 1) - cst(V, s, C, 3, 1) - cst(V, s, C, 1, 3));
  // (i=1,j=0): v1 = (+e,+e), v2 = (-e,-e), v3 = (δ+e, a-e), v4 = (δ-e, a+e)
  luu[2] = c4 * (cst(V, s, C, 3, 3) + cst(V, s, C, 1, 1) - cst(V, s, C, 1, 3) - cst(V, s, C, 3, 1));
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 4; j++) {
      for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
      sp[j] = s[j] + e;
      sm[j] = s[j] - e;
      const int ap = i == 0 ? 3 : 2, dp = i == 1 ? 3 : 2, am = i == 0 ? 1 : 2, dm = i == 1 ? 1 : 2;
      lux[4 * i + j] = c4 * (cst(V, sp, C, ap, dp) + cst(V, sm, C, am, dm) - cst(V, sm, C, ap, dp) -
                             cst(V, sp, C, am, dm));
    }
}

__global__ __launch_bounds__(256) void ilqr_deriv_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                         const int* active, double* D) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int Nm = P.N - 1;
  if (t >= (long long)B * Nm) return;
  const int b = (int)(t / Nm), j = (int)(t % Nm);
  if (active && !active[b]) return;
  double out[ND];
  knot_derivs(P, X + ((size_t)b * P.N + j) * 4, U + ((size_t)b * P.N + j) * 2, out);
  double* d = D + (size_t)t * ND;
#pragma unroll
  for (int i = 0; i < ND; i++) d[i] = out[i];
}

// pinv of a 2x2 (closed-form SVD; identical operation sequence to oracle/or_ilqr.c or_pinv2)
__device__ void pinv2(const double* M, double* Pm) {
  const double E = (M[0] + M[3]) / 2, F = (M[0] - M[3]) / 2, G = (M[2] + M[1]) / 2, H = (M[2] - M[1]) / 2;
  const double Q = mpj_sqrt(E * E + H * H), R = mpj_sqrt(F * F + G * G);
  const double sx = Q + R, sy = Q - R;
  const double a1 = mpj_atan2(G, F), a2 = mpj_atan2(H, E);
  const double th = (a2 - a1) / 2, ph = (a2 + a1) / 2;
  double st, ct, sp, cp;
  mpj_sincos(th, &st, &ct);
  mpj_sincos(ph, &sp, &cp);
  const double smax = __builtin_fabs(sx) > __builtin_fabs(sy) ? __builtin_fabs(sx) : __builtin_fabs(sy);
  const double tol = 4.440892098500626e-16 * smax;
  const double i1 = __builtin_fabs(sx) > tol ? 1.0 / sx : 0.0;
  const double i2 = __builtin_fabs(sy) > tol ? 1.0 / sy : 0.0;
  Pm[0] = ct * i1 * cp - st * i2 * sp;
  Pm[1] = ct * i1 * sp + st * i2 * cp;
  Pm[2] = -st * i1 * cp - ct * i2 * sp;
  Pm[3] = -st * i1 * sp + ct * i2 * cp;
}

// ILQR.jl:46-67 for instance b
__global__ __launch_bounds__(64) void ilqr_backward_kernel(IlqrDev P, int B, const double* X, const double* D,
                                                           const int* active, double* kout, double* Kout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || (active && !active[b])) return;
  const int N = P.N;
  const double e = P.eps;
  const int V = P.variant;
  double Vx[4], Vxx[16];
  {  // CalculateMatrix(StatesList[:, end], [0 0], TerminalCost): only lx, lxx are used
    const double* s = X + ((size_t)b * N + N - 1) * 4;
    double sp[4], sm[4], t1[4], t2[4], t3[4], t4[4];
    const double c12 = 1 / (12 * (e * e)), c4 = 1 / (4 * (e * e));
    for (int i = 0; i < 4; i++) {
      for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
      sp[i] = s[i] + e;
      sm[i] = s[i] - e;
      Vx[i] = (terminal(V, sp) - terminal(V, sm)) / (2 * e);
    }
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) {
        for (int r = 0; r < 4; r++) { t1[r] = s[r]; t2[r] = s[r]; t3[r] = s[r]; t4[r] = s[r]; }
        if (i == j) {
          t1[i] = s[i] + 2 * e; t2[i] = s[i] + e; t3[i] = s[i] - e; t4[i] = s[i] - 2 * e;
          Vxx[4 * i + j] = c12 * (-terminal(V, t1) + 16 * terminal(V, t2) - 30 * terminal(V, s) +
                                  16 * terminal(V, t3) - terminal(V, t4));
        } else {
          t1[i] = s[i] + e; t1[j] = s[j] + e;
          t2[i] = s[i] - e; t2[j] = s[j] - e;
          t3[i] = s[i] + e; t3[j] = s[j] - e;
          t4[i] = s[i] - e; t4[j] = s[j] + e;
          Vxx[4 * i + j] = c4 * (terminal(V, t1) + terminal(V, t2) - terminal(V, t3) - terminal(V, t4));
        }
      }
  }
  for (int j = N - 2; j >= 0; j--) {
    const double* d = D + ((size_t)b * (N - 1) + j) * ND;
    double A[16], Bm[8], lx[4], lu[2], lxx[16], luu[4], lux[8];
    for (int i = 0; i < 16; i++) A[i] = d[i];
    for (int i = 0; i < 8; i++) Bm[i] = d[16 + i];
    for (int i = 0; i < 4; i++) lx[i] = d[24 + i];
    lu[0] = d[28]; lu[1] = d[29];
    for (int i = 0; i < 16; i++) lxx[i] = d[30 + i];
    for (int i = 0; i < 4; i++) luu[i] = d[46 + i];
    for (int i = 0; i < 8; i++) lux[i] = d[50 + i];
    double Qx[4], Qu[2], Qxx[16], Quu[4], Qux[8], T44[16], T24[8], Pm[4];
    for (int i = 0; i < 4; i++) {
      double acc = A[0 * 4 + i] * Vx[0];
      for (int k = 1; k < 4; k++) acc = acc + A[k * 4 + i] * Vx[k];
      Qx[i] = lx[i] + acc;
    }
    for (int i = 0; i < 2; i++) {
      double acc = Bm[0 * 2 + i] * Vx[0];
      for (int k = 1; k < 4; k++) acc = acc + Bm[k * 2 + i] * Vx[k];
      Qu[i] = lu[i] + acc;
    }
    for (int i = 0; i < 4; i++)
      for (int c = 0; c < 4; c++) {
        double acc = A[0 * 4 + i] * Vxx[0 * 4 + c];
        for (int k = 1; k < 4; k++) acc = acc + A[k * 4 + i] * Vxx[k * 4 + c];
        T44[4 * i + c] = acc;
      }
    for (int i = 0; i < 4; i++)
      for (int c = 0; c < 4; c++) {
        double acc = T44[4 * i + 0] * A[0 * 4 + c];
        for (int k = 1; k < 4; k++) acc = acc + T44[4 * i + k] * A[k * 4 + c];
        Qxx[4 * i + c] = lxx[4 * i + c] + acc;
      }
    for (int i = 0; i < 2; i++)
      for (int c = 0; c < 4; c++) {
        double acc = Bm[0 * 2 + i] * Vxx[0 * 4 + c];
        for (int k = 1; k < 4; k++) acc = acc + Bm[k * 2 + i] * Vxx[k * 4 + c];
        T24[4 * i + c] = acc;
      }
    for (int i = 0; i < 2; i++)
      for (int c = 0; c < 2; c++) {
        double acc = T24[4 * i + 0] * Bm[0 * 2 + c];
        for (int k = 1; k < 4; k++) acc = acc + T24[4 * i + k] * Bm[k * 2 + c];
        Quu[2 * i + c] = luu[2 * i + c] + acc;
      }
    for (int i = 0; i < 2; i++)
      for (int c = 0; c < 4; c++) {
        double acc = T24[4 * i + 0] * A[0 * 4 + c];
        for (int k = 1; k < 4; k++) acc = acc + T24[4 * i + k] * A[k * 4 + c];
        Qux[4 * i + c] = lux[4 * i + c] + acc;
      }
    pinv2(Quu, Pm);
    double kk[2], KK[8];
    for (int i = 0; i < 2; i++) kk[i] = (-Pm[2 * i + 0]) * Qu[0] + (-Pm[2 * i + 1]) * Qu[1];
    for (int i = 0; i < 2; i++)
      for (int c = 0; c < 4; c++) KK[4 * i + c] = (-Pm[2 * i + 0]) * Qux[0 * 4 + c] + (-Pm[2 * i + 1]) * Qux[1 * 4 + c];
    double* ko = kout + ((size_t)b * (N - 1) + j) * 2;
    double* Ko = Kout + ((size_t)b * (N - 1) + j) * 8;
    ko[0] = kk[0];
    ko[1] = kk[1];
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 4; c++) Ko[2 * c + r] = KK[4 * r + c];
    double qk[2];
    for (int i = 0; i < 2; i++) qk[i] = Quu[2 * i + 0] * kk[0] + Quu[2 * i + 1] * kk[1];
    for (int i = 0; i < 4; i++) Vx[i] = Qx[i] - (KK[0 * 4 + i] * qk[0] + KK[1 * 4 + i] * qk[1]);
    double KQ[8];
    for (int i = 0; i < 4; i++)
      for (int c = 0; c < 2; c++) KQ[2 * i + c] = KK[0 * 4 + i] * Quu[0 * 2 + c] + KK[1 * 4 + i] * Quu[1 * 2 + c];
    for (int i = 0; i < 4; i++)
      for (int c = 0; c < 4; c++)
        Vxx[4 * i + c] = Qxx[4 * i + c] - (KQ[2 * i + 0] * KK[0 * 4 + c] + KQ[2 * i + 1] * KK[1 * 4 + c]);
  }
}

// ILQR.jl:72-80: one closed-loop roll out at step size alpha; returns TotalCost
__device__ double forward_trial(const IlqrDev& P, const double* X, const double* U, const double* k,
                                const double* Kg, double alpha, double* Xn, double* Un) {
  const int N = P.N;
  for (int r = 0; r < 4; r++) Xn[r] = X[r];
  for (int i = 0; i < N - 1; i++) {
    double dx[4], u[2];
    for (int r = 0; r < 4; r++) dx[r] = Xn[4 * i + r] - X[4 * i + r];
    for (int r = 0; r < 2; r++) {
      double acc = Kg[8 * i + 2 * 0 + r] * dx[0];
      for (int c = 1; c < 4; c++) acc = acc + Kg[8 * i + 2 * c + r] * dx[c];
      u[r] = (U[2 * i + r] + alpha * k[2 * i + r]) + acc;
    }
    Un[2 * i] = u[0];
    Un[2 * i + 1] = u[1];
    const UPre q = upre(u[1]);
    rk4(Xn + 4 * i, u[0], q, P.dT, Xn + 4 * (i + 1));
  }
  Un[2 * (N - 1)] = 0.0;
  Un[2 * (N - 1) + 1] = 0.0;
  return total_cost(P.variant, N, Xn, Un);
}

__global__ __launch_bounds__(64) void ilqr_forward_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                          const double* k, const double* Kg, const double* alpha,
                                                          double* Xn, double* Un, double* Jn) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const size_t N = P.N;
  Jn[b] = forward_trial(P, X + b * N * 4, U + b * N * 2, k + b * (N - 1) * 2, Kg + b * (N - 1) * 8, alpha[b],
                        Xn + b * N * 4, Un + b * N * 2);
}

// ILQR.jl:70-88 after the backward sweep: line search, accept, convergence test.
// state[b]: J (cost at the start of this iteration, i.e. the previous J_new).
__global__ __launch_bounds__(64) void ilqr_search_kernel(IlqrDev P, int B, double* X, double* U, const double* k,
                                                         const double* Kg, double* Xn, double* Un, double* Jcur,
                                                         int* active, int* iters, int* flags, int* n_active) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || !active[b]) return;
  const size_t N = P.N;
  double* Xb = X + b * N * 4;
  double* Ub = U + b * N * 2;
  double* Xnb = Xn + b * N * 4;
  double* Unb = Un + b * N * 2;
  const double J = Jcur[b];
  double Jn = J;
  double alpha = 1.0;
  int ls = 0;
  while (Jn >= J) {
    Jn = forward_trial(P, Xb, Ub, k + b * (N - 1) * 2, Kg + b * (N - 1) * 8, alpha, Xnb, Unb);
    alpha = alpha / 2;
    ls++;
    if (P.alpha_floor > 0 && alpha <= P.alpha_floor) break;
    if (ls >= P.max_ls) { atomicOr(flags + b, 1); break; }
  }
  for (size_t i = 0; i < N * 4; i++) Xb[i] = Xnb[i];
  for (size_t i = 0; i < N * 2; i++) Ub[i] = Unb[i];
  Jcur[b] = Jn;
  const int it = iters[b] + 1;
  iters[b] = it;
  bool go = __builtin_fabs((Jn - J) / J) > P.tol;
  if (go && it > P.max_iter) {
    atomicOr(flags + b, 2);
    go = false;
  }
  active[b] = go;
  if (go) atomicAdd(n_active, 1);
}

__global__ __launch_bounds__(64) void ilqr_rollout_kernel(IlqrDev P, int B, const double* x0, const double* U,
                                                          double* X, double* J) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const size_t N = P.N;
  double* Xb = X + b * N * 4;
  const double* Ub = U + b * N * 2;
  for (int r = 0; r < 4; r++) Xb[r] = x0[4 * b + r];
  for (size_t i = 0; i + 1 < N; i++) {
    const UPre q = upre(Ub[2 * i + 1]);
    rk4(Xb + 4 * i, Ub[2 * i], q, P.dT, Xb + 4 * (i + 1));
  }
  J[b] = total_cost(P.variant, (int)N, Xb, Ub);
}

__global__ void ilqr_init_kernel(IlqrDev P, int B, const double* X, const double* U, double* Jcur, int* active,
                                 int* iters, int* flags) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Jcur[b] = total_cost(P.variant, P.N, X + (size_t)b * P.N * 4, U + (size_t)b * P.N * 2);
  active[b] = 1;
  iters[b] = 1;
  flags[b] = 0;
}

int make_ilqr(mp_ctx* ctx, const mp_ilqr_params* p, int B, IlqrDev* D) {
  MP_CHECK(ctx, p != nullptr, "params is NULL");
  MP_CHECK(ctx, B >= 1, "B (%d) must be >= 1", B);
  MP_CHECK(ctx, p->N >= 2 && p->N <= 100000, "N (%d) must be >= 2", p->N);
  MP_CHECK(ctx, p->variant == MP_ILQR_OPTIMALCONTROL || p->variant == MP_ILQR_PARKING, "bad variant %d", p->variant);
  MP_CHECK(ctx, p->dT > 0 && p->eps > 0, "dT and eps must be > 0");
  D->N = p->N;
  D->variant = p->variant;
  D->dT = p->dT;
  D->eps = p->eps;
  D->alpha_floor = p->alpha_floor;
  D->tol = p->tol;
  D->max_iter = p->max_iter > 0 ? p->max_iter : 1000;
  D->max_ls = p->max_ls > 0 ? p->max_ls : 200;
  return MP_OK;
}

int run_backward(mp_ctx* ctx, const IlqrDev& D, int B, const double* dX, const double* dU, const int* active,
                 double* dk, double* dK) {
  const size_t n = (size_t)B * (D.N - 1);
  double* dD = (double*)mp_ws(ctx, WS_ILQR0, sizeof(double) * n * ND);
  if (!dD) return MP_ERR_NOMEM;
  mp_time_begin(ctx);  // the timed region covers both kernels of the backward pass
  hipLaunchKernelGGL(ilqr_deriv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, D, B, dX, dU,
                     active, dD);
  MP_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(ilqr_backward_kernel, dim3((B + 63) / 64), dim3(64), 0, ctx->stream, D, B, dX, dD, active, dk,
                     dK);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  return MP_OK;
}

}  // namespace

extern "C" {

int mp_ilqr_rollout(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* x0, const double* U, double* X,
                    double* J) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, x0 && U && X && J, "required pointer is NULL");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t N = D.N;
  const double* dx0 = mp_upload(ctx, WS_IO0, x0, 4 * (size_t)B, &st);
  const double* dU = mp_upload(ctx, WS_IO1, U, 2 * N * B, &st);
  double* dX = mp_alloc_out(ctx, WS_IO2, X, 4 * N * B, &st);
  double* dJ = mp_alloc_out(ctx, WS_IO3, J, (size_t)B, &st);
  if (st) return st;
  hipLaunchKernelGGL(ilqr_rollout_kernel, dim3((B + 63) / 64), dim3(64), 0, ctx->stream, D, B, dx0, dU, dX, dJ);
  MP_HIP(ctx, hipGetLastError());
  if ((st = mp_download(ctx, X, (const double*)dX, 4 * N * B))) return st;
  if ((st = mp_download(ctx, J, (const double*)dJ, (size_t)B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_ilqr_backward(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X, const double* U, double* k,
                     double* Kg) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, X && U && k && Kg, "required pointer is NULL");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t N = D.N;
  const double* dX = mp_upload(ctx, WS_IO0, X, 4 * N * B, &st);
  const double* dU = mp_upload(ctx, WS_IO1, U, 2 * N * B, &st);
  double* dk = mp_alloc_out(ctx, WS_IO2, k, 2 * (N - 1) * B, &st);
  double* dK = mp_alloc_out(ctx, WS_IO3, Kg, 8 * (N - 1) * B, &st);
  if (st) return st;
  if ((st = run_backward(ctx, D, B, dX, dU, nullptr, dk, dK))) return st;
  if ((st = mp_download(ctx, k, (const double*)dk, 2 * (N - 1) * B))) return st;
  if ((st = mp_download(ctx, Kg, (const double*)dK, 8 * (N - 1) * B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_ilqr_forward(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X, const double* U,
                    const double* k, const double* Kg, const double* alpha, double* Xnew, double* Unew,
                    double* Jnew) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, X && U && k && Kg && alpha && Xnew && Unew && Jnew, "required pointer is NULL");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t N = D.N;
  const double* dX = mp_upload(ctx, WS_IO0, X, 4 * N * B, &st);
  const double* dU = mp_upload(ctx, WS_IO1, U, 2 * N * B, &st);
  const double* dk = mp_upload(ctx, WS_IO2, k, 2 * (N - 1) * B, &st);
  const double* dK = mp_upload(ctx, WS_IO3, Kg, 8 * (N - 1) * B, &st);
  const double* da = mp_upload(ctx, WS_IO4, alpha, (size_t)B, &st);
  double* dXn = mp_alloc_out(ctx, WS_IO5, Xnew, 4 * N * B, &st);
  double* dUn = mp_alloc_out(ctx, WS_IO6, Unew, 2 * N * B, &st);
  double* dJ = mp_alloc_out(ctx, WS_IO7, Jnew, (size_t)B, &st);
  if (st) return st;
  mp_time_begin(ctx);
  hipLaunchKernelGGL(ilqr_forward_kernel, dim3((B + 63) / 64), dim3(64), 0, ctx->stream, D, B, dX, dU, dk, dK, da,
                     dXn, dUn, dJ);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  if ((st = mp_download(ctx, Xnew, (const double*)dXn, 4 * N * B))) return st;
  if ((st = mp_download(ctx, Unew, (const double*)dUn, 2 * N * B))) return st;
  if ((st = mp_download(ctx, Jnew, (const double*)dJ, (size_t)B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_ilqr_backward_dev(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X, const double* U,
                         double* k, double* Kg) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, X && U && k && Kg, "required pointer is NULL");
  return run_backward(ctx, D, B, X, U, nullptr, k, Kg);
}

int mp_ilqr_forward_dev(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X, const double* U,
                        const double* k, const double* Kg, const double* alpha, double* Xnew, double* Unew,
                        double* Jnew) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, X && U && k && Kg && alpha && Xnew && Unew && Jnew, "required pointer is NULL");
  mp_time_begin(ctx);
  hipLaunchKernelGGL(ilqr_forward_kernel, dim3((B + 63) / 64), dim3(64), 0, ctx->stream, D, B, X, U, k, Kg, alpha,
                     Xnew, Unew, Jnew);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  return MP_OK;
}

int mp_ilqr_solve(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, double* X, double* U, double* J,
                  int32_t* iters) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, X && U && J && iters, "required pointer is NULL");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t N = D.N;
  double* dX = (double*)mp_upload(ctx, WS_IO0, X, 4 * N * B, &st);
  double* dU = (double*)mp_upload(ctx, WS_IO1, U, 2 * N * B, &st);
  double* dk = (double*)mp_ws(ctx, WS_IO2, sizeof(double) * 2 * (N - 1) * B);
  double* dK = (double*)mp_ws(ctx, WS_IO3, sizeof(double) * 8 * (N - 1) * B);
  double* dXn = (double*)mp_ws(ctx, WS_IO4, sizeof(double) * 4 * N * B);
  double* dUn = (double*)mp_ws(ctx, WS_IO5, sizeof(double) * 2 * N * B);
  double* dJ = (double*)mp_ws(ctx, WS_IO6, sizeof(double) * B);
  int* dint = (int*)mp_ws(ctx, WS_IO7, sizeof(int) * (3 * (size_t)B + 1));
  if (st || !dk || !dK || !dXn || !dUn || !dJ || !dint) return st ? st : MP_ERR_NOMEM;
  int* dact = dint;
  int* dit = dint + B;
  int* dfl = dint + 2 * B;
  int* dn = dint + 3 * B;
  const dim3 g1((B + 63) / 64), b1(64);
  hipLaunchKernelGGL(ilqr_init_kernel, g1, b1, 0, ctx->stream, D, B, dX, dU, dJ, dact, dit, dfl);
  MP_HIP(ctx, hipGetLastError());
  int* hn = (int*)mp_pinned(ctx, sizeof(int));
  if (!hn) return mp_fail(ctx, MP_ERR_NOMEM, "pinned allocation failed");
  for (int outer = 0; outer <= D.max_iter + 1; outer++) {
    if ((st = run_backward(ctx, D, B, dX, dU, dact, dk, dK))) return st;
    MP_HIP(ctx, hipMemsetAsync(dn, 0, sizeof(int), ctx->stream));
    mp_time_begin(ctx);
    hipLaunchKernelGGL(ilqr_search_kernel, g1, b1, 0, ctx->stream, D, B, dX, dU, dk, dK, dXn, dUn, dJ, dact, dit,
                       dfl, dn);
    MP_HIP(ctx, hipGetLastError());
    mp_time_end(ctx);
    MP_HIP(ctx, hipMemcpyAsync(hn, dn, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (*hn == 0) break;
  }
  std::vector<int> hfl(B);
  if ((st = mp_download(ctx, X, (const double*)dX, 4 * N * B))) return st;
  if ((st = mp_download(ctx, U, (const double*)dU, 2 * N * B))) return st;
  if ((st = mp_download(ctx, J, (const double*)dJ, (size_t)B))) return st;
  if ((st = mp_download(ctx, iters, (const int*)dit, (size_t)B))) return st;
  if ((st = mp_download(ctx, hfl.data(), (const int*)dfl, (size_t)B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  int any = 0;
  for (int b = 0; b < B; b++) any |= hfl[b];
  if (any & 1) return mp_fail(ctx, MP_ERR_NUMERIC, "line search hit max_ls for some instance (the reference would loop forever)");
  if (any & 2) return mp_fail(ctx, MP_ERR_NUMERIC, "max_iter reached before |dJ/J| <= tol for some instance");
  return MP_OK;
}

}  // extern "C"
