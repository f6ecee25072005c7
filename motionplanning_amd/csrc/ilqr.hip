// ilqr.hip — batched iLQR (OptimalControl/ILQR/{Dynamics,Cost,GetMatrix,ILQR}.jl and
// the PathPlanning/Parking_ILQR variant) for gfx950 + C-ABI entry points.
//
// Per outer iteration (ILQR.jl:44-88) for the active instances of a batch:
//   ilqr_deriv_kernel / ilqr_deriv4_kernel   LocallyLinearizeDynamics (12 RK4) and CalculateMatrix
//                         (130 StageCost evaluations) by finite differences for every (instance,
//                         knot): one thread per record, or -- launches with few active instances --
//                         four waves per 64 records, one part of the derivatives each.  Control-only
//                         sub-expressions (tan δ, β, cos β, the sigmoid barriers) are evaluated once
//                         per distinct perturbed control and reused: the same function of the same
//                         bits, so every derivative is bit-identical to the scalar restatement.
//   ilqr_backward_quad_kernel   the Riccati sweep j = N-2..0 (ILQR.jl:46-67) on a lane quad per
//                         instance, fed from LDS by a loader wave; Julia's pinv (LAPACK's 2x2 path).
//   line search (ILQR.jl:70-86), trial m at α = 2^-m on a lane quad (a lane pair in the pipelined
//                         launch's round 0, throughput-bound there): round 0 (16 trials per
//                         instance at once), then the trials 16..m* of the instances still searching
//                         all at once in the next launch (ilqr_search_pipe_kernel: beside the next
//                         iteration's round 0) and ilqr_search_finish_kernel (accept); with few
//                         instances left, every trial 0..m* in one pass.  The accepted trial is the
//                         first that would end the sequential loop, so the results are the loop's.
// The host loops until every instance has met |ΔJ/J| <= tol (or its max_iter).
#include "../../include/mp_jlmath.h"
#include "runtime.hpp"

namespace {

constexpr int ND = 58;  // derivative record: A16 B8 lx4 lu2 lxx16 luu4 lux8

struct IlqrDev {
  int N, variant, max_iter, max_ls;
  double dT, eps, alpha_floor, tol;
  int ls_cap;  // last trial index the halving loop can reach (max_ls - 1, or the alpha_floor stop)
  // (mp_ilqr_solve, MPGPU_ILQR_MIRROR) the backward pass's first kernel reports the previous search's
  // counts -- (seq << 32) | active, (seq << 32) | pending -- to host memory (ilqr_mirror)
  unsigned long long* mirror;
  int mirror_seq;
};

// the first thread of a backward pass's first kernel: n_dev = the list count the previous iteration's search
// wrote (final: that launch is complete), n_dev[-1] its pending count; vector stores to fine-grained host memory
__device__ __forceinline__ void ilqr_mirror(const IlqrDev& P, const int* n_dev) {
  if (P.mirror && n_dev && blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long q = (unsigned long long)(unsigned)P.mirror_seq << 32;
    __hip_atomic_store(P.mirror + 1, q | (unsigned)n_dev[-1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(P.mirror, q | (unsigned)n_dev[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ILQR.jl:76-83 break tests after trial m (alpha is then 2^-(m+1)): the floor test first
// (Parking_ILQR), then the max_ls safety cap.
__host__ __device__ inline bool floor_stop(const IlqrDev& P, int m) {
  return P.alpha_floor > 0 && ldexp(1.0, -(m + 1)) <= P.alpha_floor;
}

struct UPre {  // control-only part of Dynamics (Dynamics.jl:8-12)
  double tdl, beta, cb;
};

// libm policy.  LM<true>: straight-line FDLIBM cores (include/mp_jlmath.h *_fast): no branch
// at all, so a whole knot is one basic block the scheduler can interleave; a lane whose
// argument leaves a core's fast range sets `bad`, and the kernel then re-runs that unit of
// work (knot / sweep / trial) for the wave with LM<false>, the exact branchy routines.  The
// cores equal the exact routines bit for bit on their fast range (tests/test_jlmath.py).
template <bool F> struct LM;
// A/B builds: -DMP_ILQR_EXACT (exact libm only), -DMP_ILQR_NOREDO (timing only: no fallback)
#if defined(MP_ILQR_EXACT)
constexpr bool kFast = false;
#else
constexpr bool kFast = true;
#endif
// Per kernel (measured, gfx950, configs[2]): the straight-line cores pay off only in the Riccati
// sweep (355 vs 382 us).  The derivative kernel (405,504 threads, lanes of a wave take the same
// libm branches) runs the exact routines in 154 us vs 296 us, and the one-thread-per-instance
// forward trial / roll out (64 waves, latency-bound: fewer instructions win) in 361 vs 690 us.
// A/B (-DMP_ILQR_FASTSC): the forward trial / roll out's four RK4 stage sincos on the
// straight-line core (rk4_ilp, independent of each other) with an exact redo for arguments out
// of range.  Measured slower: forward 386 vs 361 us, roll out 356 vs 276 us (a lone wave is
// issue-limited: the straight-line core's extra instructions cost more than the overlap gains).
#if defined(MP_ILQR_NOQUAD) || defined(MP_ILQR_FASTFWD)
constexpr bool kFwdQuad = false;
#else
constexpr bool kFwdQuad = true;  // ilqr_forward_quad_kernel: a lane quad per instance
#ifndef ILQR_SEARCH_L
#define ILQR_SEARCH_L 4
#endif
constexpr int kSearchL = ILQR_SEARCH_L;  // lanes per line-search trial in mp_ilqr_solve (1 or 4)
#ifndef ILQR_ROUND0_L
#define ILQR_ROUND0_L 2
#endif
constexpr int kRound0L = ILQR_ROUND0_L;  // lanes per trial in the pipelined launch's round 0 (2 or 4) ...
#ifndef ILQR_PAIR_MIN
#define ILQR_PAIR_MIN 2048
#endif
constexpr int kPairMin = ILQR_PAIR_MIN;  // ... while at least this many instances are active (else 4)
#ifndef ILQR_ONEPASS_MAX
#define ILQR_ONEPASS_MAX 512
#endif
constexpr int kOnePassMax = ILQR_ONEPASS_MAX;  // active instances up to which the search is one pass
#ifndef ILQR_PIPE
#define ILQR_PIPE 1
#endif
constexpr bool kPipe = ILQR_PIPE;  // overlap each rest pass with the next iteration's round 0
#ifndef ILQR_DERIV4_MAX
#define ILQR_DERIV4_MAX 2048
#endif
constexpr int kDeriv4Max = ILQR_DERIV4_MAX;  // derivative launches for at most this many instances: 4 lanes each
#ifndef ILQR_SEARCH_G
#define ILQR_SEARCH_G 16
#endif
constexpr int kSearchG = ILQR_SEARCH_G;  // trials per instance in the first round (a power of two <= 16)
#endif
#if defined(MP_ILQR_FASTSC)
constexpr bool kFastSC = true;
#else
constexpr bool kFastSC = false;
#endif
#if defined(MP_ILQR_FASTFWD)  // A/B build (measured slower: forward 689 vs 363 us, roll out 341 vs 277 us)
constexpr bool kFastDeriv = false, kFastBwd = kFast, kFastFwd = kFast;
#else
constexpr bool kFastDeriv = false, kFastBwd = kFast, kFastFwd = false;
#endif
#if defined(MP_ILQR_NOREDO)
constexpr bool kRedo = false;
#else
constexpr bool kRedo = true;
#endif
#if defined(MP_ILQR_BADSTAT)  // diagnostics build: print arguments that leave a core's range
__device__ int g_nbad = 0;
#endif
template <> struct LM<true> {
#if !defined(MP_ILQR_BADSTAT)
  static __device__ __forceinline__ double tan(double x, int& b) { return mpj_tan_wide(x, &b); }
  static __device__ __forceinline__ double atan(double x, int&) { return mpj_atan_bl(x); }
  static __device__ __forceinline__ void sincos(double x, double* s, double* c, int& b) { mpj_sincos_wide(x, s, c, &b); }
  // Julia's table-driven exp is one basic block for |x| <= 708.39 (the far branch is wave-uniform here)
  static __device__ __forceinline__ double exp(double x, int&) { return mpj_exp(x); }
  static __device__ __forceinline__ double atan2(double y, double x, int& b) { return mpj_atan2_fast(y, x, &b); }
#else
  static __device__ double tan(double x, int& b) { int t = 0; double r = mpj_tan_wide(x, &t); if (t) { b |= 1; if (atomicAdd(&g_nbad, 1) < 8) printf("tan %.17g\n", x); } return r; }
  static __device__ double atan(double x, int&) { return mpj_atan_bl(x); }
  static __device__ void sincos(double x, double* s, double* c, int& b) { int t = 0; mpj_sincos_wide(x, s, c, &t); if (t) { b |= 2; if (atomicAdd(&g_nbad, 1) < 8) printf("sincos %.17g\n", x); } }
  static __device__ double exp(double x, int&) { return mpj_exp(x); }
  static __device__ double atan2(double y, double x, int& b) { int t = 0; double r = mpj_atan2_fast(y, x, &t); if (t) { b |= 8; if (atomicAdd(&g_nbad, 1) < 8) printf("atan2 %.17g %.17g\n", y, x); } return r; }
#endif
};
template <> struct LM<false> {
  static __device__ __forceinline__ double tan(double x, int&) { return mpj_tan(x); }
  static __device__ __forceinline__ double atan(double x, int&) { return mpj_atan(x); }
  static __device__ __forceinline__ void sincos(double x, double* s, double* c, int&) { mpj_sincos(x, s, c); }
  static __device__ __forceinline__ double exp(double x, int&) { return mpj_exp(x); }
  static __device__ __forceinline__ double atan2(double y, double x, int&) { return mpj_atan2(y, x); }
};

template <bool F>
__device__ __forceinline__ UPre upre(double dl, int& bad) {
  const double la = 1.56, lb = 1.64;
  UPre q;
  q.tdl = LM<F>::tan(dl, bad);
  q.beta = LM<F>::atan(la / (la + lb) * q.tdl, bad);
  double sb;
  LM<F>::sincos(q.beta, &sb, &q.cb, bad);  // cos β (the cos of sincos == mpj_cos bit for bit)
  return q;
}

// Dynamics.jl:1-16
template <bool F>
__device__ __forceinline__ void dyn(const double* s, double ax, const UPre& q, double* d, int& bad) {
  const double la = 1.56, lb = 1.64;
  double sb, cbb;
  LM<F>::sincos(s[3] + q.beta, &sb, &cbb, bad);
  d[0] = s[2] * cbb;
  d[1] = s[2] * sb;
  d[2] = ax;
  d[3] = s[2] * q.cb * q.tdl / (la + lb);
}

// RK4Integration, Dynamics.jl:18-28, as its increment: o[i] = inc[i] + s[i] with
// inc[i] = 1/6·(k1 + 2k2 + 2k3 + k4)·dT.  dyn reads only s[2] (speed) and s[3] (heading), so the
// stage slopes -- and inc -- do not depend on s[0] / s[1] at all (knot_derivs uses that).
template <bool F>
__device__ __forceinline__ void rk4_inc(const double* s, double ax, const UPre& q, double dT, double* inc, int& bad) {
  double k1[4], k2[4], k3[4], k4[4], x2[4], x3[4], x4[4];
  dyn<F>(s, ax, q, k1, bad);
#pragma unroll
  for (int i = 0; i < 4; i++) x2[i] = s[i] + dT / 2 * k1[i];
  dyn<F>(x2, ax, q, k2, bad);
#pragma unroll
  for (int i = 0; i < 4; i++) x3[i] = s[i] + dT / 2 * k2[i];
  dyn<F>(x3, ax, q, k3, bad);
#pragma unroll
  for (int i = 0; i < 4; i++) x4[i] = s[i] + dT * k3[i];
  dyn<F>(x4, ax, q, k4, bad);
#pragma unroll
  for (int i = 0; i < 4; i++) inc[i] = 1.0 / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]) * dT;
}
template <bool F>
__device__ __forceinline__ void rk4(const double* s, double ax, const UPre& q, double dT, double* o, int& bad) {
  double inc[4];
  rk4_inc<F>(s, ax, q, dT, inc, bad);
#pragma unroll
  for (int i = 0; i < 4; i++) o[i] = inc[i] + s[i];
}
// rk4_inc with the (sin, cos) of the first NS stage headings supplied in sc (NS = 0: all computed,
// stages 1-2 written to sc).  knot_derivs' RK4s of the knot's own state, of its speed ± eps and of
// ax ± eps have bit-identical stage-1 headings s[3] + β, and the ax pair also the stage-2 heading
// (ax enters only the speed slope k[2]): the same sincos on the same argument, evaluated once.
template <bool F, int NS>
__device__ __forceinline__ void rk4_inc_sh(const double* s, double ax, const UPre& q, double dT, double* inc,
                                           int& bad, double (&sc)[2][2]) {
  const double la = 1.56, lb = 1.64;
  double k[4][4], xs[4];
#pragma unroll
  for (int st = 0; st < 4; st++) {
    const double* xi = st == 0 ? s : xs;
    double sn, cs;
    if (st < NS) {
      sn = sc[st][0];
      cs = sc[st][1];
    } else {
      LM<F>::sincos(xi[3] + q.beta, &sn, &cs, bad);
      if (NS == 0 && st < 2) {
        sc[st][0] = sn;
        sc[st][1] = cs;
      }
    }
    k[st][0] = xi[2] * cs;  // dyn (Dynamics.jl:1-16)
    k[st][1] = xi[2] * sn;
    k[st][2] = ax;
    k[st][3] = xi[2] * q.cb * q.tdl / (la + lb);
    if (st < 3) {
      double nx[4];
#pragma unroll
      for (int i = 0; i < 4; i++) nx[i] = s[i] + (st < 2 ? dT / 2 : dT) * k[st][i];
#pragma unroll
      for (int i = 0; i < 4; i++) xs[i] = nx[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) inc[i] = 1.0 / 6 * (k[0][i] + 2 * k[1][i] + 2 * k[2][i] + k[3][i]) * dT;
}

// The x / y columns of the dynamics Jacobian (GetMatrix.jl:3-25, states ± eps): RK4 of the
// perturbed state is the unperturbed increment plus the perturbed state (rk4_inc), so one RK4 of
// the knot's own state gives all four perturbed evaluations -- the same operations on the same
// operands as four rk4 calls, so the same bits.
__device__ __forceinline__ void dyn_jac_xy_inc(const double* s, const double* inc, double e, double* out, size_t stride) {
#pragma unroll
  for (int i = 0; i < 2; i++) {
    double sp[4], sm[4];
#pragma unroll
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[i] = s[i] + e;
    sm[i] = s[i] - e;
#pragma unroll
    for (int r = 0; r < 4; r++) out[(size_t)(4 * r + i) * stride] = ((inc[r] + sp[r]) - (inc[r] + sm[r])) / (2 * e);
  }
}
template <bool F>
__device__ __forceinline__ void dyn_jac_xy(const double* s, double ax, const UPre& q, double dT, double e, double* out,
                                           size_t stride, int& bad) {
  double inc[4];
  rk4_inc<F>(s, ax, q, dT, inc, bad);
  dyn_jac_xy_inc(s, inc, e, out, stride);
}

// RK4Integration with the four stage headings computed first.  The stage speed and heading
// (dyn's d[2] = ax, d[3] = s2·cb·tδ/L) never depend on a sine or cosine, so the four stage
// sincos are independent of each other: with the straight-line core (SC = true) the scheduler
// overlaps them instead of running four dependent libm chains.  The same operations on the
// same operands as rk4, so the same bits.
template <bool SC>
__device__ __forceinline__ void rk4_ilp(const double* s, double ax, const UPre& q, double dT, double* o, int& bad) {
  const double la = 1.56, lb = 1.64;
  const double k1_3 = s[2] * q.cb * q.tdl / (la + lb);
  const double x2_2 = s[2] + dT / 2 * ax, x2_3 = s[3] + dT / 2 * k1_3;
  const double k2_3 = x2_2 * q.cb * q.tdl / (la + lb);
  const double x3_2 = s[2] + dT / 2 * ax, x3_3 = s[3] + dT / 2 * k2_3;
  const double k3_3 = x3_2 * q.cb * q.tdl / (la + lb);
  const double x4_2 = s[2] + dT * ax, x4_3 = s[3] + dT * k3_3;
  const double k4_3 = x4_2 * q.cb * q.tdl / (la + lb);
  double s1, c1, s2, c2, s3, c3, s4, c4;
  LM<SC>::sincos(s[3] + q.beta, &s1, &c1, bad);
  LM<SC>::sincos(x2_3 + q.beta, &s2, &c2, bad);
  LM<SC>::sincos(x3_3 + q.beta, &s3, &c3, bad);
  LM<SC>::sincos(x4_3 + q.beta, &s4, &c4, bad);
  const double k1[4] = {s[2] * c1, s[2] * s1, ax, k1_3};
  const double k2[4] = {x2_2 * c2, x2_2 * s2, ax, k2_3};
  const double k3[4] = {x3_2 * c3, x3_2 * s3, ax, k3_3};
  const double k4[4] = {x4_2 * c4, x4_2 * s4, ax, k4_3};
#pragma unroll
  for (int i = 0; i < 4; i++) o[i] = 1.0 / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]) * dT + s[i];
}

// sigmoid_boundary, Cost.jl:42-49
template <bool F>
__device__ __forceinline__ double sigmoid_boundary(double st, double mn, double mx, int& bad) {
  const double slope = 10, mag = 100;
  const double c1 = 1 / (1 + LM<F>::exp(-slope * (st - mx), bad));
  const double c2 = 1 / (1 + LM<F>::exp(slope * (st - mn), bad));
  return mag * (c1 + c2);
}
template <bool F>
__device__ __forceinline__ double sig_d(double dl, int& bad) {
  return sigmoid_boundary<F>(dl, -MPJ_PI / 6, MPJ_PI / 6, bad);
}
template <bool F>
__device__ __forceinline__ double sig_a(double ax, int& bad) { return sigmoid_boundary<F>(ax, -2, 2, bad); }

// StageCost (Cost.jl:10-27 / Parking_ILQR/Cost.jl:21) with the barrier terms supplied
__device__ __forceinline__ double stage_pre(int variant, const double* s, double ax, double dl, double sd,
                                            double sa) {
  const double x = s[0], y = s[1], ux = s[2], psi = s[3];
  if (variant == MP_ILQR_PARKING)
    return 0.01 * (ax * ax) + 0.01 * (dl * dl) + 10 * (y * y) + 0.5 * (x * x) + 100 * (psi * psi) +
           0.01 * (ux * ux) + sd + sa;
  return 10 * (ax * ax) + 10 * (dl * dl) + 0.01 * (ux * ux) + sd + sa;
}
template <bool F>
__device__ __forceinline__ double stage(int variant, const double* s, const double* u, int& bad) {
  return stage_pre(variant, s, u[0], u[1], sig_d<F>(u[1], bad), sig_a<F>(u[0], bad));
}
// TerminalCost, Cost.jl:29-40
__device__ __forceinline__ double terminal(int variant, const double* s) {
  const double x = s[0], y = s[1], ux = s[2], psi = s[3];
  const double w = variant == MP_ILQR_PARKING ? 10 : 1000;
  return w * (((x - 0.0) * (x - 0.0) + (y - 0.0) * (y - 0.0)) + 0.1 * ((ux - 0.0) * (ux - 0.0)) +
              1 * ((psi - 0.0) * (psi - 0.0)));
}

__device__ double total_cost(int variant, int N, const double* X, const double* U) {  // exact libm
  double J = 0.0;
  int bad = 0;
  for (int i = 0; i < N - 1; i++) J = J + stage<false>(variant, X + 4 * i, U + 2 * i, bad);
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

// LocallyLinearizeDynamics + CalculateMatrix for one knot (GetMatrix.jl:3-91).  Output
// component q goes to out[q * stride] (the record is component-major across instances, so
// consecutive threads store consecutive doubles); every loop is unrolled so the perturbed
// states stay in registers (no scratch).
template <bool F>
__device__ __forceinline__ void knot_cost_derivs(const IlqrDev& P, const double* s, const double* u, double* out,
                                                 size_t stride, int& bad);
// the dynamics Jacobians of knot_derivs (LocallyLinearizeDynamics, GetMatrix.jl:70-91): A, B
template <bool F>
__device__ __forceinline__ void knot_dyn_derivs(const IlqrDev& P, const double* s, const double* u, double* out,
                                                size_t stride, int& bad) {
  const double e = P.eps;
#define DOUT(q) out[(size_t)(q) * stride]
  // ---- dynamics Jacobians: A (row-major 4x4) at 0, B (4x2) at 16
  const UPre q0 = upre<F>(u[1], bad);
  double sp[4], sm[4], fp[4], fm[4], inc[4], incm[4], sc[2][2];
  rk4_inc_sh<F, 0>(s, u[0], q0, P.dT, inc, bad, sc);  // the knot's own state: stage 1-2 sincos kept
  dyn_jac_xy_inc(s, inc, e, out, stride);
  {  // speed ± eps: stage 1's heading is s[3]
#pragma unroll
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[2] = s[2] + e;
    sm[2] = s[2] - e;
    rk4_inc_sh<F, 1>(sp, u[0], q0, P.dT, inc, bad, sc);
    rk4_inc_sh<F, 1>(sm, u[0], q0, P.dT, incm, bad, sc);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(4 * r + 2) = ((inc[r] + sp[r]) - (incm[r] + sm[r])) / (2 * e);
  }
  {  // heading ± eps
#pragma unroll
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[3] = s[3] + e;
    sm[3] = s[3] - e;
    rk4<F>(sp, u[0], q0, P.dT, fp, bad);
    rk4<F>(sm, u[0], q0, P.dT, fm, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(4 * r + 3) = (fp[r] - fm[r]) / (2 * e);
  }
  {  // ax perturbation leaves the δ-only terms unchanged (and stage 1-2 headings: rk4_inc_sh)
    rk4_inc_sh<F, 2>(s, u[0] + e, q0, P.dT, inc, bad, sc);
    rk4_inc_sh<F, 2>(s, u[0] - e, q0, P.dT, incm, bad, sc);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(16 + 2 * r + 0) = ((inc[r] + s[r]) - (incm[r] + s[r])) / (2 * e);
    const UPre qp = upre<F>(u[1] + e, bad), qm = upre<F>(u[1] - e, bad);
    rk4<F>(s, u[0], qp, P.dT, fp, bad);
    rk4<F>(s, u[0], qm, P.dT, fm, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(16 + 2 * r + 1) = (fp[r] - fm[r]) / (2 * e);
  }
#undef DOUT
}
template <bool F>
__device__ __forceinline__ void knot_derivs(const IlqrDev& P, const double* s, const double* u, double* out,
                                            size_t stride, int& bad) {
  knot_dyn_derivs<F>(P, s, u, out, stride, bad);
  knot_cost_derivs<F>(P, s, u, out, stride, bad);
}

// the cost derivatives of knot_derivs (GetMatrix.jl CalculateMatrix): lx 24, lu 28, lxx 30, luu 46, lux 50
template <bool F>
__device__ __forceinline__ void knot_cost_derivs(const IlqrDev& P, const double* s, const double* u, double* out,
                                                 size_t stride, int& bad) {
  const double e = P.eps;
#define DOUT(q) out[(size_t)(q) * stride]
  double sp[4], sm[4];
  SigCache C;
  C.a[0] = u[0] - 2 * e; C.a[1] = u[0] - e; C.a[2] = u[0]; C.a[3] = u[0] + e; C.a[4] = u[0] + 2 * e;
  C.d[0] = u[1] - 2 * e; C.d[1] = u[1] - e; C.d[2] = u[1]; C.d[3] = u[1] + e; C.d[4] = u[1] + 2 * e;
#pragma unroll
  for (int t = 0; t < 5; t++) {
    C.sa[t] = sig_a<F>(C.a[t], bad);
    C.sd[t] = sig_d<F>(C.d[t], bad);
  }
  const int V = P.variant;
  const double c12 = 1 / (12 * (e * e)), c4 = 1 / (4 * (e * e));
  const double c0 = cst(V, s, C, 2, 2);
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[i] = s[i] + e;
    sm[i] = s[i] - e;
    DOUT(24 + i) = (cst(V, sp, C, 2, 2) - cst(V, sm, C, 2, 2)) / (2 * e);
  }
  DOUT(28) = (cst(V, s, C, 3, 2) - cst(V, s, C, 1, 2)) / (2 * e);
  DOUT(29) = (cst(V, s, C, 2, 3) - cst(V, s, C, 2, 1)) / (2 * e);
  double t1[4], t2[4], t3[4], t4[4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int r = 0; r < 4; r++) { t1[r] = s[r]; t2[r] = s[r]; t3[r] = s[r]; t4[r] = s[r]; }
      if (i == j) {
        t1[i] = s[i] + 2 * e; t2[i] = s[i] + e; t3[i] = s[i] - e; t4[i] = s[i] - 2 * e;
        DOUT(30 + 4 * i + j) = c12 * (-cst(V, t1, C, 2, 2) + 16 * cst(V, t2, C, 2, 2) - 30 * c0 +
                                      16 * cst(V, t3, C, 2, 2) - cst(V, t4, C, 2, 2));
      } else {
        t1[i] = s[i] + e; t1[j] = s[j] + e;
        t2[i] = s[i] - e; t2[j] = s[j] - e;
        t3[i] = s[i] + e; t3[j] = s[j] - e;
        t4[i] = s[i] - e; t4[j] = s[j] + e;
        DOUT(30 + 4 * i + j) =
            c4 * (cst(V, t1, C, 2, 2) + cst(V, t2, C, 2, 2) - cst(V, t3, C, 2, 2) - cst(V, t4, C, 2, 2));
      }
    }
  // luu: index 0 = ax, 1 = δ
  DOUT(46) = c12 * (-cst(V, s, C, 4, 2) + 16 * cst(V, s, C, 3, 2) - 30 * c0 + 16 * cst(V, s, C, 1, 2) - cst(V, s, C, 0, 2));
  DOUT(49) = c12 * (-cst(V, s, C, 2, 4) + 16 * cst(V, s, C, 2, 3) - 30 * c0 + 16 * cst(V, s, C, 2, 1) - cst(V, s, C, 2, 0));
  // (i=0,j=1): v1 = (+e,+e), v2 = (-e,-e), v3 = (a+e, d-e), v4 = (a-e, d+e)
  DOUT(47) = c4 * (cst(V, s, C, 3, 3) + cst(V, s, C, 1, 1) - cst(V, s, C, 3, 1) - cst(V, s, C, 1, 3));
  // (i=1,j=0): v1 = (+e,+e), v2 = (-e,-e), v3 = (δ+e, a-e), v4 = (δ-e, a+e)
  DOUT(48) = c4 * (cst(V, s, C, 3, 3) + cst(V, s, C, 1, 1) - cst(V, s, C, 1, 3) - cst(V, s, C, 3, 1));
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
      sp[j] = s[j] + e;
      sm[j] = s[j] - e;
      const int ap = i == 0 ? 3 : 2, dp = i == 1 ? 3 : 2, am = i == 0 ? 1 : 2, dm = i == 1 ? 1 : 2;
      DOUT(50 + 4 * i + j) = c4 * (cst(V, sp, C, ap, dp) + cst(V, sm, C, am, dm) - cst(V, sm, C, ap, dp) -
                                   cst(V, sp, C, am, dm));
    }
#undef DOUT
}

// Derivative records D[j][q][b] (component-major, instance fastest): thread t = j*B + b, so
// both the stores here and the backward sweep's per-knot loads are coalesced.
// list (mp_ilqr_solve): the n active instances in compact order; record i (of instance list[i])
// then sits in column i.  Without a list, all B instances, column b.  n_dev: n read on the device
// (the grid is sized for nmax >= n by a host that has not waited for the count), else n = nmax.
__global__ __launch_bounds__(256) void ilqr_deriv_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                         const int* list, const int* n_dev, int nmax, double* D) {
  ilqr_mirror(P, n_dev);
  const int n = n_dev ? *n_dev : nmax;
  const long long Bn = (long long)n * (P.N - 1);
  if ((long long)blockIdx.x * blockDim.x >= Bn) return;  // block-uniform: past the live records
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= Bn) t = Bn - 1;  // tail lanes recompute the last knot (identical values): all lanes stay active
  const int j = (int)(t / n), i = (int)(t % n);
  const int b = list ? list[i] : i;
  const double* xs = X + ((size_t)b * P.N + j) * 4;
  const double* us = U + ((size_t)b * P.N + j) * 2;
  const double s[4] = {xs[0], xs[1], xs[2], xs[3]};
  const double u[2] = {us[0], us[1]};
  double* out = D + (size_t)j * ND * B + i;
  int bad = 0;
  knot_derivs<kFastDeriv>(P, s, u, out, (size_t)B, bad);
  if (kFastDeriv && kRedo && __any(bad)) {  // some lane left a straight-line core's range: redo the wave exactly
    int d = 0;
    knot_derivs<false>(P, s, u, out, (size_t)B, d);
  }
}

// knot_derivs split four ways for the latency-bound launches (few active instances): parts 0-2
// the dynamics Jacobian (state columns x, y, v / heading + the ax column / the δ column), part 3
// the cost derivatives -- the same operations on the same operands per output as knot_derivs (exact libm),
// so the same bits, on four lanes instead of one.
template <int PART>
__device__ __forceinline__ void knot_derivs_part(const IlqrDev& P, const double* s, const double* u, double* out,
                                                 size_t stride) {
  const double e = P.eps;
  int bad = 0;
#define DOUT(q) out[(size_t)(q) * stride]
  // the dynamics Jacobian over three waves (RK4 counts 3 / 4 / 2 + the two perturbed upre)
  auto state_col = [&](int i, const UPre& q0) {  // column i of A: state i ± eps
    double sp[4], sm[4], fp[4], fm[4];
#pragma unroll
    for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
    sp[i] = s[i] + e;
    sm[i] = s[i] - e;
    rk4<false>(sp, u[0], q0, P.dT, fp, bad);
    rk4<false>(sm, u[0], q0, P.dT, fm, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(4 * r + i) = (fp[r] - fm[r]) / (2 * e);
  };
  if (PART == 0) {  // x, y (one RK4, dyn_jac_xy) and speed columns
    const UPre q0 = upre<false>(u[1], bad);
    dyn_jac_xy<false>(s, u[0], q0, P.dT, e, out, stride, bad);
    state_col(2, q0);
  } else if (PART == 1) {  // heading column and the ax column of B
    const UPre q0 = upre<false>(u[1], bad);
    state_col(3, q0);
    double fp[4], fm[4];
    rk4<false>(s, u[0] + e, q0, P.dT, fp, bad);
    rk4<false>(s, u[0] - e, q0, P.dT, fm, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(16 + 2 * r + 0) = (fp[r] - fm[r]) / (2 * e);
  } else if (PART == 2) {  // the δ column of B
    double fp[4], fm[4];
    const UPre qp = upre<false>(u[1] + e, bad), qm = upre<false>(u[1] - e, bad);
    rk4<false>(s, u[0], qp, P.dT, fp, bad);
    rk4<false>(s, u[0], qm, P.dT, fm, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) DOUT(16 + 2 * r + 1) = (fp[r] - fm[r]) / (2 * e);
  } else {
    knot_cost_derivs<false>(P, s, u, out, stride, bad);
  }
#undef DOUT
}

// ilqr_deriv_kernel with four waves per 64 records (knot_derivs_part: wave w of a block evaluates
// part w of records 64·blockIdx.x + lane, a wave-uniform role), for launches whose active count
// leaves most of the chip idle.
__global__ __launch_bounds__(256) void ilqr_deriv4_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                          const int* list, const int* n_dev, int nmax, double* D) {
  ilqr_mirror(P, n_dev);
  const int n = n_dev ? *n_dev : nmax;
  const long long Bn = (long long)n * (P.N - 1);
  if ((long long)blockIdx.x * 64 >= Bn) return;  // block-uniform: past the live records
  long long t = (long long)blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (t >= Bn) t = Bn - 1;  // tail lanes recompute the last knot (identical values)
  const int j = (int)(t / n), i = (int)(t % n);
  const int b = list ? list[i] : i;
  const double* xs = X + ((size_t)b * P.N + j) * 4;
  const double* us = U + ((size_t)b * P.N + j) * 2;
  const double s[4] = {xs[0], xs[1], xs[2], xs[3]};
  const double u[2] = {us[0], us[1]};
  double* out = D + (size_t)j * ND * B + i;
  if (part == 0) knot_derivs_part<0>(P, s, u, out, (size_t)B);
  else if (part == 1) knot_derivs_part<1>(P, s, u, out, (size_t)B);
  else if (part == 2) knot_derivs_part<2>(P, s, u, out, (size_t)B);
  else knot_derivs_part<3>(P, s, u, out, (size_t)B);
}

// pinv of a 2x2: Julia's LinearAlgebra.pinv through LAPACK dgesdd's 2x2 path (mp_jlmath.h
// mpj_pinv2, the oracle's or_pinv2): no libm calls, a few square roots and divisions.  FT: the
// straight-line general path (mpj_pinv2_fast) with a wave-uniform exact fallback for the rare lanes
// (diagonal / triangular Quu, dbdsqr splits): the branchy routine's uniform branches cost a lone wave
// ~4,300 cycles per call vs ~2,000 straight-line (tools/ubench/pinvlat.hip).
template <bool FT>
__device__ __forceinline__ void pinv2(const double* M, double* Pm, int&) {
  if (FT) mpj_pinv2_bl(M, Pm);
  else mpj_pinv2(M, Pm);
}

// The products of ILQR.jl:56-66 and :76 are BLAS calls in Julia (lx, lu and hence Vx, Qx, Qu, k are
// n x 1 matrices, GetMatrix.jl:6-7, so every Riccati product is dgemm; Klist * (xtilde .- xn) is dgemv
// 'N'), and they round as OpenBLAS's FMA kernels do (oracle/or_blas.h, pinned against OpenBLAS 0.3.29):
//   dgemm, K = 2 or 4: the fma chain from k = 0, acc = a0*b0, acc = fma(a_k, b_k, acc)
//   dgemv 'N' 2x4:     fma(a0, x0, a1*x1) + fma(a2, x2, a3*x3)
__device__ __forceinline__ double bk2(double a0, double b0, double a1, double b1) {
  return __builtin_fma(a1, b1, a0 * b0);
}
__device__ __forceinline__ double bk4(double a0, double b0, double a1, double b1, double a2, double b2, double a3,
                                      double b3) {
  return __builtin_fma(a3, b3, __builtin_fma(a2, b2, __builtin_fma(a1, b1, a0 * b0)));
}
// row r of the knot's gain K ([4][2] column-major: K[r][c] = Kr[2c + r]) times dx
__device__ __forceinline__ double kdx(const double* Kr, int r, const double* dx) {
  return __builtin_fma(Kr[r], dx[0], Kr[2 + r] * dx[1]) + __builtin_fma(Kr[4 + r], dx[2], Kr[6 + r] * dx[3]);
}

// LDS barrier between the compute wave and the loader wave of a staged block: LDS traffic
// retired, no vmcnt wait (the compute wave's gain stores and the loader's in-flight record
// loads stay outstanding across it), and a compiler barrier for memory.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Broadcast lane k of each lane quad to the quad (DPP quad_perm [k,k,k,k], one VALU op per half).
template <int K>
__device__ __forceinline__ double qbcast(double v) {
  constexpr int ctl = K | (K << 2) | (K << 4) | (K << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), ctl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), ctl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void qgather(double v, double* out) {  // out[k] = lane k's v
  out[0] = qbcast<0>(v);
  out[1] = qbcast<1>(v);
  out[2] = qbcast<2>(v);
  out[3] = qbcast<3>(v);
}

// ILQR.jl:46-67 on a LANE QUAD per instance (lane q = 0..3), records from the LDS stage
// [2][ND][IPB].  Every product entry is computed by exactly the operations (and summation order)
// of backward_sweep / the oracle, only on the lane that owns it: lane q owns row q of T44, Qxx, Vxx
// and KQ, entry q of Qx and Vx, column q of T24, Qux and KK; the 2x2 Quu, the pinv, Qu, kk and qk
// are evaluated on all four lanes (the pinv is the chain every lane waits on anyway).  Quad
// broadcasts (DPP) assemble T24, KK, Vx and Vxx where a full copy is needed.  The lone wave issues
// ~40 % of the one-lane sweep's instructions per knot, leaving the pinv chain as the bound.
// The staged sweep's record source: knot t's records sit in LDS buffer t & 1, handed over by the
// loader wave at one s_barrier per knot.
struct QuadFetchStaged {
  const double* lds;
  __device__ __forceinline__ const double* at(int t, int IPB) const {
    lds_barrier();  // knot j's records staged by the loader wave before barrier t
    return lds + (size_t)(t & 1) * ND * IPB;
  }
  __device__ __forceinline__ void done(int) const {}
};

template <int IPB, class Fetch = QuadFetchStaged>
__device__ __forceinline__ void backward_sweep_quad(const IlqrDev& P, int b, bool live, const double* X,
                                                    double* kout, double* Kout, const Fetch& src, int inst, int q) {
  const int N = P.N;
  const double e = P.eps;
  const int V = P.variant;
  double Vx[4], Vxx[16];
  {  // CalculateMatrix(StatesList[:, end], [0 0], TerminalCost): lx, lxx (every lane, once per sweep)
    const double* xs = X + ((size_t)b * N + N - 1) * 4;
    const double s[4] = {xs[0], xs[1], xs[2], xs[3]};
    double sp[4], sm[4], t1[4], t2[4], t3[4], t4[4];
    const double c12 = 1 / (12 * (e * e)), c4 = 1 / (4 * (e * e));
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
      for (int r = 0; r < 4; r++) { sp[r] = s[r]; sm[r] = s[r]; }
      sp[i] = s[i] + e;
      sm[i] = s[i] - e;
      Vx[i] = (terminal(V, sp) - terminal(V, sm)) / (2 * e);
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
#pragma unroll
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
  for (int j = N - 2, t = 0; j >= 0; j--, t++) {
    const double* bf = src.at(t, IPB) + inst;
    // no run-time index into a register array (q is per lane): column q of A comes from LDS, column
    // q of Vxx from the selects below
    double A[16], Bm[8], Acol[4], Vcol[4];
#pragma unroll
    for (int r = 0; r < 16; r++) A[r] = bf[r * IPB];
#pragma unroll
    for (int k = 0; k < 4; k++) Acol[k] = bf[(4 * k + q) * IPB];
#pragma unroll
    for (int k = 0; k < 4; k++)
      Vcol[k] = q < 2 ? (q == 0 ? Vxx[4 * k + 0] : Vxx[4 * k + 1]) : (q == 2 ? Vxx[4 * k + 2] : Vxx[4 * k + 3]);
#pragma unroll
    for (int r = 0; r < 8; r++) Bm[r] = bf[(16 + r) * IPB];
    const double lxq = bf[(24 + q) * IPB];
    const double lu0 = bf[28 * IPB], lu1 = bf[29 * IPB];
    double lxxq[4], luu[4];
#pragma unroll
    for (int c = 0; c < 4; c++) lxxq[c] = bf[(30 + 4 * q + c) * IPB];
#pragma unroll
    for (int c = 0; c < 4; c++) luu[c] = bf[(46 + c) * IPB];
    const double lux0q = bf[(50 + q) * IPB], lux1q = bf[(54 + q) * IPB];
    // Qx[q] = lx[q] + fx' * Vx  (own entry)
    // every product is dgemm in Julia: bk4 / bk2 (the fma chain from k = 0)
    const double Qxq = lxq + bk4(Acol[0], Vx[0], Acol[1], Vx[1], Acol[2], Vx[2], Acol[3], Vx[3]);  // lx + fx' * Vx
    double Qu[2];  // every lane: lu + fu' * Vx
    Qu[0] = lu0 + bk4(Bm[0], Vx[0], Bm[2], Vx[1], Bm[4], Vx[2], Bm[6], Vx[3]);
    Qu[1] = lu1 + bk4(Bm[1], Vx[0], Bm[3], Vx[1], Bm[5], Vx[2], Bm[7], Vx[3]);
    // T24 column q = (fu' Vxx)[:, q], gathered to the full 2x4
    double T24[8];
    {
      const double c0 = bk4(Bm[0], Vcol[0], Bm[2], Vcol[1], Bm[4], Vcol[2], Bm[6], Vcol[3]);
      const double c1 = bk4(Bm[1], Vcol[0], Bm[3], Vcol[1], Bm[5], Vcol[2], Bm[7], Vcol[3]);
      qgather(c0, T24);
      qgather(c1, T24 + 4);
    }
    // T44 row q = (fx' Vxx)[q, :], Qxx row q = lxx[q, :] + T44[q, :] fx  (own)
    double T44q[4], Qxxq[4];
#pragma unroll
    for (int c = 0; c < 4; c++)
      T44q[c] = bk4(Acol[0], Vxx[c], Acol[1], Vxx[4 + c], Acol[2], Vxx[8 + c], Acol[3], Vxx[12 + c]);
#pragma unroll
    for (int c = 0; c < 4; c++)
      Qxxq[c] = lxxq[c] + bk4(T44q[0], A[c], T44q[1], A[4 + c], T44q[2], A[8 + c], T44q[3], A[12 + c]);
    // Quu (every lane), Qux column q (own)
    double Quu[4];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int c = 0; c < 2; c++)
        Quu[2 * i + c] = luu[2 * i + c] + bk4(T24[4 * i], Bm[c], T24[4 * i + 1], Bm[2 + c], T24[4 * i + 2], Bm[4 + c],
                                              T24[4 * i + 3], Bm[6 + c]);
    double Quxq[2];
    Quxq[0] = lux0q + bk4(T24[0], Acol[0], T24[1], Acol[1], T24[2], Acol[2], T24[3], Acol[3]);
    Quxq[1] = lux1q + bk4(T24[4], Acol[0], T24[5], Acol[1], T24[6], Acol[2], T24[7], Acol[3]);
    double Pm[4];
    int bad = 0;
    pinv2<true>(Quu, Pm, bad);
    double kk[2], KKq[2];
#pragma unroll
    for (int i = 0; i < 2; i++) kk[i] = bk2(-Pm[2 * i + 0], Qu[0], -Pm[2 * i + 1], Qu[1]);
#pragma unroll
    for (int i = 0; i < 2; i++) KKq[i] = bk2(-Pm[2 * i + 0], Quxq[0], -Pm[2 * i + 1], Quxq[1]);
    if (live) {
      if (q < 2) kout[((size_t)b * (N - 1) + j) * 2 + q] = q == 0 ? kk[0] : kk[1];
      double* Ko = Kout + ((size_t)b * (N - 1) + j) * 8 + 2 * q;  // Klist[:, :, j] column q = (KK[0][q], KK[1][q])
      Ko[0] = KKq[0];
      Ko[1] = KKq[1];
    }
    double qk[2];
#pragma unroll
    for (int i = 0; i < 2; i++) qk[i] = bk2(Quu[2 * i + 0], kk[0], Quu[2 * i + 1], kk[1]);  // Quu * k
    const double vxq = Qxq - bk2(KKq[0], qk[0], KKq[1], qk[1]);                                // K' * (Quu k)
    double KQ[2];  // (K' * Quu)[q, :]
#pragma unroll
    for (int c = 0; c < 2; c++) KQ[c] = bk2(KKq[0], Quu[0 * 2 + c], KKq[1], Quu[1 * 2 + c]);
    double KK0[4], KK1[4];
    qgather(KKq[0], KK0);
    qgather(KKq[1], KK1);
    double vxxq[4];
#pragma unroll
    for (int c = 0; c < 4; c++) vxxq[c] = Qxxq[c] - bk2(KQ[0], KK0[c], KQ[1], KK1[c]);
    qgather(vxq, Vx);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      double col[4];
      qgather(vxxq[c], col);
#pragma unroll
      for (int k = 0; k < 4; k++) Vxx[4 * k + c] = col[k];
    }
    src.done(t);
  }
}

#ifndef ILQR_LOADER_DEPTH
#define ILQR_LOADER_DEPTH 2
#endif
constexpr int kLoaderDepth = ILQR_LOADER_DEPTH;  // knots of records in flight in the loader wave

// The loader wave of a quad-sweep block: knot j's records of the block's IPB instances into LDS
// buffer t&1 ([ND][IPB]) before barrier t; lane l loads components l/IPB, l/IPB + 64/IPB, ... of
// instance column l % IPB (IPB consecutive columns per component: coalesced 8*IPB-byte rows).
template <int IPB>
__device__ __forceinline__ void record_loader_quad(const IlqrDev& P, int B, int col0, int ncol, const double* D,
                                                   double* lds, int lane) {
  constexpr int CPL = 64 / IPB;                      // components per pass
  constexpr int NP = (ND + CPL - 1) / CPL;           // passes
  const int N = P.N;
  const size_t ks = (size_t)ND * B;
  const int ci = lane % IPB, c0 = lane / IPB;
  const int col = col0 + (ci < ncol ? ci : ncol - 1);  // columns past the list end repeat the last one
  const double* Db = D + col;
  // kLoaderDepth knots in flight: the loads of knot j-PD are issued while knot j is handed over, so
  // the global-load latency overlaps PD compute steps.  Measured at configs[2]: depth 1 388 us per
  // sweep (the loads' latency, not the compute, set the pace), 2: 180 us, 3 / 4 / 6: 181 / 183 / 182 us.
  constexpr int PD = kLoaderDepth;
  double v[PD][NP];
#pragma unroll
  for (int d = 0; d < PD; d++)
#pragma unroll
    for (int pq = 0; pq < NP; pq++) {
      const int qq = c0 + pq * CPL;
      v[d][pq] = qq < ND && N - 2 - d >= 0 ? Db[(size_t)(N - 2 - d) * ks + (size_t)qq * B] : 0.0;
    }
  for (int j = N - 2, t = 0; j >= 0; j--, t++) {
    double* bf = lds + (size_t)(t & 1) * ND * IPB + ci;
#pragma unroll
    for (int pq = 0; pq < NP; pq++) {
      const int qq = c0 + pq * CPL;
      if (qq < ND) bf[qq * IPB] = v[0][pq];
    }
#pragma unroll
    for (int d = 0; d + 1 < PD; d++)
#pragma unroll
      for (int pq = 0; pq < NP; pq++) v[d][pq] = v[d + 1][pq];
    if (j - PD >= 0) {
#pragma unroll
      for (int pq = 0; pq < NP; pq++) {
        const int qq = c0 + pq * CPL;
        if (qq < ND) v[PD - 1][pq] = Db[(size_t)(j - PD) * ks + (size_t)qq * B];
      }
    }
    lds_barrier();
  }
}

// Riccati sweep, quad mapping (default): block = one compute wave (IPB = 16 instances x 4 lanes)
// + one loader wave; 4,096 instances -> 256 blocks, one per CU.
constexpr int kQuadIPB = 16;
__global__ __launch_bounds__(128) void ilqr_backward_quad_kernel(IlqrDev P, int B, const double* X, const double* D,
                                                                 const int* list, const int* n_dev, int nmax,
                                                                 double* kout, double* Kout) {
  extern __shared__ double recs[];  // [2][ND][kQuadIPB]
  const int tid = threadIdx.x;
  const int n = n_dev ? *n_dev : nmax;
  const int col0 = blockIdx.x * kQuadIPB;
  if (col0 >= n) return;  // block-uniform: the grid covers nmax >= n
  if (tid >= 64) {
    record_loader_quad<kQuadIPB>(P, B, col0, n - col0, D, recs, tid - 64);
    return;
  }
  const int inst = tid >> 2, q = tid & 3;
  const int i0 = col0 + inst;
  const bool live = i0 < n;
  const int i = live ? i0 : n - 1;  // dead quads recompute the last column and store nothing
  const int b = list ? list[i] : i;
  backward_sweep_quad<kQuadIPB>(P, b, live, X, kout, Kout, QuadFetchStaged{recs}, live ? inst : (n - 1 - col0), q);
}

// ---------------------------------------------------------------- fused derivatives + Riccati sweep
// ilqr_backward_quad_kernel's compute wave (16 instances on lane quads) with the derivative records
// computed in the same block instead of read from HBM: kFusedDW derivative waves evaluate
// LocallyLinearizeDynamics / CalculateMatrix (GetMatrix.jl:3-91) of the block's instances for the knots
// in sweep order (N-2 first) and write them into an LDS ring that the sweep consumes.  A derivative
// wave takes one part of knot_derivs_part (a wave-uniform role, as ilqr_deriv4_kernel) for a group of
// kFusedGK knots x 16 instances (64 lanes); two waves per part alternate groups.  Per ring slot a
// cumulative count of parts written (kFusedParts per group) and one count of groups the sweep has finished are the
// only synchronisation (LDS, polled with s_sleep; every wave of the block is resident).  The records are
// the same operations on the same operands as the two-kernel path, so the gains are the same bits; the
// 464 B per knot record round trip through HBM and the separate derivative launch are gone, and the
// derivative work runs on the SIMDs the sweep leaves idle (one compute wave per CU).
#ifndef ILQR_FUSED_DW
#define ILQR_FUSED_DW 7
#endif
// derivative waves per block: at most 7, so no SIMD holds more than two of the block's waves and the
// sweep keeps the ~230 VGPRs it needs (9 waves cap every wave at 168: the sweep spilled 240 B per lane).
// One wave per part (4) could not keep up with the sweep: 0.292 ms per backward pass vs 0.264 ms for
// the two-kernel path (profiles/r04_ilqr_fused_ab.txt).
constexpr int kFusedDW = ILQR_FUSED_DW;
#ifndef ILQR_FUSED_PARTS
#define ILQR_FUSED_PARTS 2
#endif
// wave-uniform parts per record: 2 = the Jacobians (9 RK4 sharing stage sincos) / the cost
// derivatives; 4 = knot_derivs_part (three Jacobian parts without the sharing + the costs)
constexpr int kFusedParts = ILQR_FUSED_PARTS;
static_assert(kFusedParts == 2 || kFusedParts == 4, "2 or 4 parts");
static_assert(kFusedDW >= 1 && kFusedDW <= 7, "at most two waves per SIMD");
constexpr int kFusedGK = 4;  // knots per group: 4 knots x 16 instances = 64 lanes
#ifndef ILQR_FUSED_RG
#define ILQR_FUSED_RG 4
#endif
constexpr int kFusedRG = ILQR_FUSED_RG;  // ring slots (groups); LDS = RG x GK x ND x 16 x 8 B
constexpr size_t kFusedLds = sizeof(double) * kFusedRG * kFusedGK * ND * kQuadIPB;

__device__ __forceinline__ int lds_ld(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct QuadFetchRing {
  const double* ring;
  const int* ready;  // [RG] cumulative parts written into the slot
  int* consumed;     // groups the sweep has finished with
  int NK;
  __device__ __forceinline__ const double* at(int t, int IPB) const {
    const int g = t / kFusedGK, kk = t - g * kFusedGK, slot = g % kFusedRG;
    if (kk == 0) {  // wave-uniform: the group's four parts written
      const int want = kFusedParts * (g / kFusedRG + 1);
      while (lds_ld(ready + slot) < want) __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    return ring + ((size_t)slot * kFusedGK + kk) * ND * IPB;
  }
  __device__ __forceinline__ void done(int t) const {
    const int g = t / kFusedGK, kk = t - g * kFusedGK;
    if (kk == kFusedGK - 1 || t == NK - 1) {  // the group's records read (LDS reads retired) -> slot free
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if ((threadIdx.x & 63) == 0)
        __hip_atomic_store(consumed, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
};

__global__ __launch_bounds__(64 * (1 + kFusedDW)) void ilqr_backward_fused_kernel(
    IlqrDev P, int B, const double* X, const double* U, const int* list, const int* n_dev, int nmax, double* kout,
    double* Kout) {
  ilqr_mirror(P, n_dev);
  extern __shared__ double ring[];  // [RG][GK][ND][IPB]
  __shared__ int ready[kFusedRG];
  __shared__ int consumed;
  const int tid = threadIdx.x;
  const int n = n_dev ? *n_dev : nmax;
  const int col0 = blockIdx.x * kQuadIPB;
  if (col0 >= n) return;  // block-uniform: the grid covers nmax >= n
  if (tid < kFusedRG) ready[tid] = 0;
  if (tid == 0) consumed = 0;
  __syncthreads();  // the last block-wide barrier: the roles below synchronise through LDS counts only
  const int N = P.N, NK = N - 1, NG = (NK + kFusedGK - 1) / kFusedGK;
  if (tid >= 64) {
    // derivative wave w: tasks w, w + DW, w + 2 DW, ... of the sequence (group g, part p) = (t / 4, t % 4),
    // in order.  No deadlock: the sweep waits for the least unfinished group g0, every task of a group
    // <= g0 + RG - 1 runs without waiting for a slot, and a wave reaches its task of g0 after finishing
    // only tasks of earlier groups.  (A first version fetched tasks from a shared LDS counter -- one lane's
    // LDS atomic broadcast to the wave -- and hung; its cause was not isolated before the static order replaced
    // it, and the counter protocol itself is sound: tools/ubench/task_counter.hip runs it -- readfirstlane or
    // __shfl broadcast, with and without a divergent branch before the fetch, 7 producer waves feeding a
    // consumer wave through per-slot LDS counts as here -- 200 x 256 blocks x 200 tasks with every task run
    // exactly once, profiles/r05j_task_counter.txt, fetch ISA in profiles/r05j_task_counter_fetch_isa.txt.
    // So it was not a miscompile of the counter; the LDS-count hand-offs below are the ones that test runs.)
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6) - 1, lane = tid & 63;
    const int kk = lane / kQuadIPB, ci = lane % kQuadIPB;
    const int ncol = n - col0;
    const int col = col0 + (ci < ncol ? ci : ncol - 1);  // columns past the list end repeat the last one
    const int b = list ? list[col] : col;
    for (int task = w; task < kFusedParts * NG; task += kFusedDW) {
      const int g = task / kFusedParts, part = task - g * kFusedParts;
      const int slot = g % kFusedRG;
      if (g >= kFusedRG) {  // the slot's previous group consumed by the sweep
        while (lds_ld(&consumed) < g - kFusedRG + 1) __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
      const int jj = g * kFusedGK + kk;
      const int j = jj < NK ? NK - 1 - jj : 0;  // past the last knot: knot 0 again, written where no one reads
      const double* xs = X + ((size_t)b * N + j) * 4;
      const double* us = U + ((size_t)b * N + j) * 2;
      const double sv[4] = {xs[0], xs[1], xs[2], xs[3]};
      const double uv[2] = {us[0], us[1]};
      double* out = ring + ((size_t)slot * kFusedGK + kk) * ND * kQuadIPB + ci;
      if (kFusedParts == 2) {  // the Jacobians (shared stage sincos, knot_dyn_derivs) / the cost derivatives
        int bad = 0;
        if (part == 0) knot_dyn_derivs<false>(P, sv, uv, out, kQuadIPB, bad);
        else knot_cost_derivs<false>(P, sv, uv, out, kQuadIPB, bad);
      } else {
        if (part == 0) knot_derivs_part<0>(P, sv, uv, out, kQuadIPB);
        else if (part == 1) knot_derivs_part<1>(P, sv, uv, out, kQuadIPB);
        else if (part == 2) knot_derivs_part<2>(P, sv, uv, out, kQuadIPB);
        else knot_derivs_part<3>(P, sv, uv, out, kQuadIPB);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this wave's record writes retired
      if (lane == 0) __hip_atomic_fetch_add(ready + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return;
  }
  // the sweep: issue priority above the derivative waves sharing its SIMD (its chain sets the pace)
  __builtin_amdgcn_s_setprio(3);
  const int inst = tid >> 2, q = tid & 3;
  const int i0 = col0 + inst;
  const bool live = i0 < n;
  const int i = live ? i0 : n - 1;
  const int b = list ? list[i] : i;
  backward_sweep_quad<kQuadIPB>(P, b, live, X, kout, Kout, QuadFetchRing{ring, ready, &consumed, NK},
                                live ? inst : (n - 1 - col0), q);
}

// ILQR.jl:72-80: one closed-loop roll out at step size alpha; returns TotalCost.  (Staging the
// per-knot inputs through LDS as the Riccati sweep does measured no gain here, 371 vs 365 us: the
// one-knot-ahead prefetch already covers the loads under the knot's ~8k-cycle RK4 chain.)  The rolled
// state stays in registers (Xn is only written), the next knot's reference state, gains and
// nominal control are loaded one knot ahead, and TotalCost (Cost.jl:1-8) is accumulated in
// the loop in the reference's order (J = J + stage_i, then + terminal).
template <bool F, bool SC = F>
__device__ double forward_trial(const IlqrDev& P, const double* X, const double* U, const double* k,
                                const double* Kg, double alpha, double* Xn, double* Un, bool wr, int& bad) {
  const int N = P.N;
  double x[4] = {X[0], X[1], X[2], X[3]};
  if (wr)
#pragma unroll
    for (int r = 0; r < 4; r++) Xn[r] = x[r];
  double xr[4], Kr[8], kr[2], ur[2];
#pragma unroll
  for (int r = 0; r < 4; r++) xr[r] = X[r];
#pragma unroll
  for (int r = 0; r < 8; r++) Kr[r] = Kg[r];
  kr[0] = k[0]; kr[1] = k[1];
  ur[0] = U[0]; ur[1] = U[1];
  double J = 0.0;
  for (int i = 0; i < N - 1; i++) {
    const int in = i + 2 < N ? i + 1 : i;  // prefetch knot i+1 (clamped)
    double nxr[4], nK[8], nk[2], nu[2];
#pragma unroll
    for (int r = 0; r < 4; r++) nxr[r] = X[4 * in + r];
#pragma unroll
    for (int r = 0; r < 8; r++) nK[r] = Kg[8 * in + r];
    nk[0] = k[2 * in]; nk[1] = k[2 * in + 1];
    nu[0] = U[2 * in]; nu[1] = U[2 * in + 1];
    double dx[4], u[2];
#pragma unroll
    for (int r = 0; r < 4; r++) dx[r] = x[r] - xr[r];
#pragma unroll
    for (int r = 0; r < 2; r++) u[r] = (ur[r] + alpha * kr[r]) + kdx(Kr, r, dx);  // Klist * (xtilde .- xn): dgemv
    if (wr) {
      Un[2 * i] = u[0];
      Un[2 * i + 1] = u[1];
    }
    J = J + stage<F>(P.variant, x, u, bad);
    const UPre q = upre<F>(u[1], bad);
    double xn[4];
    rk4_ilp<SC>(x, u[0], q, P.dT, xn, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      x[r] = xn[r];
      if (wr) Xn[4 * (i + 1) + r] = xn[r];
      xr[r] = nxr[r];
    }
#pragma unroll
    for (int r = 0; r < 8; r++) Kr[r] = nK[r];
    kr[0] = nk[0]; kr[1] = nk[1];
    ur[0] = nu[0]; ur[1] = nu[1];
  }
  if (wr) {
    Un[2 * (N - 1)] = 0.0;
    Un[2 * (N - 1) + 1] = 0.0;
  }
  return J + terminal(P.variant, x);
}

#ifndef ILQR_FWD_NOSTORE
#define ILQR_FWD_NOSTORE 0  // timing probe only: the forward kernel's trajectory stores off
#endif
// Broadcast lane j of each quad to the quad (DPP quad_perm [j,j,j,j]).
template <int J>
__device__ __forceinline__ double quad_bcast(double v) {
  constexpr int c = J * 85;
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), c, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), c, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// The forward trial (ILQR.jl:72-80) on a QUAD of lanes per instance (sub = lane & 3), exact
// FDLIBM.  The knot's independent transcendentals are spread over the quad as one instruction
// stream with lane-selected operands: the four sigmoid exponentials of StageCost (ax: c1, c2;
// δ: c1, c2; Cost.jl:42-49) and the four RK4 stage sincos (the stage headings never depend on a
// sine or cosine, see rk4_ilp); each lane computes one of each, four DPP broadcasts share them.
// tan/atan/sincos(β) of the control run on all four lanes.  Same operations on the same
// operands as forward_trial: bit-identical.
__device__ double forward_trial_quad(const IlqrDev& P, const double* X, const double* U, const double* k,
                                     const double* Kg, double alpha, double* Xn, double* Un, bool wr, int sub) {
  const int N = P.N;
  const double la = 1.56, lb = 1.64, dT = P.dT;
  int bad = 0;
  double x[4] = {X[0], X[1], X[2], X[3]};
  // the trajectory is written a knot group at a time: every lane holds the whole state, lane sub
  // keeps knot j of X and knot i of U with j, i = sub (mod 4), and after each 4th knot the quad
  // writes the group's 128 B of X / 64 B of U as 16 B stores (one 8 B store per lane per knot put
  // 20-25 % on the kernel at 1-4 waves/SIMD, profiles/r03fs_ilqr_fwd_store.log)
  double sx[4] = {x[0], x[1], x[2], x[3]}, su[2] = {0.0, 0.0};
  double J = 0.0;
  // knot i's inputs were loaded during knot i-1 (the loads are off the x chain; loading them at the
  // top of the knot put an L2 round trip on it)
  double xr[4], Kr[8], kr[2], ur[2];
#pragma unroll
  for (int r = 0; r < 4; r++) xr[r] = X[r];
#pragma unroll
  for (int r = 0; r < 8; r++) Kr[r] = Kg[r];
  kr[0] = k[0]; kr[1] = k[1];
  ur[0] = U[0]; ur[1] = U[1];
  for (int i = 0; i < N - 1; i++) {
    const int in = i + 2 < N ? i + 1 : i;  // knot i+1 (clamped)
    double nxr[4], nK[8], nk[2], nu[2];
#pragma unroll
    for (int r = 0; r < 4; r++) nxr[r] = X[4 * in + r];
#pragma unroll
    for (int r = 0; r < 8; r++) nK[r] = Kg[8 * in + r];
    nk[0] = k[2 * in]; nk[1] = k[2 * in + 1];
    nu[0] = U[2 * in]; nu[1] = U[2 * in + 1];
    double dx[4], u[2];
#pragma unroll
    for (int r = 0; r < 4; r++) dx[r] = x[r] - xr[r];
#pragma unroll
    for (int r = 0; r < 2; r++) u[r] = (ur[r] + alpha * kr[r]) + kdx(Kr, r, dx);  // Klist * (xtilde .- xn): dgemv
    if ((i & 3) == sub) {
      su[0] = u[0];
      su[1] = u[1];
    }
    if (wr && (i & 3) == 3)
      *reinterpret_cast<double2*>(Un + 2 * (i - 3 + sub)) = make_double2(su[0], su[1]);
    // StageCost: sigmoid_boundary(ax; -2, 2) on subs 0/1, sigmoid_boundary(δ; -π/6, π/6) on 2/3
    {
      const double slope = 10, mag = 100;
      const double st = sub < 2 ? u[0] : u[1];
      const double mn = sub < 2 ? -2.0 : -MPJ_PI / 6, mx = sub < 2 ? 2.0 : MPJ_PI / 6;
      const double ci = (sub & 1) ? 1 / (1 + mpj_exp(slope * (st - mn))) : 1 / (1 + mpj_exp(-slope * (st - mx)));
      const double a1 = quad_bcast<0>(ci), a2 = quad_bcast<1>(ci), d1 = quad_bcast<2>(ci), d2 = quad_bcast<3>(ci);
      const double sa = mag * (a1 + a2), sd = mag * (d1 + d2);
      J = J + stage_pre(P.variant, x, u[0], u[1], sd, sa);
    }
    // RK4Integration with the stage sincos spread over the quad
    const UPre q = upre<false>(u[1], bad);
    const double ax = u[0];
    const double k1_3 = x[2] * q.cb * q.tdl / (la + lb);
    const double x2_2 = x[2] + dT / 2 * ax, x2_3 = x[3] + dT / 2 * k1_3;
    const double k2_3 = x2_2 * q.cb * q.tdl / (la + lb);
    const double x3_2 = x[2] + dT / 2 * ax, x3_3 = x[3] + dT / 2 * k2_3;
    const double k3_3 = x3_2 * q.cb * q.tdl / (la + lb);
    const double x4_2 = x[2] + dT * ax, x4_3 = x[3] + dT * k3_3;
    const double k4_3 = x4_2 * q.cb * q.tdl / (la + lb);
    const double hd = sub == 0 ? x[3] : sub == 1 ? x2_3 : sub == 2 ? x3_3 : x4_3;
    double sn, cs;
    mpj_sincos(hd + q.beta, &sn, &cs);
    const double s1 = quad_bcast<0>(sn), c1 = quad_bcast<0>(cs), s2 = quad_bcast<1>(sn), c2 = quad_bcast<1>(cs);
    const double s3 = quad_bcast<2>(sn), c3 = quad_bcast<2>(cs), s4 = quad_bcast<3>(sn), c4 = quad_bcast<3>(cs);
    const double k1[4] = {x[2] * c1, x[2] * s1, ax, k1_3};
    const double k2[4] = {x2_2 * c2, x2_2 * s2, ax, k2_3};
    const double k3[4] = {x3_2 * c3, x3_2 * s3, ax, k3_3};
    const double k4[4] = {x4_2 * c4, x4_2 * s4, ax, k4_3};
    double xn[4];
#pragma unroll
    for (int r = 0; r < 4; r++) xn[r] = 1.0 / 6 * (k1[r] + 2 * k2[r] + 2 * k3[r] + k4[r]) * dT + x[r];
#pragma unroll
    for (int r = 0; r < 4; r++) x[r] = xn[r];
    if (((i + 1) & 3) == sub) {
#pragma unroll
      for (int r = 0; r < 4; r++) sx[r] = xn[r];
    }
    if (wr && ((i + 1) & 3) == 3) {
      double2* d = reinterpret_cast<double2*>(Xn + 4 * (i - 2 + sub));
      d[0] = make_double2(sx[0], sx[1]);
      d[1] = make_double2(sx[2], sx[3]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) xr[r] = nxr[r];
#pragma unroll
    for (int r = 0; r < 8; r++) Kr[r] = nK[r];
    kr[0] = nk[0]; kr[1] = nk[1];
    ur[0] = nu[0]; ur[1] = nu[1];
  }
  // the last group (partial, or U's knot N-1 alone): U's knot N-1 is zero (ILQR.jl never
  // writes U[:, end]); X's group went out in the loop when N-1 = 3 (mod 4)
  const int gl = (N - 1) & 3, g0 = N - 1 - gl;
  if (gl == sub) su[0] = su[1] = 0.0;
  if (wr && sub <= gl) {
    *reinterpret_cast<double2*>(Un + 2 * (g0 + sub)) = make_double2(su[0], su[1]);
    if (gl != 3) {
      double2* d = reinterpret_cast<double2*>(Xn + 4 * (g0 + sub));
      d[0] = make_double2(sx[0], sx[1]);
      d[1] = make_double2(sx[2], sx[3]);
    }
  }
  return J + terminal(P.variant, x);
}

// Broadcast lane J (0 / 1) of each lane pair to the pair (DPP quad_perm [J, J, J+2, J+2]).
template <int J>
__device__ __forceinline__ double pair_bcast(double v) {
  constexpr int c = J | (J << 2) | ((J + 2) << 4) | ((J + 2) << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), c, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), c, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// forward_trial_quad on a lane PAIR (sub = lane & 1): lane 0 evaluates StageCost's two ax sigmoid
// exponentials and the RK4 stage-1 / stage-3 sincos, lane 1 the two δ exponentials and stages 2 / 4;
// pair broadcasts share them.  Half the lanes of the quad trial per trial, two independent libm
// calls per lane instead of one: fewer instructions per trial where the search is throughput-bound
// (round 0 at full activity).  Same operations on the same operands: bit-identical.
// The trajectory goes out in 4-knot groups: knot j of a group is held by lane (j & 3) >> 1, slot
// j & 1, and each lane writes its two consecutive knots (64 B of X, 32 B of U).
#ifndef ILQR_PAIR_PRIO
#define ILQR_PAIR_PRIO 0  // (A/B) quarter priority levels in the pair trial
#endif
__device__ double forward_trial_pair(const IlqrDev& P, const double* X, const double* U, const double* k,
                                     const double* Kg, double alpha, double* Xn, double* Un, bool wr, int sub) {
  const int N = P.N;
  const double la = 1.56, lb = 1.64, dT = P.dT;
  int bad = 0;
  double x[4] = {X[0], X[1], X[2], X[3]};
  double sx[2][4], su[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
#pragma unroll
  for (int r = 0; r < 4; r++) sx[0][r] = sx[1][r] = x[r];
  double J = 0.0;
  double xr[4], Kr[8], kr[2], ur[2];
#pragma unroll
  for (int r = 0; r < 4; r++) xr[r] = X[r];
#pragma unroll
  for (int r = 0; r < 8; r++) Kr[r] = Kg[r];
  kr[0] = k[0]; kr[1] = k[1];
  ur[0] = U[0]; ur[1] = U[1];
#if ILQR_PAIR_PRIO
  // (A/B) self-balancing issue priority over the trial's knots (a wave drops one level per quarter)
  const int q1 = (N - 1) / 4, q2 = (N - 1) / 2, q3 = 3 * (N - 1) / 4;
  __builtin_amdgcn_s_setprio(3);
#endif
  for (int i = 0; i < N - 1; i++) {
#if ILQR_PAIR_PRIO
    if (i == q1) __builtin_amdgcn_s_setprio(2);
    else if (i == q2) __builtin_amdgcn_s_setprio(1);
    else if (i == q3) __builtin_amdgcn_s_setprio(0);
#endif
    const int in = i + 2 < N ? i + 1 : i;  // knot i+1 (clamped)
    double nxr[4], nK[8], nk[2], nu[2];
#pragma unroll
    for (int r = 0; r < 4; r++) nxr[r] = X[4 * in + r];
#pragma unroll
    for (int r = 0; r < 8; r++) nK[r] = Kg[8 * in + r];
    nk[0] = k[2 * in]; nk[1] = k[2 * in + 1];
    nu[0] = U[2 * in]; nu[1] = U[2 * in + 1];
    double dx[4], u[2];
#pragma unroll
    for (int r = 0; r < 4; r++) dx[r] = x[r] - xr[r];
#pragma unroll
    for (int r = 0; r < 2; r++) u[r] = (ur[r] + alpha * kr[r]) + kdx(Kr, r, dx);  // Klist * (xtilde .- xn): dgemv
    if (((i & 3) >> 1) == sub) {
      su[i & 1][0] = u[0];
      su[i & 1][1] = u[1];
    }
    if (wr && (i & 3) == 3) {
      double2* d = reinterpret_cast<double2*>(Un + 2 * (i - 3 + 2 * sub));
      d[0] = make_double2(su[0][0], su[0][1]);
      d[1] = make_double2(su[1][0], su[1][1]);
    }
    {  // StageCost: sigmoid_boundary(ax; -2, 2) on lane 0, sigmoid_boundary(δ; -π/6, π/6) on lane 1
      const double slope = 10, mag = 100;
      const double st = sub ? u[1] : u[0];
      const double mn = sub ? -MPJ_PI / 6 : -2.0, mx = sub ? MPJ_PI / 6 : 2.0;
      const double cA = 1 / (1 + mpj_exp(-slope * (st - mx)));
      const double cB = 1 / (1 + mpj_exp(slope * (st - mn)));
      const double a1 = pair_bcast<0>(cA), a2 = pair_bcast<0>(cB), d1 = pair_bcast<1>(cA), d2 = pair_bcast<1>(cB);
      const double sa = mag * (a1 + a2), sd = mag * (d1 + d2);
      J = J + stage_pre(P.variant, x, u[0], u[1], sd, sa);
    }
    const UPre q = upre<false>(u[1], bad);
    const double ax = u[0];
    const double k1_3 = x[2] * q.cb * q.tdl / (la + lb);
    const double x2_2 = x[2] + dT / 2 * ax, x2_3 = x[3] + dT / 2 * k1_3;
    const double k2_3 = x2_2 * q.cb * q.tdl / (la + lb);
    const double x3_2 = x[2] + dT / 2 * ax, x3_3 = x[3] + dT / 2 * k2_3;
    const double k3_3 = x3_2 * q.cb * q.tdl / (la + lb);
    const double x4_2 = x[2] + dT * ax, x4_3 = x[3] + dT * k3_3;
    const double k4_3 = x4_2 * q.cb * q.tdl / (la + lb);
    double snA, csA, snB, csB;
    mpj_sincos((sub ? x2_3 : x[3]) + q.beta, &snA, &csA);  // stage 1 / 2
    mpj_sincos((sub ? x4_3 : x3_3) + q.beta, &snB, &csB);  // stage 3 / 4
    const double s1 = pair_bcast<0>(snA), c1 = pair_bcast<0>(csA), s2 = pair_bcast<1>(snA), c2 = pair_bcast<1>(csA);
    const double s3 = pair_bcast<0>(snB), c3 = pair_bcast<0>(csB), s4 = pair_bcast<1>(snB), c4 = pair_bcast<1>(csB);
    const double k1[4] = {x[2] * c1, x[2] * s1, ax, k1_3};
    const double k2[4] = {x2_2 * c2, x2_2 * s2, ax, k2_3};
    const double k3[4] = {x3_2 * c3, x3_2 * s3, ax, k3_3};
    const double k4[4] = {x4_2 * c4, x4_2 * s4, ax, k4_3};
    double xn[4];
#pragma unroll
    for (int r = 0; r < 4; r++) xn[r] = 1.0 / 6 * (k1[r] + 2 * k2[r] + 2 * k3[r] + k4[r]) * dT + x[r];
#pragma unroll
    for (int r = 0; r < 4; r++) x[r] = xn[r];
    if ((((i + 1) & 3) >> 1) == sub) {
#pragma unroll
      for (int r = 0; r < 4; r++) sx[(i + 1) & 1][r] = xn[r];
    }
    if (wr && ((i + 1) & 3) == 3) {
      double2* d = reinterpret_cast<double2*>(Xn + 4 * (i - 2 + 2 * sub));
      d[0] = make_double2(sx[0][0], sx[0][1]);
      d[1] = make_double2(sx[0][2], sx[0][3]);
      d[2] = make_double2(sx[1][0], sx[1][1]);
      d[3] = make_double2(sx[1][2], sx[1][3]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) xr[r] = nxr[r];
#pragma unroll
    for (int r = 0; r < 8; r++) Kr[r] = nK[r];
    kr[0] = nk[0]; kr[1] = nk[1];
    ur[0] = nu[0]; ur[1] = nu[1];
  }
  // the last group (partial, or U's knot N-1 alone): U's knot N-1 is zero; X's group went out in
  // the loop when N-1 = 3 (mod 4)
  const int gl = (N - 1) & 3, g0 = N - 1 - gl;
  if ((gl >> 1) == sub) su[gl & 1][0] = su[gl & 1][1] = 0.0;
  if (wr && 2 * sub <= gl) {
    const int kn = g0 + 2 * sub;
    const bool two = 2 * sub + 1 <= gl;
    double2* du = reinterpret_cast<double2*>(Un + 2 * kn);
    du[0] = make_double2(su[0][0], su[0][1]);
    if (two) du[1] = make_double2(su[1][0], su[1][1]);
    if (gl != 3) {
      double2* d = reinterpret_cast<double2*>(Xn + 4 * kn);
      d[0] = make_double2(sx[0][0], sx[0][1]);
      d[1] = make_double2(sx[0][2], sx[0][3]);
      if (two) {
        d[2] = make_double2(sx[1][0], sx[1][1]);
        d[3] = make_double2(sx[1][2], sx[1][3]);
      }
    }
  }
  return J + terminal(P.variant, x);
}

__global__ __launch_bounds__(64) void ilqr_forward_quad_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                               const double* k, const double* Kg, const double* alpha,
                                                               double* Xn, double* Un, double* Jn) {
  const int b0 = blockIdx.x * 16 + (threadIdx.x >> 2), sub = threadIdx.x & 3;
  const bool live = b0 < B;
  const size_t b = live ? b0 : B - 1;  // all lanes active (DPP quads); tail quads store nothing
  const size_t N = P.N;
  const double J = forward_trial_quad(P, X + b * N * 4, U + b * N * 2, k + b * (N - 1) * 2, Kg + b * (N - 1) * 8,
                                      alpha[b], Xn + b * N * 4, Un + b * N * 2, live && !ILQR_FWD_NOSTORE, sub);
  if (live && sub == 0) Jn[b] = J;
}

__global__ __launch_bounds__(64) void ilqr_forward_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                          const double* k, const double* Kg, const double* alpha,
                                                          double* Xn, double* Un, double* Jn) {
  const int b0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = b0 < B;
  const size_t b = live ? b0 : B - 1;  // all lanes active (ballot-based libm); tail lanes store nothing
  const size_t N = P.N;
  int bad = 0;
  double J = forward_trial<kFastFwd, kFastSC>(P, X + b * N * 4, U + b * N * 2, k + b * (N - 1) * 2,
                                             Kg + b * (N - 1) * 8, alpha[b], Xn + b * N * 4, Un + b * N * 2, live, bad);
  if ((kFastFwd || kFastSC) && kRedo && __any(bad)) {  // redo the wave's trials with the exact libm
    int d = 0;
    J = forward_trial<false>(P, X + b * N * 4, U + b * N * 2, k + b * (N - 1) * 2, Kg + b * (N - 1) * 8, alpha[b],
                             Xn + b * N * 4, Un + b * N * 2, live, d);
  }
  if (live) Jn[b] = J;
}

// The trial fixpoint m*: the least m in [0, ls_cap] with (U_e + 2^-m k_e) == U_e bit for bit for
// every control entry e of the instance (ls_cap + 1 if there is none).  A trial's control at knot i
// is u = (U_i + α k_i) + K_i (x - X_i), and only the first sum depends on α = 2^-m: for m ≥ m*,
// fl(2^-m k) shrinks towards zero with the sign of k (fl is monotone), so U ≤ U + fl(2^-m k) ≤
// U + fl(2^-m* k) (or ≥ ≥) and its rounding is sandwiched to U_e (signed zeros: equality at m* needs
// fl(2^-m* k) = ±0 with the sign that keeps U, and every later term is the same zero).  Every trial
// m ≥ m* therefore evaluates the same controls from the same x_0, i.e. is bit-identical to trial m*:
// if trial m* does not decrease J, neither does any later one, and the reference's halving loop runs
// on to its break at ls_cap (floor or max_ls) and accepts that trial -- trial m*'s outputs.  So the
// search never evaluates a trial beyond m*; trial m* stops it, reported as ls_cap unless it
// decreases J.  (Measured at configs[2]: m* = 51..75, against ls_cap = 199 for the
// OptimalControl variant, whose stalling instances ran all 200 trials.)
__device__ __forceinline__ bool fixed_at(double u, double kv, int m) {
  const double v = u + ldexp(1.0, -m) * kv;  // the trial's first sum, same operations
  return __double_as_longlong(v) == __double_as_longlong(u);
}

// m* over the instance's 2(N-1) control entries, on the GL lanes of a group (li = lane in group).
template <int GL>
__device__ int trial_fixpoint(const IlqrDev& P, const double* U, const double* k, int li) {
  const int ne = 2 * (P.N - 1), cap = P.ls_cap;
  int ms = 0;
  for (int e = li; e < ne; e += GL) {
    const double u = U[e], kv = k[e];
    if (fixed_at(u, kv, ms)) continue;  // the entry's own m* is <= the running max
    int lo = ms + 1, hi = cap + 1;      // least m in (ms, cap] with fixed_at, else cap + 1
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (fixed_at(u, kv, mid)) hi = mid;
      else lo = mid + 1;
    }
    ms = lo;
  }
#pragma unroll
  for (int o = 1; o < GL; o <<= 1) ms = max(ms, __shfl_xor(ms, o));
  return ms;
}

// ILQR.jl:70-88 after the backward sweep: line search, accept, convergence test, with the
// halving trials evaluated G at a time.  Trial m of the reference loop runs at alpha = 2^-m
// (repeated halving of 1.0 is exact), so the m-th trial is a pure function of m and the G lanes
// of an instance evaluate trials rG..rG+G-1 of round r concurrently, each into its own slot
// (Xs/Us [G][B][N]).  The accepted trial is the first m that would end the sequential loop:
// J_m < J (written !(J_m >= J), as the loop condition), or a break test (floor_stop, max_ls).
// Identical results to the sequential search; one round instead of G trials of latency.
// Jcur[b]: J at the start of this iteration (the previous J_new).
// The end of ILQR.jl's iteration for instance b once trial mw (cost Jn) is accepted: the
// max_ls flag, J, the iteration count and the convergence test.
__device__ __forceinline__ void search_accept(const IlqrDev& P, size_t b, double J, double Jn, int mw, double* Jcur,
                                              int* active, int* iters, int* flags, int* n_active) {
  if (mw + 1 >= P.max_ls && !floor_stop(P, mw)) atomicOr(flags + b, 1);
  Jcur[b] = Jn;
  const int it = iters[b] + 1;
  iters[b] = it;
  bool go = __builtin_fabs((Jn - J) / J) > P.tol;
  if (go && it > P.max_iter) {
    atomicOr(flags + b, 2);
    go = false;
  }
  active[b] = go;
  if (go) n_active[1 + atomicAdd(n_active, 1)] = (int)b;  // n_active[1..]: the next iteration's compact list
}

// one_round: stop after round 0 and mark the instances still searching in pending[] (their
// trials G..ls_cap then run all at once in ilqr_search_rest_kernel).
// L = lanes per trial: 1 (forward_trial on one lane) or 4 (forward_trial_quad: the trial's
// exponentials and stage sincos spread over a lane quad, ~2.5x shorter chain per trial).
// skip (pipelined search, may be nullptr): instances whose previous line search is still in its
// rest pass (they sit this iteration out); n_pend (may be nullptr) counts the instances marked pending.
template <int G, int L = 1>
__device__ __forceinline__ void search_round0(const IlqrDev& P, int B, double* X, double* U, const double* k,
                                              const double* Kg, double* Xs, double* Us, double* Jcur, int* active,
                                              int* iters, int* flags, int* n_active, int one_round, int* pending,
                                              int* mstar, const int* skip, int* n_pend, int bx) {
  constexpr int GL = G * L;     // lanes per instance
  constexpr int IPW = 64 / GL;  // instances per wave
  static_assert(GL <= 64 && 64 % GL == 0, "G*L must divide 64");
  const int lane = threadIdx.x, g = (lane % GL) / L, sub = lane % L, inst = lane / GL;
  const int b0 = bx * IPW + inst;
  const bool live = b0 < B && active[b0] && !(skip && skip[b0]);
  if (__all(!live)) return;
  const size_t b = b0 < B ? b0 : B - 1;
  const size_t N = P.N;
  double* Xb = X + b * N * 4;
  double* Ub = U + b * N * 2;
  double* Xg = Xs + ((size_t)g * B + b) * N * 4;
  double* Ug = Us + ((size_t)g * B + b) * N * 2;
  const double* kb = k + b * (N - 1) * 2;
  const double* Kb = Kg + b * (N - 1) * 8;
  const double J = Jcur[b];
  const int ms = trial_fixpoint<GL>(P, Ub, kb, lane % GL);  // no trial beyond m* (see trial_fixpoint)
  double Jn = J;
  int mw = -1;  // accepted trial index
  bool searching = live;
  // lanes that report a trial's outcome: every lane (L = 1) or the quad's first
  constexpr unsigned long long lead = L == 1 ? ~0ull : L == 2 ? 0x5555555555555555ull : 0x1111111111111111ull;
  for (int r = 0; __any(searching) && !(one_round && r > 0); r++) {
    const int m = r * G + g;
    const bool mine = searching && m <= P.ls_cap && m <= ms;  // uniform over a trial's lanes
    double jt = 0.0;
    if (mine) {
      if (L == 4) {
        jt = forward_trial_quad(P, Xb, Ub, kb, Kb, ldexp(1.0, -m), Xg, Ug, true, sub);
      } else if (L == 2) {
        jt = forward_trial_pair(P, Xb, Ub, kb, Kb, ldexp(1.0, -m), Xg, Ug, true, sub);
      } else {
        int d = 0;
        jt = forward_trial<false>(P, Xb, Ub, kb, Kb, ldexp(1.0, -m), Xg, Ug, true, d);
      }
    }
    const bool stop = mine && (!(jt >= J) || m == P.ls_cap || m == ms);
    const unsigned long long bal = __ballot(stop) & lead;
    const unsigned long long grp = (bal >> (inst * GL)) & (GL == 64 ? ~0ull : ((1ull << GL) - 1));
    const int gw = grp ? __builtin_ctzll(grp) / L : 0;
    const double jw = __shfl(jt, inst * GL + gw * L);  // every lane takes part in the exchange
    if (searching && grp) {
      Jn = jw;
      mw = r * G + gw;
      if (mw == ms && jw >= J) mw = P.ls_cap;  // trials m*..ls_cap are trial m*: the loop breaks at ls_cap
      searching = false;
      // the instance's lanes copy the winning slot together, 8 loads in flight per lane before
      // the stores (instead of the winner alone, one dependent load->store at a time): the
      // winner's slot stores are released at workgroup scope (the same wave) and L1 is
      // invalidated before the reads
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const double* Xw = Xs + ((size_t)gw * B + b) * N * 4;
      const double* Uw = Us + ((size_t)gw * B + b) * N * 2;
      const size_t nx = N * 4, nt = N * 6;
      const int li = lane % GL;
      for (size_t i0 = (size_t)li; i0 < nt; i0 += 8 * GL) {
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const size_t i = i0 + (size_t)e * GL;
          v[e] = i < nx ? Xw[i] : i < nt ? Uw[i - nx] : 0.0;
        }
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const size_t i = i0 + (size_t)e * GL;
          if (i < nx) Xb[i] = v[e];
          else if (i < nt) Ub[i - nx] = v[e];
        }
      }
    }
  }
  if (!live || (lane % GL) != 0) return;
  if (searching) {  // one_round only: trials G..ls_cap follow in ilqr_search_rest_kernel
    pending[b] = 1;
    mstar[b] = ms;
    if (n_pend) atomicAdd(n_pend, 1);
    return;
  }
  search_accept(P, b, J, Jn, mw, Jcur, active, iters, flags, n_active);
}
template <int G, int L = 1>
__global__ __launch_bounds__(64) void ilqr_search_kernel(IlqrDev P, int B, double* X, double* U, const double* k,
                                                         const double* Kg, double* Xs, double* Us, double* Jcur,
                                                         int* active, int* iters, int* flags, int* n_active,
                                                         int one_round, int* pending, int* mstar) {
  search_round0<G, L>(P, B, X, U, k, Kg, Xs, Us, Jcur, active, iters, flags, n_active, one_round, pending, mstar,
                      nullptr, nullptr, blockIdx.x);
}

// Trials first..min(m*, ls_cap) of the pending instances, all at once: block (b, w) runs trials
// m = first + (64/L)w + lane/L into slots [b][m-first] (Xs2/Us2/Jt, T2 per instance), one lane
// (L = 1) or a lane quad (L = 4) per trial, and the first stopping trial is the least m whose loop
// test would end the reference's halving loop (atomicMin).  first = G after the G-wide round 0
// (m* from it in mstar[]); first = 0 is the one-pass search of every active instance (pending =
// active), each block computing m* itself and block w = 0 publishing it.
template <int G, int L = 1>
__device__ __forceinline__ void search_rest(const IlqrDev& P, int B, const double* X, const double* U,
                                            const double* k, const double* Kg, const double* Jcur, const int* pending,
                                            int* mstar, double* Xs2, double* Us2, double* Jt, int* winm, int first,
                                            size_t T2, int b, int by) {
  const int sub = (int)threadIdx.x % L, m = first + (64 / L) * by + (int)threadIdx.x / L;
  if (!pending[b]) return;
  const size_t N = P.N, t = (size_t)(m - first);
  int ms;
  if (first == 0) {
    if (m - (int)threadIdx.x / L > P.ls_cap) return;  // the block's first trial (uniform)
    ms = trial_fixpoint<64>(P, U + b * N * 2, k + b * (N - 1) * 2, threadIdx.x);
    if (by == 0 && threadIdx.x == 0) mstar[b] = ms;
  } else {
    ms = mstar[b];
  }
  if (m > P.ls_cap || m > ms) return;  // uniform over a trial's lanes
  double jt;
  if (L == 4) {
    jt = forward_trial_quad(P, X + b * N * 4, U + b * N * 2, k + b * (N - 1) * 2, Kg + b * (N - 1) * 8,
                            ldexp(1.0, -m), Xs2 + ((size_t)b * T2 + t) * N * 4, Us2 + ((size_t)b * T2 + t) * N * 2,
                            true, sub);
  } else {
    int d = 0;
    jt = forward_trial<false>(P, X + b * N * 4, U + b * N * 2, k + b * (N - 1) * 2, Kg + b * (N - 1) * 8,
                              ldexp(1.0, -m), Xs2 + ((size_t)b * T2 + t) * N * 4, Us2 + ((size_t)b * T2 + t) * N * 2,
                              true, d);
  }
  if (sub != 0) return;
  Jt[(size_t)b * T2 + t] = jt;
  if (!(jt >= Jcur[b]) || m == P.ls_cap || m == ms) atomicMin(winm + b, m);
}
template <int G, int L = 1>
__global__ __launch_bounds__(64) void ilqr_search_rest_kernel(IlqrDev P, int B, const double* X, const double* U,
                                                              const double* k, const double* Kg, const double* Jcur,
                                                              const int* pending, int* mstar, double* Xs2,
                                                              double* Us2, double* Jt, int* winm, int first,
                                                              size_t T2) {
  search_rest<G, L>(P, B, X, U, k, Kg, Jcur, pending, mstar, Xs2, Us2, Jt, winm, first, T2, blockIdx.x, blockIdx.y);
}

// The pipelined two-pass search (mp_ilqr_solve): one launch runs round 0 of this iteration for the
// instances not in a rest pass (blocks [0, n0)) and the rest pass of the instances the previous
// iteration's round 0 left pending (blocks n0.., instance-major within each 16-trial column), so
// the rest pass's latency hides under round 0 instead of following it.  An instance's own sequence
// of operations is unchanged (its next backward pass simply comes one launch later).
// (A/B) ILQR_PIPE_WPE: waves per SIMD the pipelined search kernel is compiled for (0: the compiler's choice,
// 244 VGPRs = 2 waves per SIMD -- exactly the 2,048 round-0 waves of a full-activity launch, so the rest-pass
// waves of the same launch wait for round-0 waves to retire instead of running beside them)
#ifndef ILQR_PIPE_WPE
#define ILQR_PIPE_WPE 0
#endif
#if ILQR_PIPE_WPE
#define ILQR_PIPE_ATTR __attribute__((amdgpu_waves_per_eu(ILQR_PIPE_WPE)))
#else
#define ILQR_PIPE_ATTR
#endif
template <int G, int L, int L0 = L>
__global__ __launch_bounds__(64) ILQR_PIPE_ATTR void ilqr_search_pipe_kernel(IlqrDev P, int B, double* X, double* U, const double* k,
                                                              const double* Kg, double* Xs, double* Us, double* Jcur,
                                                              int* active, int* iters, int* flags, int* n_active,
                                                              int* pend_new, int* mstar_new, int* npend_new,
                                                              const int* pend_old, int* mstar_old, double* Xs2,
                                                              double* Us2, double* Jt, int* winm_old, size_t T2,
                                                              int n0) {
  const int bx = blockIdx.x;
  if (bx < n0) {
    search_round0<G, L0>(P, B, X, U, k, Kg, Xs, Us, Jcur, active, iters, flags, n_active, 1, pend_new, mstar_new,
                         pend_old, npend_new, bx);
  } else {
    const int r = bx - n0;
    search_rest<G, L>(P, B, X, U, k, Kg, Jcur, pend_old, mstar_old, Xs2, Us2, Jt, winm_old, G, T2, r % B, r / B);
  }
}

// Accept the winning trial of each pending instance: 64 lanes copy its slot into X/U.
// reset: after use, clear pending[b] (reset & 1; the pipelined pend arrays, not the active flags of
// the one-pass search) and set winm[b] back to 0x7f7f7f7f (reset & 2), so that the next launch that
// uses these arrays needs no memset.
template <int G>
__global__ __launch_bounds__(64) void ilqr_search_finish_kernel(IlqrDev P, int B, double* X, double* U,
                                                                int* pending, const int* mstar,
                                                                const double* Xs2, const double* Us2, const double* Jt,
                                                                int* winm, double* Jcur, int* active, int* iters,
                                                                int* flags, int* n_active, int first, size_t T2,
                                                                int reset = 0, int* zero_next = nullptr) {
  const size_t b = blockIdx.x;
  // the counts (pending, active) of the next iteration's list buffer, instead of a memset launch: that
  // buffer's list was read by this iteration's backward pass and its counts by the last host poll
  if (zero_next && b == 0 && threadIdx.x < 2) zero_next[threadIdx.x] = 0;
  if (pending[b]) {
    const size_t N = P.N;
    const int mw = winm[b];
    const size_t t = (size_t)(mw - first);
    const double* Xw = Xs2 + ((size_t)b * T2 + t) * N * 4;
    const double* Uw = Us2 + ((size_t)b * T2 + t) * N * 2;
    for (size_t i = threadIdx.x; i < N * 4; i += 64) X[b * N * 4 + i] = Xw[i];
    for (size_t i = threadIdx.x; i < N * 2; i += 64) U[b * N * 2 + i] = Uw[i];
    if (threadIdx.x == 0) {
      const double J = Jcur[b], Jn = Jt[(size_t)b * T2 + t];
      search_accept(P, b, J, Jn, mw == mstar[b] && Jn >= J ? P.ls_cap : mw, Jcur, active, iters, flags, n_active);
      if (reset & 1) pending[b] = 0;
      if (reset & 2) winm[b] = 0x7f7f7f7f;
    }
  }
}

// Initial guess roll out (ILQR.jl:31-37) with TotalCost accumulated in order.
template <bool F, bool SC = F>
__device__ __forceinline__ double rollout_one(const IlqrDev& P, const double* x0, const double* Ub, double* Xb,
                                              bool live, int& bad) {
  const size_t N = P.N;
  double x[4] = {x0[0], x0[1], x0[2], x0[3]};
  if (live)
#pragma unroll
    for (int r = 0; r < 4; r++) Xb[r] = x[r];
  double Jb = 0.0;
  for (size_t i = 0; i + 1 < N; i++) {
    const double u[2] = {Ub[2 * i], Ub[2 * i + 1]};
    Jb = Jb + stage<F>(P.variant, x, u, bad);
    const UPre q = upre<F>(u[1], bad);
    double xn[4];
    rk4_ilp<SC>(x, u[0], q, P.dT, xn, bad);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      x[r] = xn[r];
      if (live) Xb[4 * (i + 1) + r] = xn[r];
    }
  }
  return Jb + terminal(P.variant, x);
}

__global__ __launch_bounds__(64) void ilqr_rollout_kernel(IlqrDev P, int B, const double* x0, const double* U,
                                                          double* X, double* J) {
  const int b0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = b0 < B;
  const size_t b = live ? b0 : B - 1;  // all lanes active (ballot-based libm)
  const size_t N = P.N;
  int bad = 0;
  double Jb = rollout_one<kFastFwd, kFastSC>(P, x0 + 4 * b, U + b * N * 2, X + b * N * 4, live, bad);
  if ((kFastFwd || kFastSC) && kRedo && __any(bad)) {
    int d = 0;
    Jb = rollout_one<false>(P, x0 + 4 * b, U + b * N * 2, X + b * N * 4, live, d);
  }
  if (live) J[b] = Jb;
}

__global__ void ilqr_init_kernel(IlqrDev P, int B, const double* X, const double* U, double* Jcur, int* active,
                                 int* iters, int* flags, int* list) {
  const int b0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = b0 < B ? b0 : B - 1;  // all lanes active (ballot-based libm)
  const double J = total_cost(P.variant, P.N, X + (size_t)b * P.N * 4, U + (size_t)b * P.N * 2);
  if (b0 >= B) return;
  Jcur[b] = J;
  active[b] = 1;
  iters[b] = 1;
  flags[b] = 0;
  list[b] = b;
  if (b0 == 0) list[-1] = B;  // the count before the list
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
  D->ls_cap = D->max_ls - 1;
  D->mirror = nullptr;
  D->mirror_seq = 0;
  for (int m = 0; m < D->max_ls - 1; m++)
    if (floor_stop(*D, m)) {
      D->ls_cap = m;
      break;
    }
  return MP_OK;
}

// list/n_dev/na: the compact list of the *n_dev <= na active instances (mp_ilqr_solve; grids sized
// for na), or nullptr/nullptr/B for all.
int run_backward(mp_ctx* ctx, const IlqrDev& D, int B, const double* dX, const double* dU, const int* list,
                 const int* n_dev, int na, double* dk, double* dK) {
  const size_t n = (size_t)na * (D.N - 1);
  // derivatives + sweep in one launch (ilqr_backward_fused_kernel) while more than kDeriv4Max instances
  // are active.  A fused block makes the records of its 16 instances on its own CU, so with few blocks (the
  // solve's tail) the derivative work, spread over the whole chip by ilqr_deriv4_kernel, is confined to a
  // few CUs: measured 252 us per fused launch over a whole solve vs 32 + 180 us split, and 210 vs 108 +
  // 180 us at full activity (profiles/r04_ilqr_fused_ab.txt)
  if (na > kDeriv4Max) {
    if (!ctx->ilqr_fused_attr) {
      MP_HIP(ctx, hipSetDevice(ctx->device));
      MP_HIP(ctx, hipFuncSetAttribute((const void*)ilqr_backward_fused_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFusedLds));
      ctx->ilqr_fused_attr = true;
    }
    mp_time_begin(ctx);
    hipLaunchKernelGGL(ilqr_backward_fused_kernel, dim3((na + kQuadIPB - 1) / kQuadIPB), dim3(64 * (1 + kFusedDW)),
                       kFusedLds, ctx->stream, D, B, dX, dU, list, n_dev, na, dk, dK);
    MP_HIP(ctx, hipGetLastError());
    mp_time_end(ctx);
    return MP_OK;
  }
  double* dD = (double*)mp_ws(ctx, WS_ILQR0, sizeof(double) * (size_t)B * (D.N - 1) * ND);  // knot stride ND*B
  if (!dD) return MP_ERR_NOMEM;
  mp_time_begin(ctx);  // the timed region covers both kernels of the backward pass
  if (na <= kDeriv4Max)  // few active instances: four lanes per record (latency-bound launch)
    hipLaunchKernelGGL(ilqr_deriv4_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, ctx->stream, D, B, dX,
                       dU, list, n_dev, na, dD);
  else
    hipLaunchKernelGGL(ilqr_deriv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, D, B, dX, dU,
                       list, n_dev, na, dD);
  MP_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(ilqr_backward_quad_kernel, dim3((na + kQuadIPB - 1) / kQuadIPB), dim3(128),
                     sizeof(double) * 2 * ND * kQuadIPB, ctx->stream, D, B, dX, dD, list, n_dev, na, dk, dK);
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
  if ((st = run_backward(ctx, D, B, dX, dU, nullptr, nullptr, B, dk, dK))) return st;
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
  if (kFwdQuad)
    hipLaunchKernelGGL(ilqr_forward_quad_kernel, dim3((B + 15) / 16), dim3(64), 0, ctx->stream, D, B, dX, dU, dk, dK,
                       da, dXn, dUn, dJ);
  else
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
  return run_backward(ctx, D, B, X, U, nullptr, nullptr, B, k, Kg);
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
  if (kFwdQuad)
    hipLaunchKernelGGL(ilqr_forward_quad_kernel, dim3((B + 15) / 16), dim3(64), 0, ctx->stream, D, B, X, U, k, Kg,
                       alpha, Xnew, Unew, Jnew);
  else
    hipLaunchKernelGGL(ilqr_forward_kernel, dim3((B + 63) / 64), dim3(64), 0, ctx->stream, D, B, X, U, k, Kg, alpha,
                       Xnew, Unew, Jnew);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  return MP_OK;
}

// mp_ilqr_solve (dev = false: host X / U / J / iters, uploaded and downloaded here) and mp_ilqr_solve_dev (dev:
// the caller's device buffers, X / U solved in place)
static int ilqr_solve(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, double* X, double* U, double* J,
                      int32_t* iters, bool dev) {
  if (!ctx) return MP_ERR_INVALID;
  IlqrDev D;
  int st = make_ilqr(ctx, p, B, &D);
  if (st) return st;
  MP_CHECK(ctx, X && U && J && iters, "required pointer is NULL");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t N = D.N;
  double* dX = dev ? X : (double*)mp_upload(ctx, WS_IO0, X, 4 * N * B, &st);
  double* dU = dev ? U : (double*)mp_upload(ctx, WS_IO1, U, 2 * N * B, &st);
  double* dk = (double*)mp_ws(ctx, WS_IO2, sizeof(double) * 2 * (N - 1) * B);
  double* dK = (double*)mp_ws(ctx, WS_IO3, sizeof(double) * 8 * (N - 1) * B);
  // trial slots for the G-wide line search: G = kSearchG = 16 trials per instance on lane quads
  // (4096 waves at B = 4096) while the slots stay within 1 GiB of HBM (and the context's workspace
  // cap), else 4 single-lane trials, else 1 (the sequential loop)
  auto fits = [&](size_t g) {  // X slots 32 B, U slots 16 B per (trial, instance, knot)
    return g * B * N * 48 <= ((size_t)1 << 30) && (!ctx->ws_limit || g * B * N * 32 <= ctx->ws_limit);
  };
  const int G = fits(kSearchG) ? kSearchG : fits(4) ? 4 : 1;
  double* dXn = (double*)mp_ws(ctx, WS_IO4, sizeof(double) * 4 * N * B * G);
  double* dUn = (double*)mp_ws(ctx, WS_IO5, sizeof(double) * 2 * N * B * G);
  double* dJ = (double*)mp_ws(ctx, WS_IO6, sizeof(double) * B);
  int* dint = (int*)mp_ws(ctx, WS_IO7, sizeof(int) * (5 * (size_t)B + 4));
  if (st || !dk || !dK || !dXn || !dUn || !dJ || !dint) return st ? st : MP_ERR_NOMEM;
  int* dact = dint;
  int* dit = dint + B;
  int* dfl = dint + 2 * B;
  // two list buffers, [0] instances the pipelined round 0 left pending, [1] active count, [2 ..] their compact
  // list (search_accept): iteration q's backward pass reads par[(q + 1) & 1], its search writes par[q & 1],
  // whose counts the finish kernel of iteration q - 1 zeroed (a memset only after a path without one)
  int* par[2] = {dint + 3 * (size_t)B, dint + 3 * (size_t)B + (2 + (size_t)B)};
  int* dnp = par[0];
  int* dn = dnp + 1;
  // trials G..ls_cap in one pass for the instances still searching after round 0 (G = kSearchG only),
  // while their slots fit in 8 GiB, in half of the free device memory and in the context's
  // workspace cap.  Otherwise -- or when allocating them fails -- the G-wide kernel runs its
  // rounds to the end: the same accepted trials (tests/test_gpu_ilqr.py), more latency.
  // Slots for trials 0..ls_cap, so that the same buffers serve the one-pass search (below).
  const size_t T2 = G == kSearchG && D.ls_cap + 1 > G ? (size_t)(D.ls_cap + 1) : 0;
  bool rest = T2 > 0 && T2 * B * N * 48 <= ((size_t)8 << 30) &&
              mp_ws_affordable(ctx, WS_ILQR1, sizeof(double) * 4 * N * B * T2, 0.5) &&
              mp_ws_affordable(ctx, WS_ILQR2, sizeof(double) * 2 * N * B * T2, 0.25);
  double *dXs2 = nullptr, *dUs2 = nullptr, *dJt = nullptr;
  // pending[B], winm[B], mstar[B]; pipelined: pend[2][B], winm[2][B], mstar[2][B] at [0, 6B);
  // the one-pass search has its own winm[B], mstar[B] at [6B, 8B), so it never reads a slot the
  // pipelined launches left set
  int* dpw = nullptr;
  if (rest) {
    dXs2 = (double*)mp_ws(ctx, WS_ILQR1, sizeof(double) * 4 * N * B * T2);
    dUs2 = dXs2 ? (double*)mp_ws(ctx, WS_ILQR2, sizeof(double) * 2 * N * B * T2) : nullptr;
    dJt = dUs2 ? (double*)mp_ws(ctx, WS_IO12, sizeof(double) * B * T2) : nullptr;
    dpw = dJt ? (int*)mp_ws(ctx, WS_IO13, sizeof(int) * 8 * (size_t)B) : nullptr;
    if (!dXs2 || !dUs2 || !dJt || !dpw) {
      rest = false;      // fall back to the multi-round 16-wide search
      ctx->err.clear();  // (the failed allocation left a message; mp_ws already cleared the HIP error)
    }
  }
  const dim3 g1((B + 63) / 64), b1(64);
  MP_HIP(ctx, hipMemsetAsync(par[0], 0, 2 * sizeof(int), ctx->stream));
  MP_HIP(ctx, hipMemsetAsync(par[1], 0, 2 * sizeof(int), ctx->stream));
  hipLaunchKernelGGL(ilqr_init_kernel, g1, b1, 0, ctx->stream, D, B, dX, dU, dJ, dact, dit, dfl, par[1] + 2);
  MP_HIP(ctx, hipGetLastError());
  int* hn = (int*)mp_pinned(ctx, 4 * sizeof(int));
  if (!hn) return mp_fail(ctx, MP_ERR_NOMEM, "pinned allocation failed");
  // One-pass search: once at most kOnePassMax instances are active (the host's last poll), every
  // active instance's trials 0..min(m*, ls_cap) run in one launch (m* = 51..75 measured, so ~4
  // waves per instance) -- the round-0 latency chain and the rest chain become one.
  // The host runs one iteration ahead: after enqueueing iteration t it waits for the active count
  // after t-1 (copied into hn[(t-1)&1], event-ordered), which bounds iteration t+1's count, so the
  // GPU never idles between iterations while the host polls.  Launch grids are sized by that bound;
  // the derivative and sweep kernels read the exact count (dn[0]) on the device, the search kernels
  // skip inactive instances; once the count reads 0 the iteration just enqueued was a no-op.
  struct EvPair {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~EvPair() { for (hipEvent_t x : e) if (x) (void)hipEventDestroy(x); }
  } evp;
  for (int q = 0; q < 2; q++) MP_HIP(ctx, hipEventCreateWithFlags(&evp.e[q], hipEventDisableTiming));
  int n_act = B;  // upper bound on the active count of the iteration being enqueued
  // hn[2q] = instances left pending by the pipelined round 0 (their rest pass runs in the next
  // launch, then they rejoin the list), hn[2q + 1] = the list count: their sum bounds the next list
  // the counts come from host memory the next backward pass's first kernel writes (ilqr_mirror) instead of a
  // stream copy + event per iteration: 0.3-0.5 ms per 4096-instance solve (r05zd); the copy + event poll
  // remains for a context without mapped host memory
  unsigned long long* dmr = nullptr;
  volatile unsigned long long* hmr = mp_mapped(ctx, &dmr);
  if (hmr) hmr[0] = hmr[1] = 0;
  auto poll = [&](int outer, bool* stop) -> int {
    *stop = false;
    if (hmr) {  // the counts of iteration outer - 1's search, reported by this iteration's backward pass
      if (outer == 0) return MP_OK;
      const unsigned long long want = (unsigned long long)(unsigned)(outer - 1 + 1);  // seq = iteration + 1
      unsigned long long a = hmr[0], pd = hmr[1];  // (each word carries its seq: no order between them)
      long long spins = 0;
      while ((a >> 32) < want || (pd >> 32) < want) {
        if ((++spins & 1023) == 0) {
          const hipError_t q = hipStreamQuery(ctx->stream);
          if (q != hipErrorNotReady) {
            // the stream is idle (or failed): the kernel's stores are visible now, so one more read decides
            a = hmr[0];
            pd = hmr[1];
            if ((a >> 32) >= want && (pd >> 32) >= want) break;
            if (q != hipSuccess) return mp_fail(ctx, MP_ERR_HIP, "iLQR solve stream failed: %s", hipGetErrorString(q));
            return mp_fail(ctx, MP_ERR_HIP, "iLQR count mirror never arrived");
          }
        }
        a = hmr[0];
        pd = hmr[1];
      }
      const int nprev = (int)(a & 0xffffffffu) + (int)(pd & 0xffffffffu);
      if (nprev == 0) *stop = true;
      else n_act = nprev;
      return MP_OK;
    }
    MP_HIP(ctx, hipMemcpyAsync(hn + 2 * (outer & 1), dnp, 2 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipEventRecord(evp.e[outer & 1], ctx->stream));
    if (outer == 0) return MP_OK;
    MP_HIP(ctx, hipEventSynchronize(evp.e[(outer - 1) & 1]));
    const int nprev = hn[2 * ((outer - 1) & 1)] + hn[2 * ((outer - 1) & 1) + 1];
    if (nprev == 0) *stop = true;
    else n_act = nprev;
    return MP_OK;
  };
  // pipelined two-pass search (ilqr_search_pipe_kernel): launch q marks pend[q & 1] and runs the rest
  // pass of pend[(q - 1) & 1]; pend[1] starts empty
  const bool pipe = rest && kPipe;
  int q2 = 0;  // two-pass launches so far
  if (pipe) {  // pend[2][B] = 0, winm[2][B] = 0x7f7f7f7f; afterwards the finish kernels reset what they use
    MP_HIP(ctx, hipMemsetAsync(dpw, 0, sizeof(int) * 2 * B, ctx->stream));
    MP_HIP(ctx, hipMemsetAsync(dpw + 2 * B, 0x7f, sizeof(int) * 2 * B, ctx->stream));
  }
  bool onepass_armed = false;  // winm of the one-pass search set (then reset by its finish kernels)
  // (an instance in a rest pass sits one launch out, so the pipelined loop may take more launches
  // than max_iter + 2; each instance still stops at its own max_iter)
  bool w_zeroed = true;  // this iteration's list buffer's counts are zero (initially: the memsets above)
  for (int outer = 0; outer <= 2 * (D.max_iter + 2); outer++) {
    int* rd = par[(outer + 1) & 1];  // the list the previous iteration wrote (or the init kernel)
    dnp = par[outer & 1];
    dn = dnp + 1;
    int* zn = rd;  // zeroed by this iteration's finish kernel, for the next iteration
    // the derivative and sweep launches cover the active instances only (compact list)
    IlqrDev Dm = D;  // (the mirror: the previous iteration's counts, seq = outer; 0 = none yet)
    if (hmr && outer > 0) {
      Dm.mirror = dmr;
      Dm.mirror_seq = outer;
    }
    if ((st = run_backward(ctx, Dm, B, dX, dU, rd + 2, rd + 1, n_act, dk, dK))) return st;
    if (!w_zeroed) MP_HIP(ctx, hipMemsetAsync(dnp, 0, 2 * sizeof(int), ctx->stream));
    w_zeroed = false;
    mp_time_begin(ctx);
    // The switch to the one-pass search is terminal (once armed it stays, whatever later polls
    // say).  Instances the last pipelined launch left pending keep their active flag and their
    // gains (they sat the backward pass out), so the one-pass search reruns them from trial 0:
    // trials 0..15 give the bits round 0 gave, so they end exactly where their rest pass would.
    if (rest && (onepass_armed || n_act <= kOnePassMax)) {
      int *winm1 = dpw + 6 * (size_t)B, *ms1 = dpw + 7 * (size_t)B;
      if (!onepass_armed) MP_HIP(ctx, hipMemsetAsync(winm1, 0x7f, sizeof(int) * B, ctx->stream));
      onepass_armed = true;
      hipLaunchKernelGGL((ilqr_search_rest_kernel<kSearchG, kSearchL>),
                         dim3((unsigned)B, (unsigned)((T2 + 64 / kSearchL - 1) / (64 / kSearchL))), b1, 0, ctx->stream, D,
                         B, dX, dU, dk, dK, dJ, dact, ms1, dXs2, dUs2, dJt, winm1, 0, T2);
      MP_HIP(ctx, hipGetLastError());
      hipLaunchKernelGGL(ilqr_search_finish_kernel<kSearchG>, dim3((unsigned)B), b1, 0, ctx->stream, D, B, dX, dU, dact,
                         ms1, dXs2, dUs2, dJt, winm1, dJ, dact, dit, dfl, dn, 0, T2, 2, zn);
      MP_HIP(ctx, hipGetLastError());
      w_zeroed = zn != nullptr;
      mp_time_end(ctx);
      bool stop;
      if ((st = poll(outer, &stop))) return st;
      if (stop) break;
      continue;
    }
    // G = 16: a lane quad per trial (4 waves per SIMD at B = 4096); the narrower fallbacks one lane
    const int l0 = pipe && n_act >= kPairMin ? kRound0L : kSearchL;
    const int ipw = G == kSearchG ? 64 / (kSearchG * l0) : 64 / G;
    const dim3 gs((unsigned)((B + ipw - 1) / ipw));
    if (pipe) {
      const int cur = q2 & 1, old = cur ^ 1;
      q2++;
      int *pend_n = dpw + cur * B, *pend_o = dpw + old * B;
      int* winm_o = dpw + (2 + old) * B;  // pend_n is 0 and winm[cur] 0x7f7f7f7f: reset by the finish
      int *ms_n = dpw + (4 + cur) * B, *ms_o = dpw + (4 + old) * B;  // kernel that last used them
      const unsigned ncol = (unsigned)((T2 + 64 / kSearchL - 1) / (64 / kSearchL));
      auto pipe_k = l0 == kRound0L ? ilqr_search_pipe_kernel<kSearchG, kSearchL, kRound0L>
                                   : ilqr_search_pipe_kernel<kSearchG, kSearchL, kSearchL>;
      hipLaunchKernelGGL(pipe_k, dim3(gs.x + (unsigned)B * ncol), b1, 0,
                         ctx->stream, D, B, dX, dU, dk, dK, dXn, dUn, dJ, dact, dit, dfl, dn, pend_n, ms_n, dnp,
                         pend_o, ms_o, dXs2, dUs2, dJt, winm_o, T2, (int)gs.x);
      MP_HIP(ctx, hipGetLastError());
      hipLaunchKernelGGL(ilqr_search_finish_kernel<kSearchG>, dim3((unsigned)B), b1, 0, ctx->stream, D, B, dX, dU, pend_o,
                         ms_o, dXs2, dUs2, dJt, winm_o, dJ, dact, dit, dfl, dn, kSearchG, T2, 3, zn);
      MP_HIP(ctx, hipGetLastError());
      w_zeroed = zn != nullptr;
      mp_time_end(ctx);
      bool stop;
      if ((st = poll(outer, &stop))) return st;
      if (stop) break;
      continue;
    }
    if (rest) {
      MP_HIP(ctx, hipMemsetAsync(dpw, 0, sizeof(int) * B, ctx->stream));             // pending
      MP_HIP(ctx, hipMemsetAsync(dpw + B, 0x7f, sizeof(int) * B, ctx->stream));      // winm = 0x7f7f7f7f
    }
    if (G == kSearchG)
      hipLaunchKernelGGL((ilqr_search_kernel<kSearchG, kSearchL>), gs, b1, 0, ctx->stream, D, B, dX, dU, dk, dK, dXn, dUn, dJ, dact,
                         dit, dfl, dn, rest ? 1 : 0, dpw, dpw ? dpw + 2 * B : nullptr);
    else if (G == 4)
      hipLaunchKernelGGL(ilqr_search_kernel<4>, gs, b1, 0, ctx->stream, D, B, dX, dU, dk, dK, dXn, dUn, dJ, dact, dit, dfl, dn,
                         0, dpw, nullptr);
    else
      hipLaunchKernelGGL(ilqr_search_kernel<1>, gs, b1, 0, ctx->stream, D, B, dX, dU, dk, dK, dXn, dUn, dJ, dact, dit, dfl, dn,
                         0, dpw, nullptr);
    MP_HIP(ctx, hipGetLastError());
    if (rest) {
      hipLaunchKernelGGL((ilqr_search_rest_kernel<kSearchG, kSearchL>), dim3((unsigned)B, (unsigned)((T2 + 64 / kSearchL - 1) /
                         (64 / kSearchL))), b1, 0, ctx->stream, D, B, dX, dU, dk, dK, dJ, dpw, dpw + 2 * B, dXs2, dUs2, dJt, dpw + B, kSearchG,
                         T2);
      MP_HIP(ctx, hipGetLastError());
      hipLaunchKernelGGL(ilqr_search_finish_kernel<kSearchG>, dim3((unsigned)B), b1, 0, ctx->stream, D, B, dX, dU, dpw, dpw + 2 * B,
                         dXs2, dUs2, dJt, dpw + B, dJ, dact, dit, dfl, dn, kSearchG, T2, 0, zn);
      MP_HIP(ctx, hipGetLastError());
      w_zeroed = zn != nullptr;
    }
    mp_time_end(ctx);
    bool stop;
    if ((st = poll(outer, &stop))) return st;
    if (stop) break;
  }
  std::vector<int> hfl(B);
  if (dev) {  // X / U are already the caller's; J and the iteration counts device to device
    MP_HIP(ctx, hipMemcpyAsync(J, dJ, sizeof(double) * B, hipMemcpyDeviceToDevice, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(iters, dit, sizeof(int) * B, hipMemcpyDeviceToDevice, ctx->stream));
  } else {
    if ((st = mp_download(ctx, X, (const double*)dX, 4 * N * B))) return st;
    if ((st = mp_download(ctx, U, (const double*)dU, 2 * N * B))) return st;
    if ((st = mp_download(ctx, J, (const double*)dJ, (size_t)B))) return st;
    if ((st = mp_download(ctx, iters, (const int*)dit, (size_t)B))) return st;
  }
  if ((st = mp_download(ctx, hfl.data(), (const int*)dfl, (size_t)B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  int any = 0;
  for (int b = 0; b < B; b++) any |= hfl[b];
  if (any & 1) return mp_fail(ctx, MP_ERR_NUMERIC, "line search hit max_ls for some instance (the reference would loop forever)");
  if (any & 2) return mp_fail(ctx, MP_ERR_NUMERIC, "max_iter reached before |dJ/J| <= tol for some instance");
  return MP_OK;
}

int mp_ilqr_solve(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, double* X, double* U, double* J,
                  int32_t* iters) {
  return ilqr_solve(ctx, p, B, X, U, J, iters, false);
}

int mp_ilqr_solve_dev(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, double* X, double* U, double* J,
                      int32_t* iters) {
  return ilqr_solve(ctx, p, B, X, U, J, iters, true);
}

}  // extern "C"
