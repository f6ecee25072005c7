// mppi_device.hpp — device-side restatement of the MPPI rollout
// (OptimalControl/MPPI/src/MPPIUtils.jl:31-57, vehicledynamics.jl:1-54).
//
// Mapping (gfx950): one rollout = one LANE PAIR of a 64-wide wavefront.
// The two lanes of a pair evaluate the two tire models of VehicleDynamics in
// SIMD (front on the even lane, rear on the odd lane: the same instruction
// stream with lane-selected constants, bit-identical to the scalar formulas),
// exchange the lateral forces with one DPP/ds_swizzle shuffle, and carry the
// 7-state replicated in registers.  That halves the serial transcendental
// chain per step (4 instead of 8 dependent atan/sin per dynamics call) and
// doubles the waves in flight for a fixed K.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mp_jlmath.h"

namespace mpk {

struct MppiDev {
  int K, H, FC, n_obs;
  double dt, lambda, nil;  // nil = (-1)/λ as evaluated by the reference (MPPIUtils.jl:160)
  double L[4];             // chol(Σ).L row-major
  double Si[4];            // inv(Σ) row-major
  double XL[7], XU[7], CL[2], CU[2];
  double slack, obs_pen;
  int gnx, gny;
  double gx0, gy0, gdx, gdy;
  int noise_mode, ctrl_cost;
  unsigned long long seed, offset;
  int scene_base;
  int in_flight;  // (host side) mp_mppi_params.calls_in_flight, at least 1: the launch layout's choice
};

// Exchange a double with the other lane of the pair: DPP quad_perm [1,0,3,2]
// (one VALU op per 32-bit half, no LDS round trip as __shfl_xor would take).
__device__ __forceinline__ double pair_swap(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// ---------------------------------------------------------------- dynamics
// The tyre chain's libm (vehicledynamics.jl:32-44: atan, sin, and sin/cos(ψ)).  Default: the FDLIBM
// restatement of include/mp_jlmath.h -- Julia's own algorithms, bit-identical to the CPU oracle.
// (A/B) -DMPPI_LIBM_OCML=1: ROCm's device libm (__ocml_atan_f64 / sin / sincos, ~1 ulp,
// not Julia's bits) for the same calls, to measure what a non-FDLIBM tyre chain saves; tools/mppi_libm_ab.py
// compares it with the oracle at north_star's tolerances.  Not a shipped mode.
#ifndef MPPI_LIBM_OCML
#define MPPI_LIBM_OCML 0
#endif
#if MPPI_LIBM_OCML
#define TY_ATAN(x, tab) ::atan(x)
#define TY_SIN(x) ::sin(x)
#define TY_SINCOS(a, s, c) ::sincos((a), (s), (c))
#else
#define TY_ATAN(x, tab) mpj_atan_tab((x), (tab))
#define TY_SIN(x) mpj_sin_34(x)
#define TY_SINCOS(a, s, c) mpj_sincos_bl((a), (s), (c))
#endif
// VehicleDynamics for a lane pair.  side = lane & 1 (0: front tire, 1: rear).
// atab: the mpj_atan_tab range table (LDS).
//
// Lane constants of the pair, fixed for a rollout (kept in registers instead of selected every
// call): the axle load constant, the sign of t, the slip lever arm, the force-division operands.
struct PairK {
  double kfz, tsg, lr, cown, cother, div;
};
__device__ __forceinline__ PairK pair_k(int side) {
  const double la = 1.56, lb = 1.64, M = 2020.0, Izz = 4095.0;
  const double KFZF = 1018.28 / 2, KFZR = 963.34 / 2;
  PairK k;
  k.kfz = side ? KFZR : KFZF;
  k.tsg = side ? 1.0 : -1.0;
  k.lr = side ? -lb : la;
  k.cown = side ? -lb : 1.0;
  k.cother = side ? la : 1.0;
  k.div = side ? Izz : M;
  return k;
}
// dyn_pair with sin/cos(ψ) supplied (rollout_pair evaluates both RK2 stages' in one call)
__device__ __forceinline__ void dyn_pair_sc(const double* x, double sr, double ax, double* d, int side,
                                            const double* atab, double sp, double cp, const PairK& pk) {
  const double g = 9.81, mu = 0.8, KFZX = 186.22;
  const double B = -10.4 / mu, C = 1.3, E = 0.1556;
  const double v = x[2], r = x[3], ux = x[5], sa = x[6];
  const double t = (ax - r * v) * KFZX;
  // front: 2*(KFZF*g - t);  rear: 2*(KFZR*g + t)   (vehicledynamics.jl:30-31); t·(∓1) is exact
  const double FZ = 2 * (pk.kfz * g + t * pk.tsg);
  // front: (v + la*r) ... - sa;  rear: (v - lb*r) ... [(-lb)*r == -(lb*r) exactly]  (:32-33)
  const double alpha = TY_ATAN((v + pk.lr * r) / (ux + 0.01), atab) - (side ? 0.0 : sa);
  const double X1 = B * alpha;
  const double FY = mu * FZ * 1.0 * TY_SIN(C * TY_ATAN(X1 - E * (X1 - TY_ATAN(X1, atab)), atab));  // (:35-38)
  const double FYo = pair_swap(FY);
  const double uxc = MPJ_SEL(ux <= 0, 0.0, ux);  // (:40-42)
  d[0] = uxc * cp - v * sp;
  d[1] = uxc * sp + v * cp;
  // the two force divisions (:45-46) split across the pair: even lane (FY1+FY2)/M, odd lane
  // (FY1*la - FY2*lb)/Izz, exchanged with one DPP swap.  The numerator is own·cown + other·cother:
  // the same two rounded products (x·1.0 = x, y·(-lb) = -(y·lb)) summed commutatively, so the
  // same bits as the reference expression without selecting FY1/FY2 per lane.
  const double q = (FY * pk.cown + FYo * pk.cother) / pk.div;
  const double qo = pair_swap(q);
  d[2] = (side ? qo : q) - r * uxc;
  d[3] = side ? q : qo;
  d[4] = r;
  d[5] = ax;
  d[6] = sr;
}
__device__ __forceinline__ void dyn_pair(const double* x, double sr, double ax, double* d, int side, const double* atab) {
  double sp, cp;
  TY_SINCOS(x[4], &sp, &cp);
  dyn_pair_sc(x, sr, ax, d, side, atab, sp, cp, pair_k(side));
}

// VehicleDynamics for one lane holding the whole rollout: the front and rear tire chains of
// dyn_pair as two independent instruction chains of the same lane (the same operations on
// the same operands, so the same bits), no lane exchange.  Used when the launch has enough
// rollouts for one per lane to fill every SIMD: the costs and the state update are then not
// evaluated twice, and the two tire chains interleave in the single wave's latency bubbles.
__device__ __forceinline__ void dyn_lane(const double* x, double sr, double ax, double* d, const double* atab) {
  const double la = 1.56, lb = 1.64, M = 2020.0, Izz = 4095.0, g = 9.81, mu = 0.8;
  const double KFZF = 1018.28 / 2, KFZR = 963.34 / 2, KFZX = 186.22;
  const double B = -10.4 / mu, C = 1.3, E = 0.1556;
  const double v = x[2], r = x[3], psi = x[4], ux = x[5], sa = x[6];
  const double t = (ax - r * v) * KFZX;
  const double FZf = 2 * (KFZF * g + -t), FZr = 2 * (KFZR * g + t);
  const double af = TY_ATAN((v + la * r) / (ux + 0.01), atab) - sa;
  const double ar = TY_ATAN((v + (-lb) * r) / (ux + 0.01), atab) - 0.0;
  const double Xf = B * af, Xr = B * ar;
  const double FY1 = mu * FZf * 1.0 * TY_SIN(C * TY_ATAN(Xf - E * (Xf - TY_ATAN(Xf, atab)), atab));
  const double FY2 = mu * FZr * 1.0 * TY_SIN(C * TY_ATAN(Xr - E * (Xr - TY_ATAN(Xr, atab)), atab));
  const double uxc = MPJ_SEL(ux <= 0, 0.0, ux);
  double sp, cp;
  TY_SINCOS(psi, &sp, &cp);
  d[0] = uxc * cp - v * sp;
  d[1] = uxc * sp + v * cp;
  d[2] = (FY1 + FY2) / M - r * uxc;
  d[3] = (FY1 * la - FY2 * lb) / Izz;
  d[4] = r;
  d[5] = ax;
  d[6] = sr;
}

// running cost, vehicledynamics.jl:52
__device__ __forceinline__ double run_cost(const double* x, double sr, double ax) {
  const double y = x[1], v = x[2], r = x[3], sa = x[6];
  return v * v * 1 + 1 * (r * r) + 5 * (ax * ax) + 3 * (sr * sr) + 2 * (sa * sa) + 10 * (y * y);
}

// ObstacleEvaluation (MPPIUtils.jl:120-132) + occupancy grid (build extension).
// Branch-free: `c = hit ? c + pen : c` is bit-identical to `if (hit) c = c + pen`.
template <int LPR = 2>
__device__ __forceinline__ double obstacle_cost(const MppiDev& P, const double* x, const double* obs,
                                                const unsigned char* grid, int* ok, int side) {
  double c = 0.0;
  for (int o = 0; o < P.n_obs; o++) {
    const double dx = x[0] - obs[3 * o], dy = x[1] - obs[3 * o + 1], R = obs[3 * o + 2];
    const int hit = dx * dx + dy * dy <= R * R;
    *ok &= !hit;
    c = (hit ? c + P.obs_pen : c);
  }
  if (P.gnx > 0) {
    double fx, fy;
    if (LPR == 2) {  // cell coordinates: even lane divides x, odd lane y, one DPP swap
      const double f = (side ? x[1] - P.gy0 : x[0] - P.gx0) / (side ? P.gdy : P.gdx);
      const double fo = pair_swap(f);
      fx = side ? fo : f;
      fy = side ? f : fo;
    } else {
      fx = (x[0] - P.gx0) / P.gdx;
      fy = (x[1] - P.gy0) / P.gdy;
    }
    const int inb = fx >= 0.0 && fy >= 0.0 && fx < (double)P.gnx && fy < (double)P.gny;
    const int ix = inb ? (int)fx : 0, iy = inb ? (int)fy : 0;
    const int hit = inb && grid[iy * P.gnx + ix];
    *ok &= !hit;
    c = (hit ? c + P.obs_pen : c);
  }
  return c;
}

// BoundEvaluation, MPPIUtils.jl:135-151 (branch-free, same accumulation order)
__device__ __forceinline__ double bound_cost(const MppiDev& P, const double* x, int* ok) {
  int viol = 0;
#pragma unroll
  for (int i = 0; i < 7; i++) viol |= (x[i] < P.XL[i]) | (x[i] > P.XU[i]);
  *ok &= !viol;
  double c = 0.0;
  if (__any(viol)) {  // wave-uniform: with no violation in the wave every lane's sum is exactly 0.0
#pragma unroll
    for (int i = 0; i < 7; i++) {
      const int lo = x[i] < P.XL[i], hi = x[i] > P.XU[i];
      const double vl = c + P.slack * __builtin_fabs(x[i] - P.XL[i]);
      c = lo ? vl : c;
      const double vh = c + P.slack * __builtin_fabs(x[i] - P.XU[i]);
      c = hi ? vh : c;
    }
  }
  return c;
}

// ------------------------------------------------------------------ noise
__device__ __forceinline__ void philox4x32(unsigned c0, unsigned c1, unsigned c2, unsigned c3, unsigned k0,
                                           unsigned k1, unsigned* o) {
  // The key schedule is wave-uniform: an opaque register copy makes the scalar unit recompute
  // the 20 round keys per call (s_add), instead of the compiler hoisting them out of the rollout
  // loop, spilling them to VGPR lanes and restoring them with v_readlane (VALU work) every call.
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
    const unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    const unsigned n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  o[0] = c0;
  o[1] = c1;
  o[2] = c2;
  o[3] = c3;
}

// two N(0,1) draws for (scene, rollout k, step h): Philox4x32-10 + Box–Muller
__device__ __forceinline__ void philox_normal2(const MppiDev& P, unsigned scene, unsigned k, unsigned h,
                                               double* z) {
  unsigned o[4];
  philox4x32(k, h, scene + (unsigned)P.scene_base, (unsigned)P.offset, (unsigned)P.seed,
             (unsigned)(P.seed >> 32) ^ (unsigned)(P.offset >> 32), o);
  const unsigned long long b1 = ((unsigned long long)(o[0] >> 5) << 26) | (unsigned long long)(o[1] >> 6);
  const unsigned long long b2 = ((unsigned long long)(o[2] >> 5) << 26) | (unsigned long long)(o[3] >> 6);
  const double u1 = ((double)b1 + 0.5) * 1.1102230246251565e-16;
  const double u2 = ((double)b2 + 0.5) * 1.1102230246251565e-16;
  const double rr = mpj_sqrt(-2.0 * mpj_log_bl(u1));
  double sn, cs;
  mpj_sincos_bl(MPJ_TWO_PI * u2, &sn, &cs);
  z[0] = rr * cs;
  z[1] = rr * sn;
}

// SampleMPPIControl + PushInBounds (MPPIUtils.jl:5-20): u = min(max(u_nom + L z, CL), CU) with Julia's
// min / max (mpj_jmin / mpj_jmax): v_max_f64 / v_min_f64 already order -0.0 < +0.0, so only a NaN
// sample needs the select that keeps it NaN (the IEEE maxNum/minNum drop it).
__device__ __forceinline__ void sample_ctrl(const MppiDev& P, const double* z, const double* un, double* u) {
  const double n0 = P.L[0] * z[0];
  const double n1 = P.L[3] * z[1] + P.L[2] * z[0];
  const double v0 = n0 + un[0], v1 = n1 + un[1];
  const double c0 = __builtin_fmin(__builtin_fmax(v0, P.CL[0]), P.CU[0]);
  const double c1 = __builtin_fmin(__builtin_fmax(v1, P.CL[1]), P.CU[1]);
  u[0] = v0 != v0 ? v0 : c0;
  u[1] = v1 != v1 ? v1 : c1;
}

__device__ __forceinline__ void draw_ctrl(const MppiDev& P, const double* noise_s, const double* unom_s,
                                          unsigned scene, int k, int h, double* u) {
  double z[2];
  if (P.noise_mode == 0) {
    const double2 zz = *reinterpret_cast<const double2*>(noise_s + ((size_t)k * P.H + h) * 2);
    z[0] = zz.x;
    z[1] = zz.y;
  } else {
    philox_normal2(P, scene, (unsigned)k, (unsigned)h, z);
  }
  sample_ctrl(P, z, unom_s + 2 * h, u);
}

// Where a rollout's states go: state i of step j at p[j*rs + i*cs].  AoS rows
// (rs = 7, cs = 1: traj_out, mp_rollout) or the structure-of-arrays
// TrajectoryCollection (rs = 7K, cs = K, p offset by the rollout index k), whose
// per-step stores from a wavefront's 32 consecutive rollouts are full 128-B lines.
struct TrajOut {
  double* p;
  long long rs, cs;
};

// The even lane of the pair stores x[0..3], the odd lane x[4..6] (LPR 1: the lane all 7).
// TrajectoryCollection states are written once and read only by the caller: non-temporal stores
// (streaming, no L2 residency) -- 1.5-2 % off the 8-scene plan kernel (profiles/r03nt2_mppi_nt_ab.txt).
#ifndef MPPI_NT_STATE
#define MPPI_NT_STATE 1
#endif
__device__ __forceinline__ void st_state(double* a, double v) {
  if (MPPI_NT_STATE) __builtin_nontemporal_store(v, a);
  else *a = v;
}
template <int LPR = 2>
__device__ __forceinline__ void store_state(const TrajOut& T, int j, const double* x, int side) {
  double* q = T.p + (long long)j * T.rs;
  if (LPR == 1) {
#pragma unroll
    for (int i = 0; i < 7; i++) st_state(q + (long long)i * T.cs, x[i]);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double v = MPJ_SEL(side, x[4 + i < 7 ? 4 + i : 6], x[i]);
    if (!side || i < 3) st_state(q + (long long)(side ? 4 + i : i) * T.cs, v);
  }
}

// The control cost λ·u_nomᵀ·inv(Σ)·(u − u_nom) of step j (MPPIUtils.jl:45, Julia's n-ary `*` as a
// left fold, ((λ·u_nomᵀ)·inv(Σ))·d): its row vector t = (λ·u_nom)ᵀ·inv(Σ) depends only on the scene's
// nominal control, so the plan kernel evaluates it once per (scene, step) into LDS (same operations,
// same bits) instead of once per rollout-step.  The vector-matrix product is BLAS dgemv 'T' and the
// last one BLAS ddot in Julia; both round as OpenBLAS's FMA kernels do (oracle/or_blas.h).
__device__ __forceinline__ void ctrl_cost_row(const MppiDev& P, double un0, double un1, double* t) {
  const double a0 = P.lambda * un0, a1 = P.lambda * un1;
  t[0] = __builtin_fma(P.Si[0], a0, P.Si[2] * a1);
  t[1] = __builtin_fma(P.Si[1], a0, P.Si[3] * a1);
}

// --------------------------------------------------------------- rollout
// TrajectoryRollout for the lane pair (MPPIUtils.jl:31-57).  `ctrl(j, u)` yields the
// control of step j.  traj.p (optional) gets the H+1 states (store_state).
// cq: the control-cost rows [H][2] (ctrl_cost_row), or nullptr to evaluate them per step.
// Returns cost_total; *feas = constraint.
template <int LPR = 2, class CtrlFn, class StoreFn>
__device__ __forceinline__ double rollout_pair(const MppiDev& P, const double* X0, const double* goal,
                                               const double* obs, const unsigned char* grid,
                                               const double* unom, int side, CtrlFn ctrl, StoreFn store,
                                               const TrajOut& traj, int* feas, const double* atab,
                                               const double* cq = nullptr) {
  double x[7];
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = X0[i];
  const PairK pk = pair_k(side);
  if (traj.p) store_state<LPR>(traj, 0, x, side);
  double sum = 0.0;
  int ok_all = 1;
  for (int j = 0; j < P.H; j++) {
    double u[2];
    ctrl(j, u);
    store(j, u);
    int okc = 1, okb = 1;
    double cc = 0.0, cb = 0.0;
    if (j > 0) {
      cc = obstacle_cost<LPR>(P, x, obs, grid, &okc, side);
      cb = bound_cost(P, x, &okb);
    }
    const double pc = run_cost(x, u[0], u[1]);
    double k1[7], k2[7], x2[7];
    if (LPR == 2) {
      // sin/cos(ψ) of both RK2 stages in ONE call on the pair: the second stage's heading
      // x2[4] = x[4] + k1[4]·dt with k1[4] = r = x[3] needs no tyre force, so the even lane
      // evaluates stage 1's and the odd lane stage 2's, then they swap (same operands, same bits)
      const double psi2 = x[4] + x[3] * P.dt;
      double sn, cs;
      TY_SINCOS(side ? psi2 : x[4], &sn, &cs);
      const double so = pair_swap(sn), co = pair_swap(cs);
      dyn_pair_sc(x, u[0], u[1], k1, side, atab, side ? so : sn, side ? co : cs, pk);
#pragma unroll
      for (int i = 0; i < 7; i++) x2[i] = x[i] + k1[i] * P.dt;
      dyn_pair_sc(x2, u[0], u[1], k2, side, atab, side ? sn : so, side ? cs : co, pk);
    } else {
      dyn_lane(x, u[0], u[1], k1, atab);
#pragma unroll
      for (int i = 0; i < 7; i++) x2[i] = x[i] + k1[i] * P.dt;
      dyn_lane(x2, u[0], u[1], k2, atab);
    }
#pragma unroll
    for (int i = 0; i < 7; i++) x[i] = x[i] + P.dt * (k1[i] + k2[i]) / 2;
    double cj = pc + cb + cc;
    if (P.ctrl_cost) {
      const double un0 = unom[2 * j], un1 = unom[2 * j + 1];
      double t[2];
      if (cq) {
        t[0] = cq[2 * j];
        t[1] = cq[2 * j + 1];
      } else {
        ctrl_cost_row(P, un0, un1, t);
      }
      const double d0 = u[0] - un0, d1 = u[1] - un1;
      cj = cj + __builtin_fma(t[1], d1, t[0] * d0);  // ddot, n = 2
    }
    sum = sum + cj;
    ok_all &= okc & okb;
    if (traj.p) store_state<LPR>(traj, j + 1, x, side);
  }
  {  // terminal (:49-54): only the running cost of the extra RK2 step is used
    int okc = 1, okb = 1;
    const double pc = run_cost(x, 0.0, 0.0);
    const double cc = obstacle_cost<LPR>(P, x, obs, grid, &okc, side);
    const double cb = bound_cost(P, x, &okb);
    sum = sum + (pc + cb + cc);
    ok_all &= okc & okb;
  }
  const double tx = x[0] - goal[0], ty = x[1] - goal[1];
  const double term = tx * tx + ty * ty;
  const double dx0 = X0[0] - goal[0], dy0 = X0[1] - goal[1];
  *feas = ok_all;
  return sum + term / (dx0 * dx0 + dy0 * dy0) * 10000.0;
}

// Julia isless-style min that treats NaN as the smallest (findmin semantics)
__device__ __forceinline__ double nanmin(double a, double b) { return (a != a || a < b) ? a : b; }

}  // namespace mpk
