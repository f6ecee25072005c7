/*
 * ORACLE — test infrastructure only.  CPU restatement (scalar C, fp64) of the
 * reference's MPPI / DWA rollout path, op-for-op in the reference's evaluation
 * order.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this; the product (motionplanning_amd/) never does.
 *
 * Pinned by reference artifacts (tests/test_oracle_golden.py):
 *   - OptimalControl/DynamicWindow/DWATrajectory.csv (127 replans, full closed loop)
 *   - OptimalControl/MPPI/MPPITrajectory.csv         (VehicleDynamics + Euler plant)
 * The MPPI λ-control-cost term and the weight/average step have no artifact
 * (the reference's noise was unseeded): those are restatement-only.
 *
 * Libm: include/mp_jlmath.h (FDLIBM, the algorithms Julia's Base.Math ports).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mp_jlmath.h"
#include "../include/mpgpu.h"
#include "or_blas.h"

int or_blas = 1; /* or_blas.h: the products round as Julia's OpenBLAS dispatch rounds them */
void or_set_blas(int v) { or_blas = v; }
int or_get_blas(void) { return or_blas; }

/* OptimalControl/MPPI/src/vehicledynamics.jl:1-54.  Returns the running cost
 * (:52); ds gets dstates (:50). */
double or_vehicle_dynamics(const double* s, const double* c, double* ds) {
  const double la = 1.56, lb = 1.64, M = 2020.0, Izz = 4095.0, g = 9.81, mu = 0.8;
  const double KFZF = 1018.28 / 2, KFZR = 963.34 / 2, KFZX = 186.22;
  const double tp1 = -10.4, tp2 = 1.3, tp3 = 1.0, tp4 = 0.1556;
  volatile double vb = tp1; /* Tire_par[1]/mu evaluated at run time like Julia */
  const double B = vb / mu, C = tp2, E = tp4;
  double x = s[0], y = s[1], v = s[2], r = s[3], psi = s[4], ux = s[5], sa = s[6];
  double sr = c[0], ax = c[1];
  (void)x;
  double FZF = 2 * (KFZF * g - (ax - r * v) * KFZX);
  double FZR = 2 * (KFZR * g + (ax - r * v) * KFZX);
  double alpha_f = mpj_atan((v + la * r) / (ux + 0.01)) - sa;
  double alpha_r = mpj_atan((v - lb * r) / (ux + 0.01));
  double X1_f = B * alpha_f;
  double FY1 = mu * FZF * tp3 * mpj_sin(C * mpj_atan(X1_f - E * (X1_f - mpj_atan(X1_f))));
  double X1_r = B * alpha_r;
  double FY2 = mu * FZR * tp3 * mpj_sin(C * mpj_atan(X1_r - E * (X1_r - mpj_atan(X1_r))));
  if (ux <= 0) ux = 0.0;
  double sp = mpj_sin(psi), cp = mpj_cos(psi);
  ds[0] = ux * cp - v * sp;
  ds[1] = ux * sp + v * cp;
  ds[2] = (FY1 + FY2) / M - r * ux;
  ds[3] = (FY1 * la - FY2 * lb) / Izz;
  ds[4] = r;
  ds[5] = ax;
  ds[6] = sr;
  return v * v * 1 + 1 * (r * r) + 5 * (ax * ax) + 3 * (sr * sr) + 2 * (sa * sa) + 10 * (y * y);
}

/* Rungekutta2, MPPIUtils.jl:76-90 (the `cons` branch is dead: constraint == 0). */
static double rk2(const double* x, const double* c, double dt, double* xo) {
  double k1[7], k2[7], x2[7];
  double p = or_vehicle_dynamics(x, c, k1);
  for (int i = 0; i < 7; i++) x2[i] = x[i] + k1[i] * dt;
  or_vehicle_dynamics(x2, c, k2);
  for (int i = 0; i < 7; i++) xo[i] = x[i] + dt * (k1[i] + k2[i]) / 2;
  return p;
}

/* ObstacleEvaluation (MPPIUtils.jl:120-132) + occupancy-grid extension. */
static double obstacle_eval(const mp_mppi_params* p, const double* s, const double* obs,
                            const uint8_t* grid, int* ok) {
  double cost = 0.0;
  for (int o = 0; o < p->n_obs; o++) {
    double dx = s[0] - obs[3 * o], dy = s[1] - obs[3 * o + 1], R = obs[3 * o + 2];
    if (dx * dx + dy * dy <= R * R) {
      *ok = 0;
      cost = cost + p->obs_penalty;
    }
  }
  if (grid && p->grid_nx > 0) {
    double fx = (s[0] - p->grid_x0) / p->grid_dx;
    double fy = (s[1] - p->grid_y0) / p->grid_dy;
    if (fx >= 0.0 && fy >= 0.0 && fx < (double)p->grid_nx && fy < (double)p->grid_ny) {
      int ix = (int)fx, iy = (int)fy;
      if (grid[(size_t)iy * p->grid_nx + ix]) {
        *ok = 0;
        cost = cost + p->obs_penalty;
      }
    }
  }
  return cost;
}

/* BoundEvaluation, MPPIUtils.jl:135-151. */
static double bound_eval(const mp_mppi_params* p, const double* s, int* ok) {
  double cost = 0.0;
  for (int i = 0; i < 7; i++) {
    if (s[i] < p->XL[i]) {
      *ok = 0;
      cost = cost + p->slack_penalty * fabs(s[i] - p->XL[i]);
    }
    if (s[i] > p->XU[i]) {
      *ok = 0;
      cost = cost + p->slack_penalty * fabs(s[i] - p->XU[i]);
    }
  }
  return cost;
}

/* inv(Σ) for 2x2 (LU with partial pivoting, as LAPACK getrf/getri does). */
void or_inv2(const double* A, double* Ai) {
  double a = A[0], b = A[1], c = A[2], d = A[3];
  if (b == 0.0 && c == 0.0) {
    Ai[0] = 1.0 / a; Ai[1] = 0.0; Ai[2] = 0.0; Ai[3] = 1.0 / d;
    return;
  }
  int swap = fabs(c) > fabs(a);
  double p11 = swap ? c : a, p12 = swap ? d : b, q11 = swap ? a : c, q12 = swap ? b : d;
  double l = q11 / p11, u22 = q12 - l * p12;
  double iu11 = 1.0 / p11, iu22 = 1.0 / u22, iu12 = -(p12 * iu11) * iu22;
  /* inv(A) P^T = inv(U) inv(L);  inv(L) = [1 0; -l 1] */
  double m11 = iu11 - iu12 * l, m12 = iu12, m21 = -iu22 * l, m22 = iu22;
  if (swap) { Ai[0] = m12; Ai[1] = m11; Ai[2] = m22; Ai[3] = m21; }
  else { Ai[0] = m11; Ai[1] = m12; Ai[2] = m21; Ai[3] = m22; }
}

/* cholesky(Σ).L, row-major [L11 0; L21 L22] */
void or_chol2(const double* A, double* L) {
  double l11 = sqrt(A[0]);
  double l21 = A[2] / l11;
  double l22 = sqrt(A[3] - l21 * l21);
  L[0] = l11; L[1] = 0.0; L[2] = l21; L[3] = l22;
}

/*
 * TrajectoryRollout, MPPIUtils.jl:31-57 (DWA variant DWAUtils.jl:16-42 when
 * p->ctrl_cost == 0).  ctrl: H rows of 2 with row stride `cs` (0 = constant).
 * states_his[(H+1)][7] optional.  Returns cost_total; *feas = constraint.
 */
/* MPPIUtils.jl:45, λ * u_nom' * inv(Σ) * (u - u_nom): Base's n-ary `*` folds left, ((λ*u')*Σ⁻¹)*d;
 * the vector-matrix product is BLAS dgemv 'T' (Σ⁻¹' * λu) and the last one BLAS ddot (or_blas.h) */
static double ctrl_term(double lambda, const double* Si, const double* un, const double* u) {
  double a0 = lambda * un[0], a1 = lambda * un[1];
  double t0 = blv_t2(Si[0], a0, Si[2], a1), t1 = blv_t2(Si[1], a0, Si[3], a1);
  double d0 = u[0] - un[0], d1 = u[1] - un[1];
  return bl_dot2(t0, d0, t1, d1);
}
double or_mppi_ctrl_term(double lambda, const double* Si, const double* un, const double* u) {
  return ctrl_term(lambda, Si, un, u);
}

double or_rollout(const mp_mppi_params* p, const double* X0, const double* goal,
                  const double* ctrl, int64_t cs, const double* unom, const double* obs,
                  const uint8_t* grid, double* states_his, int* feas) {
  const int H = p->H;
  double Si[4];
  or_inv2(p->sigma, Si);
  double x[7], xn[7];
  memcpy(x, X0, sizeof x);
  if (states_his) memcpy(states_his, x, sizeof x);
  double sum = 0.0;
  int ok_all = 1;
  for (int j = 0; j < H; j++) {
    int okc = 1, okb = 1;
    double cc = 0.0, cb = 0.0;
    if (j > 0) {
      cc = obstacle_eval(p, x, obs, grid, &okc);
      cb = bound_eval(p, x, &okb);
    }
    const double* u = ctrl + (size_t)j * cs;
    double pc = rk2(x, u, p->dt, xn);
    memcpy(x, xn, sizeof x);
    double cj = pc + cb + cc;
    if (p->ctrl_cost) {
      const double* un = unom + 2 * j;
      cj = cj + ctrl_term(p->lambda, Si, un, u);
    }
    sum = sum + cj;
    if (!(okc && okb)) ok_all = 0;
    if (states_his) memcpy(states_his + 7 * (j + 1), x, sizeof x);
  }
  /* terminal, :49-54: RK2 at [0,0] (only its running cost is used) */
  {
    const double zero[2] = {0.0, 0.0};
    double k1[7];
    double pc = or_vehicle_dynamics(x, zero, k1);
    int okc = 1, okb = 1;
    double cc = obstacle_eval(p, x, obs, grid, &okc);
    double cb = bound_eval(p, x, &okb);
    sum = sum + (pc + cb + cc);
    if (!(okc && okb)) ok_all = 0;
  }
  double tx = x[0] - goal[0], ty = x[1] - goal[1];
  double term = tx * tx + ty * ty;
  double dx0 = X0[0] - goal[0], dy0 = X0[1] - goal[1];
  double total = sum + term / (dx0 * dx0 + dy0 * dy0) * 10000.0;
  *feas = ok_all;
  return total;
}

/* Philox4x32-10 (Salmon et al., SC'11), counter (k, h, scene, offset_lo), key seed. */
void or_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
               uint32_t out[4]) {
  for (int i = 0; i < 10; i++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* The device noise stream: two N(0,1) draws for (scene, rollout, step). */
void or_philox_normal2(uint64_t seed, uint64_t offset, uint32_t scene, uint32_t k, uint32_t h,
                       double* z) {
  uint32_t o[4];
  or_philox(k, h, scene, (uint32_t)offset, (uint32_t)seed,
            (uint32_t)(seed >> 32) ^ (uint32_t)(offset >> 32), o);
  uint64_t b1 = ((uint64_t)(o[0] >> 5) << 26) | (uint64_t)(o[1] >> 6);
  uint64_t b2 = ((uint64_t)(o[2] >> 5) << 26) | (uint64_t)(o[3] >> 6);
  double u1 = ((double)b1 + 0.5) * 1.1102230246251565e-16; /* 2^-53 */
  double u2 = ((double)b2 + 0.5) * 1.1102230246251565e-16;
  double rr = sqrt(-2.0 * mpj_log(u1));
  double sn, cs;
  mpj_sincos(MPJ_TWO_PI * u2, &sn, &cs);
  z[0] = rr * cs;
  z[1] = rr * sn;
}

/* SampleMPPIControl + PushInBounds, MPPIUtils.jl:5-20: u = min(max(u_nom + L z, CL), CU) with
 * Julia's min / max (a NaN sample stays NaN; -0.0 < +0.0). */
static void sample_ctrl(const mp_mppi_params* p, const double* L, const double* unom,
                        const double* z, double* u) {
  double n0 = L[0] * z[0];
  double n1 = L[3] * z[1] + L[2] * z[0];
  double v0 = n0 + unom[0], v1 = n1 + unom[1];
  u[0] = mpj_jmin(mpj_jmax(v0, p->CL[0]), p->CU[0]);
  u[1] = mpj_jmin(mpj_jmax(v1, p->CL[1]), p->CU[1]);
}

/*
 * MPPIPlan, MPPIUtils.jl:169-203, one scene.  noise[K][H][2] (external) or
 * NULL for the Philox stream of `scene`.  Returns 1 if a NaN cost was met.
 * coll_* optional (TrajectoryCollection); all K rollouts are produced.
 */
int or_mppi_plan(const mp_mppi_params* p, int scene, const double* X0, const double* goal,
                 const double* unom, const double* obs, const uint8_t* grid,
                 const double* noise, double* U_out, double* traj_out, double* cost_out,
                 int* feasible_out, int* rollout_count_out, int* feasible_count_out,
                 double* coll_traj, double* coll_ctrl, double* coll_cost, uint8_t* coll_feas) {
  const int K = p->K, H = p->H;
  double L[4];
  or_chol2(p->sigma, L);
  double* ctrls = (double*)malloc(sizeof(double) * (size_t)K * H * 2);
  double* costs = (double*)malloc(sizeof(double) * (size_t)K);
  int fc = 0, m = 0, nan_seen = 0;
  /* while FeasibilityCount <= FC && RolloutCount <= SamplingNumber (:175) */
  while (fc <= p->feasibility_count && m < K) {
    double* u = ctrls + (size_t)m * H * 2;
    for (int h = 0; h < H; h++) {
      double z[2];
      if (noise) { z[0] = noise[((size_t)m * H + h) * 2]; z[1] = noise[((size_t)m * H + h) * 2 + 1]; }
      else or_philox_normal2(p->seed, p->offset, (uint32_t)(scene + p->scene_base), (uint32_t)m, (uint32_t)h, z);
      sample_ctrl(p, L, unom + 2 * h, z, u + 2 * h);
    }
    int feas;
    double c = or_rollout(p, X0, goal, u, 2, unom, obs, grid,
                          coll_traj ? coll_traj + (size_t)m * (H + 1) * 7 : NULL, &feas);
    if (c != c) nan_seen = 1;
    if (feas) fc++;
    costs[m] = c;
    if (coll_ctrl) memcpy(coll_ctrl + (size_t)m * H * 2, u, sizeof(double) * H * 2);
    if (coll_cost) coll_cost[m] = c;
    if (coll_feas) coll_feas[m] = (uint8_t)feas;
    m++;
  }
  /* the collection beyond m is not produced by the reference; fill it anyway
   * so callers can compare all K rollouts against the device. */
  for (int i = m; i < K && (coll_traj || coll_ctrl || coll_cost || coll_feas); i++) {
    double* u = ctrls + (size_t)i * H * 2;
    for (int h = 0; h < H; h++) {
      double z[2];
      if (noise) { z[0] = noise[((size_t)i * H + h) * 2]; z[1] = noise[((size_t)i * H + h) * 2 + 1]; }
      else or_philox_normal2(p->seed, p->offset, (uint32_t)(scene + p->scene_base), (uint32_t)i, (uint32_t)h, z);
      sample_ctrl(p, L, unom + 2 * h, z, u + 2 * h);
    }
    int feas;
    double c = or_rollout(p, X0, goal, u, 2, unom, obs, grid,
                          coll_traj ? coll_traj + (size_t)i * (H + 1) * 7 : NULL, &feas);
    if (coll_ctrl) memcpy(coll_ctrl + (size_t)i * H * 2, u, sizeof(double) * H * 2);
    if (coll_cost) coll_cost[i] = c;
    if (coll_feas) coll_feas[i] = (uint8_t)feas;
  }
  /* CalculateMPPIWeights, :154-167 — argmin with Julia isless (NaN = smallest
   * for findmin; first index on ties). */
  int amin = 0;
  for (int i = 1; i < m; i++) {
    double a = costs[i], b = costs[amin];
    if (b != b) break;
    if (a != a || a < b) amin = i;
  }
  double rho = costs[amin];
  double eta = 0.0;
  for (int i = 0; i < m; i++) eta = eta + mpj_exp((-1.0) / p->lambda * (costs[i] - rho));
  for (int t = 0; t < H * 2; t++) U_out[t] = 0.0;
  for (int i = 0; i < m; i++) {
    double w = 1.0 / eta * mpj_exp((-1.0) / p->lambda * (costs[i] - rho));
    const double* u = ctrls + (size_t)i * H * 2;
    for (int t = 0; t < H * 2; t++) U_out[t] = U_out[t] + w * u[t];
  }
  int feas;
  double c = or_rollout(p, X0, goal, U_out, 2, unom, obs, grid, traj_out, &feas);
  *cost_out = c;
  *feasible_out = feas;
  *rollout_count_out = m + 1;
  *feasible_count_out = fc;
  free(ctrls);
  free(costs);
  return nan_seen;
}

/* DWAPlan, DynamicWindow/src/DWAUtils.jl:141-163: constant controls, `minimum`. */
int or_dwa_plan(const mp_mppi_params* p, const double* X0, const double* goal, int K,
                const double* ctrl, const double* obs, double* best_cost, double* costs) {
  int best = -1;
  double bc = 0.0;
  for (int i = 0; i < K; i++) {
    int feas;
    double c = or_rollout(p, X0, goal, ctrl + 2 * i, 0, NULL, obs, NULL, NULL, &feas);
    if (costs) costs[i] = c;
    if (best < 0 || mpj_isless(c, bc)) { best = i; bc = c; }
  }
  *best_cost = bc;
  return best;
}

/* Euler plant, MPPI/main.jl:259-261: states = states .+ dstates*δt. */
void or_vehicle_euler(double* states, const double* ctrl, double dt, int nsteps, double* his) {
  double ds[7];
  for (int t = 0; t < nsteps; t++) {
    or_vehicle_dynamics(states, ctrl, ds);
    for (int i = 0; i < 7; i++) states[i] = states[i] + ds[i] * dt;
    if (his) memcpy(his + 7 * t, states, sizeof(double) * 7);
  }
}

/*
 * The MPPI closed loop, OptimalControl/MPPI/main.jl:55-83, one scene.  Replan when
 * mod(time_idx - 1, update_idx) + 1 == 1 (:58): ShiftInitialCondition + NominalControl +
 * MPPIPlan (:59-61), NominalControls = r.Control (:62); the held control of plant step i of the
 * period is row hold[i] of it (the Constant{Previous} interpolation, :64-66); the plant
 * states .+= VehicleDynamics(states, u)*δt (:74-75); row [time_idx*δt; states] (:76); stop when
 * within the goal radius (:77-79).  noise: [R][K][H][2] for this scene or NULL (Philox with
 * counter word p->offset + replan).  Outputs as mp_mppi_closed_loop for one scene; logs are
 * [R][...].  Returns 1 if any plan met a NaN cost.
 */
int or_mppi_closed_loop(const mp_mppi_params* p, int scene, int update_steps, int max_steps, double dt,
                        double goal_radius, const int* hold, const double* X0, const double* goal,
                        const double* unom0, const double* obs, const uint8_t* grid, const double* noise,
                        double* his, int* n_rows, int* n_replans, double* U_log, double* traj_log,
                        double* cost_log, int* feas_log, int* rc_log) {
  const int H = p->H, K = p->K;
  const int R = (max_steps + update_steps - 1) / update_steps;
  const double r2 = goal_radius * goal_radius;
  mp_mppi_params q = *p;
  double states[7], ds[7];
  double* nominal = (double*)malloc(sizeof(double) * 2 * H);
  double* U = (double*)malloc(sizeof(double) * 2 * H);
  double* traj = (double*)malloc(sizeof(double) * 7 * (H + 1));
  memcpy(nominal, unom0, sizeof(double) * 2 * H);
  memcpy(states, X0, sizeof(states));
  his[0] = 0.0;
  memcpy(his + 1, X0, sizeof(double) * 7);
  int rows = 1, plans = 0, nan_seen = 0;
  for (int t = 1; t <= max_steps; t++) {
    const int i = (t - 1) % update_steps;
    if (i == 0) {
      const int r = plans++;
      double cost;
      int feas, rc, fc;
      q.offset = p->offset + (uint64_t)r;
      nan_seen |= or_mppi_plan(&q, scene, states, goal, nominal, obs, grid,
                               noise ? noise + (size_t)r * K * H * 2 : NULL, U, traj, &cost, &feas, &rc, &fc,
                               NULL, NULL, NULL, NULL);
      memcpy(nominal, U, sizeof(double) * 2 * H);
      if (U_log) memcpy(U_log + (size_t)r * 2 * H, U, sizeof(double) * 2 * H);
      if (traj_log) memcpy(traj_log + (size_t)r * 7 * (H + 1), traj, sizeof(double) * 7 * (H + 1));
      if (cost_log) cost_log[r] = cost;
      if (feas_log) feas_log[r] = feas;
      if (rc_log) rc_log[r] = rc;
    }
    const double* u = nominal + 2 * hold[i];
    or_vehicle_dynamics(states, u, ds);
    for (int k = 0; k < 7; k++) states[k] = states[k] + ds[k] * dt;
    double* row = his + (size_t)t * 8;
    row[0] = (double)t * dt;
    memcpy(row + 1, states, sizeof(double) * 7);
    rows = t + 1;
    const double ex = states[0] - goal[0], ey = states[1] - goal[1];
    if (ex * ex + ey * ey <= r2) break;
  }
  (void)R;
  *n_rows = rows;
  *n_replans = plans;
  free(nominal);
  free(U);
  free(traj);
  return nan_seen;
}

/* Scalar math entry points for tests/test_jlmath.py. */
double or_m_sin(double x) { return mpj_sin(x); }
double or_m_cos(double x) { return mpj_cos(x); }
double or_m_tan(double x) { return mpj_tan(x); }
double or_m_atan(double x) { return mpj_atan(x); }
double or_m_atan2(double y, double x) { return mpj_atan2(y, x); }
double or_m_asin(double x) { return mpj_asin(x); }
double or_m_acos(double x) { return mpj_acos(x); }
double or_m_exp(double x) { return mpj_exp(x); }
double or_m_log(double x) { return mpj_log(x); }
double or_m_modpi(double x) { return mpj_modpi(x); }
double or_m_atan_bl(double x) { return mpj_atan_bl(x); }
double or_m_modpi_bl(double x) { return mpj_modpi_bl(x); }
double or_m_atan2_bl(double y, double x) { return mpj_atan2_bl(y, x); }
double or_m_atan2_sel(double y, double x) { return mpj_atan2_sel(y, x); }
double or_m_exp_fdlibm(double x) { return mpj_exp_fdlibm(x); }
double or_m_sin_wide(double x) { double s, c; int b = 0; mpj_sincos_wide(x, &s, &c, &b); return b ? mpj_sin(x) : s; }
double or_m_cos_wide(double x) { double s, c; int b = 0; mpj_sincos_wide(x, &s, &c, &b); return b ? mpj_cos(x) : c; }
double or_m_tan_bl(double x) { return mpj_tan_bl(x); }
double or_m_tan_wide(double x) { int b = 0; const double t = mpj_tan_wide(x, &b); return b ? mpj_tan(x) : t; }
double or_m_atan_tab(double x) {
  static double tab[20];
  static int ready = 0;
  if (!ready) { mpj_atan_tab_init(tab); ready = 1; }
  return mpj_atan_tab(x, tab);
}
double or_m_sin_bl(double x) { return mpj_sin_bl(x); }
double or_m_sin_34(double x) { return mpj_sin_34(x); }
double or_m_log_bl(double x) { return mpj_log_bl(x); }
double or_m_cos_bl(double x) { double s, c; mpj_sincos_bl(x, &s, &c); return c; }
