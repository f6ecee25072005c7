/*
 * ORACLE — test infrastructure only.  CPU restatement of the Hybrid A* hot path:
 *   PathPlanning/HybridAstar/src/hybrid_astar_utils.jl   (planner, FindNewNode, RS_connected, Encode, ...)
 *   PathPlanning/ReedsSheppsCurves/src/ReedsSheppsUtils.jl (allpath, path1..12, createActPath, modπ)
 *   PathPlanning/CollisionDetection/src/utils.jl          (GetRectanglePts, SAT, ConvexCollision)
 * Scalar C, fp64, reference evaluation order; libm = include/mp_jlmath.h (FDLIBM).
 *
 * Parity status: no reference artifact exists for this path; the
 * discrete outputs (Encode indices, collision booleans, pop order) are pinned
 * GPU-vs-this-restatement bit-exactly, plus known-answer tests derived from the
 * reference text (CollisionDetection/main.jl:7-19, RS straight-ahead, table sizes).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mp_jlmath.h"
#include "../include/mpgpu.h"
#include "or_blas.h"

#define NRS 48
#define PI2 (MPJ_PI / 2)

/* ------------------------------------------------------------ ReedsShepp */
/* changeBasis, ReedsSheppsUtils.jl:2-11 */
void or_change_basis(const double* init, const double* term, double minR, double* out) {
  double p0 = init[2], pg = term[2];
  double dx = (term[0] - init[0]) / minR, dy = (term[1] - init[1]) / minR;
  double s0 = mpj_sin(p0), c0 = mpj_cos(p0);
  out[0] = dx * c0 + dy * s0;
  out[1] = -dx * s0 + dy * c0;
  out[2] = pg - p0;
}

static void polar(double a, double b, double* r, double* th) {
  *r = sqrt(a * a + b * b);
  *th = mpj_atan2(b, a);
}

/* one path word: fills travel/gear/steer rows (nrow <= 5); returns cost (Inf when infeasible) */
typedef struct { int n; double tr[5], ge[5], st[5]; } cmds_t;

static double finish(cmds_t* c, double t, double u, double v, double cost) {
  (void)c;
  if ((t < 0) || (v < 0) || (u < 0)) return INFINITY;
  return cost;
}

static double rs_path(int w, const double* s, cmds_t* c) {
  double x = s[0], y = s[1], p = s[2];
  double rho, th, t, u, v, a, cost;
  c->n = 0;
  switch (w) {
    case 1: /* LSL */
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &u, &t);
      v = mpj_modpi(p - t);
      cost = fabs(t) + fabs(u) + fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->st[0] = 1; c->st[1] = 0; c->st[2] = 1;
      return finish(c, t, u, v, cost);
    case 2: /* LSR */
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return INFINITY;
      u = sqrt(rho * rho - 4);
      t = mpj_modpi(th + mpj_atan2(2, u));
      v = mpj_modpi(t - p);
      cost = fabs(t) + fabs(u) + fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->st[0] = 1; c->st[1] = 0; c->st[2] = -1;
      return finish(c, t, u, v, cost);
    case 3: /* LRL */
    case 4: /* C|CC */
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho <= 4)) return INFINITY;
      a = mpj_acos(rho / 4);
      t = mpj_modpi(th + PI2 + a);
      u = mpj_modpi(MPJ_PI - 2 * a);
      v = (w == 3) ? mpj_modpi(p - t - u) : mpj_modpi(t + u - p);
      cost = fabs(t) + fabs(u) + fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = (w == 3) ? 1 : -1;
      return finish(c, t, u, v, cost);
    case 5: /* CC|C */
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho <= 4)) return INFINITY;
      u = mpj_acos(1 - (rho * rho) / 8);
      a = mpj_asin(2 * mpj_sin(u) / rho);
      t = mpj_modpi(th + PI2 - a);
      v = mpj_modpi(t - p - u);
      cost = fabs(t) + fabs(u) + fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1; c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = -1;
      return finish(c, t, u, v, cost);
    case 6: /* CCu|CuC */
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho <= 4)) return INFINITY;
      if (rho <= 2) {
        a = mpj_acos((rho + 2) / 4);
        t = mpj_modpi(th + PI2 + a);
        u = mpj_modpi(a);
        v = mpj_modpi(p - t + 2 * u);
      } else {
        a = mpj_acos((rho - 2) / 4);
        t = mpj_modpi(th + PI2 - a);
        u = mpj_modpi(MPJ_PI - a);
        v = mpj_modpi(p - t + 2 * u);
      }
      cost = fabs(t) + 2 * fabs(u) + fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = -1; c->ge[3] = -1;
      return finish(c, t, u, v, cost);
    case 7: { /* C|CuCu|C */
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      double u1 = (20 - rho * rho) / 16;
      if (!((rho <= 6) && (0 <= u1) && (u1 <= 1))) return INFINITY;
      u = mpj_acos(u1);
      a = mpj_asin(2 * mpj_sin(u) / rho);
      t = mpj_modpi(th + PI2 + a);
      v = mpj_modpi(t - p);
      cost = fabs(t) + 2 * fabs(u) + fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = 1;
      return finish(c, t, u, v, cost);
    }
    case 8: /* C|C(π/2)SC */
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return INFINITY;
      u = sqrt(rho * rho - 4) - 2;
      a = mpj_atan2(2, u + 2);
      t = mpj_modpi(th + PI2 + a);
      v = mpj_modpi(t - p + PI2);
      cost = fabs(t) + PI2 + fabs(u) + fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = PI2; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 0; c->st[3] = 1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = -1;
      return finish(c, t, u, v, cost);
    case 9: /* CS|C(π/2)C */
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return INFINITY;
      u = sqrt(rho * rho - 4) - 2;
      a = mpj_atan2(u + 2, 2);
      t = mpj_modpi(th + PI2 - a);
      v = mpj_modpi(t - p - PI2);
      cost = fabs(t) + fabs(u) + PI2 + fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = PI2; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = 0; c->st[2] = -1; c->st[3] = 1;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->ge[3] = -1;
      return finish(c, t, u, v, cost);
    case 10: /* C|C(π/2)SC */
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return INFINITY;
      t = mpj_modpi(th + PI2);
      u = rho - 2;
      v = mpj_modpi(p - t - PI2);
      cost = fabs(t) + fabs(u) + PI2 + fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = PI2; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 0; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = -1;
      return finish(c, t, u, v, cost);
    case 11: /* CSC(π/2)|C */
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return INFINITY;
      t = mpj_modpi(th);
      u = rho - 2;
      v = mpj_modpi(p - t - PI2);
      cost = fabs(t) + fabs(u) + PI2 + fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = PI2; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = 0; c->st[2] = 1; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->ge[3] = -1;
      return finish(c, t, u, v, cost);
    default: /* 12: C|C(π/2)SC(π/2)|C */
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 4)) return INFINITY;
      u = sqrt(rho * rho - 4) - 4;
      a = mpj_atan2(2, u + 4);
      t = mpj_modpi(th + PI2 + a);
      v = mpj_modpi(t - p);
      cost = fabs(t) + PI2 + fabs(u) + PI2 + fabs(v);
      c->n = 5; c->tr[0] = t; c->tr[1] = PI2; c->tr[2] = u; c->tr[3] = PI2; c->tr[4] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 0; c->st[3] = 1; c->st[4] = -1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = -1; c->ge[4] = 1;
      return finish(c, t, u, v, cost);
  }
}

/* allpath, ReedsSheppsUtils.jl:468-511.  cmds[48][5][3] (rows [travel, gear, steer],
 * zero rows / zero slots where infeasible), cost[48]; returns argmin (first NaN, else
 * first minimum — Julia findmin semantics). */
int or_ha_allpath(const double* s, double* cost, double* cmds) {
  memset(cmds, 0, sizeof(double) * NRS * 15);
  for (int w = 1; w <= 12; w++) {
    for (int var = 0; var < 4; var++) {
      double q[3] = {s[0], s[1], s[2]};
      if (var == 1) { q[0] = -q[0]; q[2] = -q[2]; }       /* timeflip :392-399 */
      else if (var == 2) { q[1] = -q[1]; q[2] = -q[2]; }  /* reflect  :383-390 */
      else if (var == 3) { q[0] = -q[0]; q[1] = -q[1]; }  /* reverse  :401-409 */
      cmds_t c;
      double cst = rs_path(w, q, &c);
      const int id = (w - 1) * 4 + var;
      if (cst < INFINITY) {
        for (int r = 0; r < c.n; r++) {
          double ge = c.ge[r], st = c.st[r];
          if (var == 1 || var == 3) ge = -1 * ge;
          if (var == 2 || var == 3) st = -1 * st;
          cmds[id * 15 + r * 3 + 0] = c.tr[r];
          cmds[id * 15 + r * 3 + 1] = ge;
          cmds[id * 15 + r * 3 + 2] = st;
        }
      }
      cost[id] = cst;
    }
  }
  int best = 0;
  for (int i = 1; i < NRS; i++) {
    double fm = cost[best], fx = cost[i];
    if (fm != fm) break;
    if (fx != fx || fx < fm) best = i;
  }
  return best;
}

/* createActPath, ReedsSheppsUtils.jl:440-466: path[n][3], returns n = 100*nseg + 1 */
int or_ha_act_path(const double* init, double minR, const double* cm, double* path) {
  int nseg = 0;
  for (int i = 0; i < 5; i++) {
    if (cm[i * 3 + 1] == 0) break;
    nseg++;
  }
  double s[3] = {init[0], init[1], init[2]};
  memcpy(path, s, sizeof s);
  int cnt = 1;
  for (int i = 0; i < nseg; i++) {
    double dt = fabs(cm[i * 3]) / 100;
    double v = cm[i * 3 + 1], st = cm[i * 3 + 2];
    for (int k = 0; k < 100; k++) {
      double d0 = v * mpj_cos(s[2]), d1 = v * mpj_sin(s[2]), d2 = st * v;
      d0 = d0 * minR;
      d1 = d1 * minR;
      s[0] = s[0] + d0 * dt;
      s[1] = s[1] + d1 * dt;
      s[2] = s[2] + d2 * dt;
      memcpy(path + 3 * cnt, s, sizeof s);
      cnt++;
    }
  }
  return cnt;
}

/* ------------------------------------------------------- collision check */
/* GetRectanglePts, CollisionDetection/src/utils.jl:14-25: pts[5][2].  R*pts is BLAS dgemm
 * (2x2 * 2x5, K = 2: or_blas.h blk2), then `.+ [ox; oy]`. */
static void rect_pts(double ox, double oy, double c, double s, double l, double w, double* pts) {
  const double px[5] = {-l, -l, l, l, -l}, py[5] = {w, -w, -w, w, w};
  for (int j = 0; j < 5; j++) {
    pts[2 * j] = blk2(c, px[j], -s, py[j]) + ox;
    pts[2 * j + 1] = blk2(s, px[j], c, py[j]) + oy;
  }
}
void or_ha_rect_pts(const double* blk, double* pts) { /* GetRectanglePts(block) with Julia's sin/cos */
  rect_pts(blk[0], blk[1], mpj_cos(blk[2]), mpj_sin(blk[2]), blk[3], blk[4], pts);
}

/* SeparatingAxisTheorem, utils.jl:37-62: 1 if an edge normal of `base` separates */
static int sat(const double* base, const double* other) {
  for (int e = 0; e < 4; e++) {
    double bx = base[2 * e], by = base[2 * e + 1];
    double vx = base[2 * e + 2] - bx, vy = base[2 * e + 3] - by;
    double nx = -vy, ny = vx;
    double mnb = 0, mxb = 0, mno = 0, mxo = 0;
    for (int j = 0; j < 5; j++) {
      /* transpose(pts .- bg_pt) * normal_vec: BLAS dgemv 'T' on the 2x5 (or_blas.h blv_t2) */
      double db = blv_t2(base[2 * j] - bx, nx, base[2 * j + 1] - by, ny);
      double dq = blv_t2(other[2 * j] - bx, nx, other[2 * j + 1] - by, ny);
      if (j == 0 || db < mnb) mnb = db;
      if (j == 0 || db > mxb) mxb = db;
      if (j == 0 || dq < mno) mno = dq;
      if (j == 0 || dq > mxo) mxo = dq;
    }
    if ((mxo <= mnb) || (mxb <= mno)) return 1;
  }
  return 0;
}

/* the projections of edge e's SAT test (utils.jl:48-49), for tests/test_oracle_blas.py */
void or_ha_sat_dps(const double* base, const double* other, int e, double* db, double* dq) {
  double bx = base[2 * e], by = base[2 * e + 1];
  double vx = base[2 * e + 2] - bx, vy = base[2 * e + 3] - by;
  double nx = -vy, ny = vx;
  for (int j = 0; j < 5; j++) {
    db[j] = blv_t2(base[2 * j] - bx, nx, base[2 * j + 1] - by, ny);
    dq[j] = blv_t2(other[2 * j] - bx, nx, other[2 * j + 1] - by, ny);
  }
}

/* ConvexCollision, utils.jl:64-74: 1 = no collision (note the && of both SATs) */
int or_ha_convex_free(const double* p1, const double* p2) { return sat(p1, p2) && sat(p2, p1); }

/* wall corners, Block2Pts */
static void wall_pts(const double* wl, double* pts) {
  rect_pts(wl[0], wl[1], mpj_cos(wl[2]), mpj_sin(wl[2]), wl[3], wl[4], pts);
}

/* tools/blas_replay.py's census: with or_ha_census set, every block check also evaluates every
 * (pose, wall) ConvexCollision under both or_blas conventions and counts the pairs and checks whose
 * booleans differ (the result returned is the current convention's). */
int or_ha_census = 0;
long long or_ha_census_n[4]; /* pairs, pairs split, checks, checks split */
void or_ha_census_set(int on) { or_ha_census = on; memset(or_ha_census_n, 0, sizeof or_ha_census_n); }
void or_ha_census_get(long long* out) { memcpy(out, or_ha_census_n, sizeof or_ha_census_n); }

static int block_free_mode(const mp_ha_params* p, const double* path, int n, const double* walls, int mode,
                           uint8_t* pair_free) {
  const int save = or_blas;
  or_blas = mode;
  const int sp = 5;
  int npose = n > sp ? (n - 1) / sp + 1 : 1;
  int nw = p->n_walls < 64 ? p->n_walls : 64;
  double L2 = p->vehicle_len / 2, W2 = p->vehicle_wid / 2;
  int all = 1;
  for (int i = 0; i < nw; i++) {
    double wp[10];
    wall_pts(walls + 5 * i, wp);
    for (int j = 0; j < npose; j++) {
      const double* q = path + 3 * (j * sp);
      double x = q[0] + L2 * mpj_cos(q[2]), y = q[1] + L2 * mpj_sin(q[2]);
      double yaw = mpj_modpi(q[2]);
      double vp[10];
      rect_pts(x, y, mpj_cos(yaw), mpj_sin(yaw), L2, W2, vp);
      const int f = or_ha_convex_free(wp, vp);
      pair_free[i * npose + j] = (uint8_t)f;
      all &= f;
    }
  }
  or_blas = save;
  return all;
}

/* block_collision_check, hybrid_astar_utils.jl:180-204 on path[n][3]; 1 = collision free */
int or_ha_block_free(const mp_ha_params* p, const double* path, int n, const double* walls) {
  if (or_ha_census) {
    const int npose = n > 5 ? (n - 1) / 5 + 1 : 1, np = (p->n_walls < 64 ? p->n_walls : 64) * npose;
    uint8_t* f0 = (uint8_t*)malloc((size_t)np * 2);
    const int r0 = block_free_mode(p, path, n, walls, 0, f0);
    const int r1 = block_free_mode(p, path, n, walls, 1, f0 + np);
    for (int i = 0; i < np; i++) or_ha_census_n[1] += f0[i] != f0[np + i];
    or_ha_census_n[0] += np;
    or_ha_census_n[2] += 1;
    or_ha_census_n[3] += r0 != r1;
    free(f0);
    return or_blas ? r1 : r0;
  }
  const int sp = 5;
  int npose = n > sp ? (n - 1) / sp + 1 : 1;
  double wp[64][10];
  int nw = p->n_walls < 64 ? p->n_walls : 64;
  for (int i = 0; i < nw; i++) wall_pts(walls + 5 * i, wp[i]);
  double L2 = p->vehicle_len / 2, W2 = p->vehicle_wid / 2;
  for (int i = 0; i < nw; i++) {
    for (int j = 0; j < npose; j++) {
      const double* q = path + 3 * (j * sp);
      double x = q[0] + L2 * mpj_cos(q[2]), y = q[1] + L2 * mpj_sin(q[2]);
      double yaw = mpj_modpi(q[2]);
      double vp[10];
      rect_pts(x, y, mpj_cos(yaw), mpj_sin(yaw), L2, W2, vp);
      if (!or_ha_convex_free(wp[i], vp)) return 0;
    }
  }
  return 1;
}

/* -------------------------------------------------------- lattice helpers */
/* regulate_states, hybrid_astar_utils.jl:211-222 */
void or_ha_regulate(const mp_ha_params* p, const double* s, double* o) {
  o[0] = mpj_round(s[0] / p->res[0]) * p->res[0];
  o[1] = mpj_round(s[1] / p->res[1]) * p->res[1];
  double psi = mpj_modpi(s[2]);
  o[2] = mpj_round(psi / p->res[2]) * p->res[2];
}

/* Encode, :316-350 (+ check_bounds :449-457) */
int64_t or_ha_encode(const mp_ha_params* p, const double* s) {
  const double* b = p->stbound;
  double x = s[0], y = s[1], psi = mpj_modpi(s[2]);
  x = fmax(fmin(x, b[1]), b[0]);
  y = fmax(fmin(y, b[3]), b[2]);
  psi = fmax(fmin(psi, b[5]), b[4]);
  double xid = mpj_round((x - b[0]) / p->res[0]) + 1;
  double yid = mpj_round((y - b[2]) / p->res[1]) + 1;
  double pid = mpj_round((psi - b[4]) / p->res[2]) + 1;
  double ynum = mpj_round((b[3] - b[2]) / p->res[1]) + 1;
  double pnum = mpj_round((b[5] - b[4]) / p->res[2]) + 1;
  double idx = (xid - 1) * ynum * pnum + (yid - 1) * pnum + pid;
  if (s[0] < b[0] || s[0] > b[1] || s[1] < b[2] || s[1] > b[3]) return 0;
  return (int64_t)idx;
}

/* neighbor_origin, :483-503 -> states_candi[nprim][3], paths_candi[nprim][ncol][3]; returns ncol */
int or_ha_neighbor_origin(double T, int n_steer, const double* steer, int n_gear, const double* gear, double* sc,
                          double* pc) {
  const double dt = 1e-2;
  int ncol = (int)floor(T / dt);
  for (int g = 0; g < n_gear; g++)
    for (int k = 0; k < n_steer; k++) {
      int id = g * n_steer + k;
      double s[3] = {0.0, 0.0, 0.0};
      for (int i = 0; i < ncol; i++) {
        double v = gear[g], c = steer[k];
        double d0 = v * mpj_cos(s[2]), d1 = v * mpj_sin(s[2]), d2 = c * v;
        s[0] = s[0] + d0 * dt;
        s[1] = s[1] + d1 * dt;
        s[2] = s[2] + d2 * dt;
        memcpy(pc + ((size_t)id * ncol + i) * 3, s, sizeof s);
      }
      memcpy(sc + 3 * id, s, sizeof s);
    }
  return ncol;
}

/* transform, :459-481 for one pose */
static void transform1(const double* node, const double* q, double* o) {
  double th = node[2], c = mpj_cos(th), s = mpj_sin(th);
  o[0] = q[0] * c - q[1] * s + node[0];
  o[1] = q[0] * s + q[1] * c + node[1];
  o[2] = q[2] + th;
}

/* rs_heuristic, :361-373 (use_astar = false) */
double or_ha_rs_heuristic(const mp_ha_params* p, const double* s, const double* goal) {
  double ns[3], cost[NRS], cmds[NRS * 15];
  or_change_basis(s, goal, p->minR, ns);
  int b = or_ha_allpath(ns, cost, cmds);
  return cost[b] * p->minR;
}

/* FindNewNode device-side part (:391-421) for one popped node */
void or_ha_expand(const mp_ha_params* p, const double* node, const double* goal, const double* walls,
                  const double* sc, const double* pc, double* nbs, int64_t* idx, uint8_t* fr, double* h) {
  double* path = (double*)malloc(sizeof(double) * 3 * p->n_col);
  for (int k = 0; k < p->n_prim; k++) {
    double t[3];
    transform1(node, sc + 3 * k, t);
    or_ha_regulate(p, t, nbs + 3 * k);
    idx[k] = or_ha_encode(p, nbs + 3 * k);
    fr[k] = 0;
    h[k] = 0.0;
    if (idx[k] == 0) continue;
    for (int i = 0; i < p->n_col; i++) transform1(node, pc + ((size_t)k * p->n_col + i) * 3, path + 3 * i);
    if (!or_ha_block_free(p, path, p->n_col, walls)) continue;
    fr[k] = 1;
    h[k] = or_ha_rs_heuristic(p, nbs + 3 * k, goal);
  }
  free(path);
}

/* RS_connected, :224-233: path[<=501][3]; returns 1 when the RS path is collision free */
int or_ha_rs_connect(const mp_ha_params* p, const double* node, const double* goal, const double* walls,
                     double* path, int32_t* len) {
  double ns[3], cost[NRS], cmds[NRS * 15];
  or_change_basis(node, goal, p->minR, ns);
  int b = or_ha_allpath(ns, cost, cmds);
  int n = or_ha_act_path(node, p->minR, cmds + 15 * b, path);
  *len = n;
  return or_ha_block_free(p, path, n, walls);
}

/* ------------------------------------------------------- planHybridAstar! */
typedef struct {
  int64_t parent; /* -1 = nothing */
  double st[3];
  int64_t index;
  double g, h, f;
} hnode;

typedef struct {
  hnode* nodes; int n, cap;          /* node storage (Dict values, mutable objects) */
  int64_t* keys; int* vals; int hcap; /* open-addressing Dict{Int64 -> node id} */
} store;

static int dict_find(store* S, int64_t key) {
  uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull;
  int i = (int)(h & (uint64_t)(S->hcap - 1));
  while (S->vals[i] >= 0) {
    if (S->keys[i] == key) return S->vals[i];
    i = (i + 1) & (S->hcap - 1);
  }
  return -1;
}
static void dict_put(store* S, int64_t key, int v) {
  uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull;
  int i = (int)(h & (uint64_t)(S->hcap - 1));
  while (S->vals[i] >= 0 && S->keys[i] != key) i = (i + 1) & (S->hcap - 1);
  S->keys[i] = key;
  S->vals[i] = v;
}

/* stable insertion sort of the open list by f (Julia isless) == sort! stable semantics */
static void stable_sort(int* open, int n, const hnode* nodes) {
  for (int i = 1; i < n; i++) {
    int v = open[i], j = i - 1;
    while (j >= 0 && mpj_isless(nodes[v].f, nodes[open[j]].f)) {
      open[j + 1] = open[j];
      j--;
    }
    open[j + 1] = v;
  }
}

/* The whole planner for one scene.  pop_seq gets the Encode index of every popped node.
 * states_out: hybrid_astar_states (goal->start order).  Returns 1 if a path was found. */
int or_ha_plan(const mp_ha_params* p, const double* start, const double* goal, const double* walls,
               const double* sc, const double* pc, int32_t* pops, int32_t* n_nodes, int64_t* pop_seq,
               int32_t* n_states, double* states_out, int32_t* rs_len, double* rs_path) {
  store S;
  S.cap = 1 << 16; S.n = 0; S.nodes = (hnode*)malloc(sizeof(hnode) * S.cap);
  S.hcap = 1 << 17; S.keys = (int64_t*)malloc(sizeof(int64_t) * S.hcap); S.vals = (int*)malloc(sizeof(int) * S.hcap);
  for (int i = 0; i < S.hcap; i++) S.vals[i] = -1;
  int ocap = 1 << 16, on = 0;
  int* open = (int*)malloc(sizeof(int) * ocap);
  double* nbs = (double*)malloc(sizeof(double) * 3 * p->n_prim);
  int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * p->n_prim);
  uint8_t* fr = (uint8_t*)malloc(p->n_prim);
  double* h = (double*)malloc(sizeof(double) * p->n_prim);
  double* path = (double*)malloc(sizeof(double) * 3 * 501);
  /* starting node (setup.jl:112-121) */
  hnode s0 = {-1, {start[0], start[1], start[2]}, or_ha_encode(p, start), 0, 0, 0};
  S.nodes[S.n] = s0;
  dict_put(&S, s0.index, S.n);
  open[on++] = S.n++;
  int64_t start_index = s0.index;
  int found = 0, loop = 0;
  *rs_len = 0;
  *n_states = 0;
  while (on > 0 && loop < p->max_pops) {
    loop++;
    stable_sort(open, on, S.nodes);
    int cur = open[0];
    memmove(open, open + 1, sizeof(int) * (on - 1));
    on--;
    pop_seq[loop - 1] = S.nodes[cur].index;
    int32_t len;
    int ok = or_ha_rs_connect(p, S.nodes[cur].st, goal, walls, path, &len);
    if (ok) {
      found = 1;
      *rs_len = len;
      memcpy(rs_path, path, sizeof(double) * 3 * len);
      int c = cur, ns = 0;
      memcpy(states_out + 3 * ns++, S.nodes[c].st, 24);
      while (S.nodes[c].parent >= 0 && S.nodes[c].index != start_index) {
        c = dict_find(&S, S.nodes[c].parent);
        memcpy(states_out + 3 * ns++, S.nodes[c].st, 24);
      }
      *n_states = ns;
      break;
    }
    /* FindNewNode (:391-447) */
    hnode cn = S.nodes[cur];
    or_ha_expand(p, cn.st, goal, walls, sc, pc, nbs, idx, fr, h);
    for (int k = 0; k < p->n_prim; k++) {
      if (idx[k] == 0 || !fr[k]) continue;
      double tg = cn.g + p->expand_time;
      double th = fmax(h[k], 0.0); /* max(rs_h, astar_h = 0) */
      if (h[k] != h[k]) th = h[k];  /* Julia max propagates NaN */
      double tf = tg + th;
      int id = dict_find(&S, idx[k]);
      int upd = 0;
      if (id >= 0) {
        if (tg < S.nodes[id].g) {
          S.nodes[id].g = tg; S.nodes[id].h = th; S.nodes[id].f = tf; S.nodes[id].parent = cn.index;
          upd = 1;
        }
      } else {
        if (S.n == S.cap) { S.cap *= 2; S.nodes = (hnode*)realloc(S.nodes, sizeof(hnode) * S.cap); }
        hnode nn = {cn.index, {nbs[3 * k], nbs[3 * k + 1], nbs[3 * k + 2]}, idx[k], tg, th, tf};
        id = S.n++;
        S.nodes[id] = nn;
        dict_put(&S, idx[k], id);
        upd = 1;
      }
      if (upd) {
        int in = 0;
        for (int q = 0; q < on; q++)
          if (S.nodes[open[q]].index == S.nodes[id].index) { in = 1; break; }
        if (!in) {
          if (on == ocap) { ocap *= 2; open = (int*)realloc(open, sizeof(int) * ocap); }
          open[on++] = id;
        }
      }
    }
  }
  *pops = loop;
  *n_nodes = S.n;
  free(S.nodes); free(S.keys); free(S.vals); free(open); free(nbs); free(idx); free(fr); free(h); free(path);
  return found;
}

/* ---------------------------------------------------------------- path finishing */
void or_pinv2(const double* M, double* P); /* or_ilqr.c: LinearAlgebra.pinv for a 2x2 */

/* cubic_fit, hybrid_astar_utils.jl:100-127: 100 points [x y ψ] from cur toward nxt. */
static void or_cubic_fit(const double* cur, const double* nxt, double* out /* [100][3] */) {
  double ns[3];
  or_change_basis(cur, nxt, 1.0, ns);
  const double xg = ns[0], yg = ns[1], pg = ns[2];
  /* A = [xg^3 xg^2; 3*xg^2 2*xg] (x^3 = x*x*x, Julia literal_pow), params = pinv(A)*[yg; tan(ψg)] */
  const double A[4] = {xg * xg * xg, xg * xg, 3 * (xg * xg), 2 * xg};
  double Pm[4];
  or_pinv2(A, Pm);
  const double b0 = yg, b1 = mpj_tan(pg);
  /* pinv(A)*B: BLAS dgemv 'N' 2x2 (or_blas.h blv_n22) */
  const double p1 = blv_n22(Pm[0], b0, Pm[1], b1), p2 = blv_n22(Pm[2], b0, Pm[3], b1);
  const double s0 = mpj_sin(cur[2]), c0 = mpj_cos(cur[2]);
  for (int k = 0; k < 100; k++) {
    const double t = (double)k / 99; /* LinRange(0, xg, 100): (1-t)*0 + t*xg */
    const double x = (1 - t) * 0.0 + t * xg;
    const double y = p1 * (x * x * x) + p2 * (x * x);
    const double psi = mpj_atan((3 * p1) * (x * x) + (2 * p2) * x);
    out[3 * k] = blk2(c0, x, -s0, y) + cur[0]; /* Rmat*path[1:2,:] (dgemm, K = 2) .+ [x0; y0] */
    out[3 * k + 1] = blk2(s0, x, c0, y) + cur[1];
    out[3 * k + 2] = psi + cur[2];
  }
}

/* retrievePath, :129-177, one scenario.  states: hybrid_astar_states as planned (goal side first),
 * n of them; rs[nr][3] RSpath_final.  pts[1 + 100(n-1) + nr][3] (actualpath columns), plen[...]
 * (cumulative arc length), samples[50][3] (x/y/ψ_interp_dense at LinRange(0, tol_length, 50); the
 * Interpolations.jl Gridded(Linear()) rule: last knot <= s, clamped to the last interval, weights
 * (1-δ, δ); a zero-width interval -- actualpath repeats points wherever an RS segment turns in place
 * or two consecutive states differ only in ψ -- takes its left value: a convention, since Julia's
 * result there depends on the (absent, unpinned) Interpolations.jl version).  Returns the number of points (0 when n == 0: nothing to retrieve). */
int or_ha_retrieve(const double* start, int n, const double* states, int nr, const double* rs, double* pts,
                   double* plen, double* tol, double* samples) {
  if (n < 1) {
    *tol = 0.0;
    memset(samples, 0, sizeof(double) * 150);
    return 0;
  }
  const int L = 1 + 100 * (n - 1) + nr;
  memcpy(pts, start, sizeof(double) * 3);
  for (int i = 0; i + 1 < n; i++) /* states reversed: start -> goal */
    or_cubic_fit(states + 3 * (n - 1 - i), states + 3 * (n - 2 - i), pts + 3 * (1 + 100 * i));
  memcpy(pts + 3 * (1 + 100 * (n - 1)), rs, sizeof(double) * 3 * nr);
  plen[0] = 0.0;
  for (int q = 1; q < L; q++) {
    const double dx = pts[3 * q] - pts[3 * (q - 1)], dy = pts[3 * q + 1] - pts[3 * (q - 1) + 1];
    plen[q] = plen[q - 1] + sqrt(dx * dx + dy * dy);
  }
  *tol = plen[L - 1];
  for (int j = 0; j < 50; j++) {
    const double t = (double)j / 49;
    const double s = (1 - t) * 0.0 + t * *tol;
    int i = 0;
    while (i + 1 < L && plen[i + 1] <= s) i++;
    if (L == 1) {
      memcpy(samples + 3 * j, pts, sizeof(double) * 3);
      continue;
    }
    if (i > L - 2) i = L - 2;
    const double w = plen[i + 1] - plen[i];
    const double d = w > 0.0 ? (s - plen[i]) / w : 0.0; /* duplicate knots: the left value */
    for (int c = 0; c < 3; c++) samples[3 * j + c] = (1 - d) * pts[3 * i + c] + d * pts[3 * (i + 1) + c];
  }
  return L;
}
