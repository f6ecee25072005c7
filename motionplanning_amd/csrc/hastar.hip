// hastar.hip — Hybrid A* hot path for gfx950 (PathPlanning/HybridAstar/src/hybrid_astar_utils.jl,
// ReedsSheppsCurves/src/ReedsSheppsUtils.jl, CollisionDetection/src/utils.jl) + C-ABI.
//
// ha_iter_kernel: one launch per search iteration for B scenes in lockstep.
//   block (s, 0)      RS_connected(node_s): the 48 Reeds–Shepp candidates on 48 lanes,
//                     Julia-argmin across the wave, the optimal command's 100-steps-per-
//                     segment Euler path (heading recurrence and x/y running sums on one
//                     lane, trigonometry on all lanes), then the SAT sweep of its poses.
//   block (s, 1+k)    FindNewNode neighbour k: transform + regulate + Encode, the 50-pose
//                     SAT collision sweep across lanes, and for a collision-free neighbour
//                     the 48-candidate rs_heuristic across lanes.
// The open list / Dict bookkeeping of planHybridAstar! runs on the host (mp_ha_plan).
#include <algorithm>
#include <cmath>
#include <unordered_map>
#include <vector>

#include "../../include/mp_jlmath.h"
#include "runtime.hpp"

namespace {

constexpr int MAXW = 16;    // walls per scene held in LDS
constexpr int MAXPATH = 501;
#define PI2 (MPJ_PI / 2)
#ifdef HA_DEBUG
// phase markers to host-mapped memory (tools/ha_dbg.cpp polls them while the kernel runs)
__device__ int* g_ha_dbg;
#define HMARK(ph) __hip_atomic_store(g_ha_dbg + (blockIdx.x * 64 + threadIdx.x), (ph), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
#else
#define HMARK(ph)
#endif

struct HaDev {
  double L2, W2, minR, expand_time;
  double res[3];
  double sb[6];
  int n_walls, n_prim, n_col;
};

// ------------------------------------------------------------ Reeds–Shepp
__device__ __forceinline__ void polar(double a, double b, double* r, double* th) {
  *r = mpj_sqrt(a * a + b * b);
  *th = mpj_atan2(b, a);
}

struct Cmd {
  int n;
  double tr[5], ge[5], st[5];
};

__device__ __forceinline__ double fin(double t, double u, double v, double cost) {
  if ((t < 0) || (v < 0) || (u < 0)) return __builtin_inf();
  return cost;
}

// path1..path12 (ReedsSheppsUtils.jl:48-380); identical operation order to oracle/or_hastar.c
__device__ __forceinline__ double rs_path(int w, const double* s, Cmd* c) {
  const double x = s[0], y = s[1], p = s[2];
  double rho, th, t, u, v, a, cost;
  c->n = 0;
  switch (w) {
    case 1:
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &u, &t);
      v = mpj_modpi(p - t);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->st[0] = 1; c->st[1] = 0; c->st[2] = 1;
      return fin(t, u, v, cost);
    case 2:
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return __builtin_inf();
      u = mpj_sqrt(rho * rho - 4);
      t = mpj_modpi(th + mpj_atan2(2, u));
      v = mpj_modpi(t - p);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->st[0] = 1; c->st[1] = 0; c->st[2] = -1;
      return fin(t, u, v, cost);
    case 3:
    case 4:
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho <= 4)) return __builtin_inf();
      a = mpj_acos(rho / 4);
      t = mpj_modpi(th + PI2 + a);
      u = mpj_modpi(MPJ_PI - 2 * a);
      v = (w == 3) ? mpj_modpi(p - t - u) : mpj_modpi(t + u - p);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = (w == 3) ? 1 : -1;
      return fin(t, u, v, cost);
    case 5:
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho <= 4)) return __builtin_inf();
      u = mpj_acos(1 - (rho * rho) / 8);
      a = mpj_asin(2 * mpj_sin(u) / rho);
      t = mpj_modpi(th + PI2 - a);
      v = mpj_modpi(t - p - u);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 3; c->tr[0] = t; c->tr[1] = u; c->tr[2] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1; c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = -1;
      return fin(t, u, v, cost);
    case 6:
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho <= 4)) return __builtin_inf();
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
      cost = __builtin_fabs(t) + 2 * __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = -1; c->ge[3] = -1;
      return fin(t, u, v, cost);
    case 7: {
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      const double u1 = (20 - rho * rho) / 16;
      if (!((rho <= 6) && (0 <= u1) && (u1 <= 1))) return __builtin_inf();
      u = mpj_acos(u1);
      a = mpj_asin(2 * mpj_sin(u) / rho);
      t = mpj_modpi(th + PI2 + a);
      v = mpj_modpi(t - p);
      cost = __builtin_fabs(t) + 2 * __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 1; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = 1;
      return fin(t, u, v, cost);
    }
    case 8:
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return __builtin_inf();
      u = mpj_sqrt(rho * rho - 4) - 2;
      a = mpj_atan2(2, u + 2);
      t = mpj_modpi(th + PI2 + a);
      v = mpj_modpi(t - p + PI2);
      cost = __builtin_fabs(t) + PI2 + __builtin_fabs(u) + __builtin_fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = PI2; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 0; c->st[3] = 1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = -1;
      return fin(t, u, v, cost);
    case 9:
      polar(x - mpj_sin(p), y - 1 + mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return __builtin_inf();
      u = mpj_sqrt(rho * rho - 4) - 2;
      a = mpj_atan2(u + 2, 2);
      t = mpj_modpi(th + PI2 - a);
      v = mpj_modpi(t - p - PI2);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + PI2 + __builtin_fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = PI2; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = 0; c->st[2] = -1; c->st[3] = 1;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->ge[3] = -1;
      return fin(t, u, v, cost);
    case 10:
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return __builtin_inf();
      t = mpj_modpi(th + PI2);
      u = rho - 2;
      v = mpj_modpi(p - t - PI2);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + PI2 + __builtin_fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = PI2; c->tr[2] = u; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 0; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = -1;
      return fin(t, u, v, cost);
    case 11:
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 2)) return __builtin_inf();
      t = mpj_modpi(th);
      u = rho - 2;
      v = mpj_modpi(p - t - PI2);
      cost = __builtin_fabs(t) + __builtin_fabs(u) + PI2 + __builtin_fabs(v);
      c->n = 4; c->tr[0] = t; c->tr[1] = u; c->tr[2] = PI2; c->tr[3] = v;
      c->st[0] = 1; c->st[1] = 0; c->st[2] = 1; c->st[3] = -1;
      c->ge[0] = 1; c->ge[1] = 1; c->ge[2] = 1; c->ge[3] = -1;
      return fin(t, u, v, cost);
    default:
      polar(x + mpj_sin(p), y - 1 - mpj_cos(p), &rho, &th);
      if (!(rho >= 4)) return __builtin_inf();
      u = mpj_sqrt(rho * rho - 4) - 4;
      a = mpj_atan2(2, u + 4);
      t = mpj_modpi(th + PI2 + a);
      v = mpj_modpi(t - p);
      cost = __builtin_fabs(t) + PI2 + __builtin_fabs(u) + PI2 + __builtin_fabs(v);
      c->n = 5; c->tr[0] = t; c->tr[1] = PI2; c->tr[2] = u; c->tr[3] = PI2; c->tr[4] = v;
      c->st[0] = 1; c->st[1] = -1; c->st[2] = 0; c->st[3] = 1; c->st[4] = -1;
      c->ge[0] = 1; c->ge[1] = -1; c->ge[2] = -1; c->ge[3] = -1; c->ge[4] = 1;
      return fin(t, u, v, cost);
  }
}

// Julia findmin order on (cost, candidate id): NaN first (lowest id among NaNs), else the
// smallest cost, ties to the lowest id.  A total order, so per-lane then cross-lane
// reduction gives the same winner as allpath's sequential findmin.
__device__ __forceinline__ bool rs_before(double a, int ia, double b, int ib) {
  const bool an = a != a, bn = b != b;
  if (an && bn) return ia < ib;
  if (an) return true;
  if (bn) return false;
  return (a < b) || (a == b && ia < ib);
}

// allpath + findmin (ReedsSheppsUtils.jl:383-436, hybrid_astar_utils.jl rs_heuristic /
// RS_connected).  The word loop is wave-uniform (no divergent 12-way switch): lane&3 is
// the variant (plain, timeflip, reflect, reverse) of candidate id = 4(w-1)+variant.
// Returns the winning cost in every lane; *best_id = winning id; if cm != nullptr the
// winner's commands [5][3] (distance, gear, steer) are written to cm (LDS) by one lane.
__device__ __forceinline__ void rs_variant(const double* s, int var, double* q) {
  q[0] = s[0]; q[1] = s[1]; q[2] = s[2];
  if (var == 1) { q[0] = -q[0]; q[2] = -q[2]; }       // timeflip
  else if (var == 2) { q[1] = -q[1]; q[2] = -q[2]; }  // reflect
  else if (var == 3) { q[0] = -q[0]; q[1] = -q[1]; }  // reverse
}

__device__ __forceinline__ double rs_best(const double* s, int lane, int* best_id, double* cm) {
  double q[3];
  rs_variant(s, lane & 3, q);
  double bc = __builtin_inf();
  int bi = 1 << 20;
#pragma unroll 1
  for (int w = 1; w <= 12; w++) {
    Cmd c;
    const double cost = rs_path(w, q, &c);
    const int id = 4 * (w - 1) + (lane & 3);
    if (rs_before(cost, id, bc, bi)) { bc = cost; bi = id; }
  }
#pragma unroll
  for (int o = 2; o >= 1; o >>= 1) {  // lanes 4j..4j+3 hold identical copies of variants 0..3
    const double ov = __shfl_xor(bc, o);
    const int oi = __shfl_xor(bi, o);
    if (rs_before(ov, oi, bc, bi)) { bc = ov; bi = oi; }
  }
  *best_id = bi;
  if (cm) {
    // the winner's commands: re-evaluate its word (wave-uniform), apply the variant's
    // gear / steer flips exactly as allpath does (-1 * x)
    const int wv = bi & 3;
    double qw[3];
    rs_variant(s, wv, qw);
    Cmd c;
    const double cost = rs_path(bi / 4 + 1, qw, &c);
    const int n = cost < __builtin_inf() ? c.n : 0;
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < 5; r++) {
        double ge = 0.0, st = 0.0, tr = 0.0;
        if (r < n) {
          tr = c.tr[r];
          ge = c.ge[r];
          st = c.st[r];
          if (wv == 1 || wv == 3) ge = -1 * ge;
          if (wv == 2 || wv == 3) st = -1 * st;
        }
        cm[r * 3 + 0] = tr;
        cm[r * 3 + 1] = ge;
        cm[r * 3 + 2] = st;
      }
    }
  }
  return bc;
}

__device__ __forceinline__ void change_basis(const double* init, const double* term, double minR, double* out) {
  const double p0 = init[2], pg = term[2];
  const double dx = (term[0] - init[0]) / minR, dy = (term[1] - init[1]) / minR;
  const double s0 = mpj_sin(p0), c0 = mpj_cos(p0);
  out[0] = dx * c0 + dy * s0;
  out[1] = -dx * s0 + dy * c0;
  out[2] = pg - p0;
}

// ------------------------------------------------------------- collision
__device__ __forceinline__ void rect_pts(double ox, double oy, double c, double s, double l, double w, double* pts) {
  const double px[5] = {-l, -l, l, l, -l}, py[5] = {w, -w, -w, w, w};
#pragma unroll
  for (int j = 0; j < 5; j++) {
    pts[2 * j] = c * px[j] + (-s) * py[j] + ox;
    pts[2 * j + 1] = s * px[j] + c * py[j] + oy;
  }
}

__device__ __forceinline__ int sat(const double* base, const double* other) {
  for (int e = 0; e < 4; e++) {
    const double bx = base[2 * e], by = base[2 * e + 1];
    const double vx = base[2 * e + 2] - bx, vy = base[2 * e + 3] - by;
    const double nx = -vy, ny = vx;
    double mnb = 0, mxb = 0, mno = 0, mxo = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const double db = (base[2 * j] - bx) * nx + (base[2 * j + 1] - by) * ny;
      const double dq = (other[2 * j] - bx) * nx + (other[2 * j + 1] - by) * ny;
      if (j == 0 || db < mnb) mnb = db;
      if (j == 0 || db > mxb) mxb = db;
      if (j == 0 || dq < mno) mno = dq;
      if (j == 0 || dq > mxo) mxo = dq;
    }
    if ((mxo <= mnb) || (mxb <= mno)) return 1;
  }
  return 0;
}

// vehicle pose q=[x,y,ψ] (rear axle) against all walls (corners in LDS); 1 = free
__device__ __forceinline__ int pose_free(const HaDev& P, const double* q, const double* wp, int nw) {
  const double x = q[0] + P.L2 * mpj_cos(q[2]), y = q[1] + P.L2 * mpj_sin(q[2]);
  const double yaw = mpj_modpi(q[2]);
  double vp[10];
  rect_pts(x, y, mpj_cos(yaw), mpj_sin(yaw), P.L2, P.W2, vp);
  for (int i = 0; i < nw; i++)
    if (!(sat(wp + 10 * i, vp) && sat(vp, wp + 10 * i))) return 0;
  return 1;
}

__device__ __forceinline__ void transform1(const double* node, const double* q, double* o) {
  const double th = node[2], c = mpj_cos(th), s = mpj_sin(th);
  o[0] = q[0] * c - q[1] * s + node[0];
  o[1] = q[0] * s + q[1] * c + node[1];
  o[2] = q[2] + th;
}

__device__ __forceinline__ void regulate(const HaDev& P, const double* s, double* o) {
  o[0] = mpj_round(s[0] / P.res[0]) * P.res[0];
  o[1] = mpj_round(s[1] / P.res[1]) * P.res[1];
  const double psi = mpj_modpi(s[2]);
  o[2] = mpj_round(psi / P.res[2]) * P.res[2];
}

__device__ __forceinline__ long long encode(const HaDev& P, const double* s) {
  const double* b = P.sb;
  double x = s[0], y = s[1], psi = mpj_modpi(s[2]);
  x = __builtin_fmax(__builtin_fmin(x, b[1]), b[0]);
  y = __builtin_fmax(__builtin_fmin(y, b[3]), b[2]);
  psi = __builtin_fmax(__builtin_fmin(psi, b[5]), b[4]);
  const double xid = mpj_round((x - b[0]) / P.res[0]) + 1;
  const double yid = mpj_round((y - b[2]) / P.res[1]) + 1;
  const double pid = mpj_round((psi - b[4]) / P.res[2]) + 1;
  const double ynum = mpj_round((b[3] - b[2]) / P.res[1]) + 1;
  const double pnum = mpj_round((b[5] - b[4]) / P.res[2]) + 1;
  const double idx = (xid - 1) * ynum * pnum + (yid - 1) * pnum + pid;
  if (s[0] < b[0] || s[0] > b[1] || s[1] < b[2] || s[1] > b[3]) return 0;
  return (long long)idx;
}

struct IterArgs {
  const double* node;    // [B][3]
  const double* goal;    // [B][3]
  const double* walls;   // [B][nw][5]
  const double* sc;      // [n_prim][3]
  const double* pc;      // [n_prim][n_col][3]
  const int* scene_of;   // active slot -> scene index
  int n_active;
  int do_rs, do_exp;
  // RS_connected outputs (per scene)
  unsigned char* rs_ok;  // [B]
  double* rs_path;       // [B][501][3]
  int* rs_len;           // [B]
  // FindNewNode outputs (per scene, per neighbour)
  double* nb;            // [B][n_prim][3]
  long long* idx;        // [B][n_prim]
  unsigned char* fr;     // [B][n_prim]
  double* h;             // [B][n_prim]
};

__global__ __launch_bounds__(64) void ha_iter_kernel(HaDev P, IterArgs A) {
  __shared__ double wp[MAXW * 10];
  __shared__ double cmd[15];
  __shared__ double psi_s[101], ix_s[101], iy_s[101];
  __shared__ double path_s[MAXPATH * 3];
  __shared__ int sh_best;
  const int per = 1 + P.n_prim;
  const int slot = blockIdx.x / per, item = blockIdx.x % per;
  if (slot >= A.n_active) return;
  if (item == 0 && !A.do_rs) return;
  if (item > 0 && !A.do_exp) return;
  const int s = A.scene_of[slot];
  const int lane = threadIdx.x;
  HMARK(1);
  const int nw = P.n_walls;
  const double* node = A.node + 3 * s;
  const double* goal = A.goal + 3 * s;
  // wall corners (Block2Pts) in LDS
  for (int i = lane; i < nw; i += 64) {
    const double* wl = A.walls + ((size_t)s * nw + i) * 5;
    rect_pts(wl[0], wl[1], mpj_cos(wl[2]), mpj_sin(wl[2]), wl[3], wl[4], wp + 10 * i);
  }
  HMARK(5);
  __syncthreads();
  HMARK(6);
  if (item == 0) {
    // ------------------------------------------------ RS_connected
    double ns[3];
    change_basis(node, goal, P.minR, ns);
    HMARK(7);
    int best;
    rs_best(ns, lane, &best, cmd);
    HMARK(3);
    __syncthreads();
    int nseg = 0;
    for (int i = 0; i < 5; i++) {
      if (cmd[i * 3 + 1] == 0) break;
      nseg++;
    }
    HMARK(4);
    double* path = A.rs_path + (size_t)s * MAXPATH * 3;
    double sx = node[0], sy = node[1], sp = node[2];
    if (lane == 0) { path_s[0] = sx; path_s[1] = sy; path_s[2] = sp; }
    for (int seg = 0; seg < nseg; seg++) {
      const double dt = __builtin_fabs(cmd[seg * 3]) / 100;
      const double v = cmd[seg * 3 + 1], st = cmd[seg * 3 + 2];
      // heading recurrence ψ_{k+1} = ψ_k + (st*v)*dt on one lane (adds only)
      if (lane == 0) {
        psi_s[0] = sp;
        double q = sp;
        for (int k = 0; k < 100; k++) {
          q = q + (st * v) * dt;
          psi_s[k + 1] = q;
        }
      }
      __syncthreads();
      // per-step increments (trigonometry on all lanes)
      for (int k = lane; k < 100; k += 64) {
        double sn, cs;
        mpj_sincos(psi_s[k], &sn, &cs);
        double d0 = v * cs, d1 = v * sn;
        d0 = d0 * P.minR;
        d1 = d1 * P.minR;
        ix_s[k] = d0 * dt;
        iy_s[k] = d1 * dt;
      }
      __syncthreads();
      if (lane == 0) {
        for (int k = 0; k < 100; k++) {
          sx = sx + ix_s[k];
          sy = sy + iy_s[k];
          double* o = path_s + 3 * (1 + seg * 100 + k);
          o[0] = sx;
          o[1] = sy;
          o[2] = psi_s[k + 1];
        }
      }
      sx = __shfl(sx, 0);
      sy = __shfl(sy, 0);
      sp = psi_s[100];
      HMARK(10 + seg);
      __syncthreads();
    }
    const int n = 100 * nseg + 1;
    __syncthreads();
    for (int i = lane; i < 3 * n; i += 64) path[i] = path_s[i];
    // block_collision_check on poses 1:5:end (or the first column only)
    const int npose = n > 5 ? (n - 1) / 5 + 1 : 1;
    int freep = 1;
    for (int j = lane; j < npose; j += 64) freep &= pose_free(P, path_s + 3 * (j * 5), wp, nw);
    HMARK(20);
    const int ok = !__any(!freep);
    if (lane == 0) {
      A.rs_ok[s] = (unsigned char)ok;
      A.rs_len[s] = n;
    }
    return;
  }
  // -------------------------------------------------- FindNewNode neighbour k
  const int k = item - 1;
  double t[3], nb[3];
  transform1(node, A.sc + 3 * k, t);
  regulate(P, t, nb);
  const long long ix = encode(P, nb);
  const size_t o = (size_t)s * P.n_prim + k;
  if (lane == 0) {
    A.nb[3 * o] = nb[0];
    A.nb[3 * o + 1] = nb[1];
    A.nb[3 * o + 2] = nb[2];
    A.idx[o] = ix;
  }
  if (ix == 0) {
    if (lane == 0) { A.fr[o] = 0; A.h[o] = 0.0; }
    return;
  }
  // dg_cost -> block_collision_check on primitive poses 1:5:n_col
  const int npose = P.n_col > 5 ? (P.n_col - 1) / 5 + 1 : 1;
  int freep = 1;
  for (int j = lane; j < npose; j += 64) {
    double q[3];
    transform1(node, A.pc + ((size_t)k * P.n_col + j * 5) * 3, q);
    freep &= pose_free(P, q, wp, nw);
  }
  if (__any(!freep)) {
    if (lane == 0) { A.fr[o] = 0; A.h[o] = 0.0; }
    return;
  }
  // rs_heuristic
  double ns[3];
  change_basis(nb, goal, P.minR, ns);
  int best;
  const double cb = rs_best(ns, lane, &best, nullptr);
  if (lane == 0) {
    A.fr[o] = 1;
    A.h[o] = cb * P.minR;
  }
}

// allpath over B normalised states: 16 states per wave, lanes 4j..4j+3 = the four variants
// of state j; the word loop is wave-uniform.  cost[B][48], cmds[B][48][5][3], best[B].
__global__ __launch_bounds__(64) void allpath_kernel(int B, const double* __restrict__ ns, double* __restrict__ cost,
                                                     double* __restrict__ cmds, int* __restrict__ best) {
  const int lane = threadIdx.x, var = lane & 3;
  const int b = blockIdx.x * 16 + (lane >> 2);
  const bool live = b < B;
  double s[3] = {0.0, 0.0, 0.0};
  if (live) { s[0] = ns[3 * b]; s[1] = ns[3 * b + 1]; s[2] = ns[3 * b + 2]; }
  double q[3];
  rs_variant(s, var, q);
  double bc = __builtin_inf();
  int bi = 1 << 20;
#pragma unroll 1
  for (int w = 1; w <= 12; w++) {
    Cmd c;
    const double cst = rs_path(w, q, &c);
    const int id = 4 * (w - 1) + var;
    if (rs_before(cst, id, bc, bi)) { bc = cst; bi = id; }
    if (live) {
      cost[(size_t)b * 48 + id] = cst;
      double* o = cmds + ((size_t)b * 48 + id) * 15;
      const int n = cst < __builtin_inf() ? c.n : 0;
#pragma unroll
      for (int r = 0; r < 5; r++) {
        double tr = 0.0, ge = 0.0, st = 0.0;
        if (r < n) {
          tr = c.tr[r];
          ge = c.ge[r];
          st = c.st[r];
          if (var == 1 || var == 3) ge = -1 * ge;
          if (var == 2 || var == 3) st = -1 * st;
        }
        o[3 * r] = tr;
        o[3 * r + 1] = ge;
        o[3 * r + 2] = st;
      }
    }
  }
#pragma unroll
  for (int o = 2; o >= 1; o >>= 1) {
    const double ov = __shfl_xor(bc, o);
    const int oi = __shfl_xor(bi, o);
    if (rs_before(ov, oi, bc, bi)) { bc = ov; bi = oi; }
  }
  if (live && var == 0) best[b] = bi;
}

// ---------------------------------------------------------------- host
int make_ha(mp_ctx* ctx, const mp_ha_params* p, HaDev* D) {
  MP_CHECK(ctx, p != nullptr, "params is NULL");
  MP_CHECK(ctx, p->n_walls >= 0 && p->n_walls <= MAXW, "n_walls (%d) must be in [0, %d]", p->n_walls, MAXW);
  MP_CHECK(ctx, p->n_prim >= 1 && p->n_col >= 1, "bad primitive table size");
  MP_CHECK(ctx, p->minR > 0 && p->res[0] > 0 && p->res[1] > 0 && p->res[2] > 0, "minR and resolutions must be > 0");
  D->L2 = p->vehicle_len / 2;
  D->W2 = p->vehicle_wid / 2;
  D->minR = p->minR;
  D->expand_time = p->expand_time;
  for (int i = 0; i < 3; i++) D->res[i] = p->res[i];
  for (int i = 0; i < 6; i++) D->sb[i] = p->stbound[i];
  D->n_walls = p->n_walls;
  D->n_prim = p->n_prim;
  D->n_col = p->n_col;
  return MP_OK;
}

int need_prims(mp_ctx* ctx, const mp_ha_params* p) {
  MP_CHECK(ctx, ctx->ha_states_candi && ctx->ha_n_prim == p->n_prim && ctx->ha_n_col == p->n_col,
           "primitive table not installed for n_prim=%d n_col=%d (call mp_ha_neighbor_origin / mp_ha_set_primitives)",
           p->n_prim, p->n_col);
  return MP_OK;
}

int launch_iter(mp_ctx* ctx, const HaDev& D, IterArgs& A) {
  if (A.n_active <= 0) return MP_OK;
  mp_time_begin(ctx);
  hipLaunchKernelGGL(ha_iter_kernel, dim3((unsigned)(A.n_active * (1 + D.n_prim))), dim3(64), 0, ctx->stream, D, A);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  return MP_OK;
}

struct HNode {
  long long parent;  // -1 = nothing
  double st[3];
  long long index;
  double g, h, f;
};

}  // namespace

extern "C" {
#ifdef HA_DEBUG
int mp_ha_debug_buf(int* host_mapped) {
  int* d = nullptr;
  hipHostGetDevicePointer((void**)&d, host_mapped, 0);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ha_dbg), &d, sizeof d) == hipSuccess ? 0 : 1;
}
#endif

int mp_ha_set_primitives(mp_ctx* ctx, const mp_ha_params* p, const double* states_candi, const double* paths_candi) {
  if (!ctx) return MP_ERR_INVALID;
  HaDev D;
  int st = make_ha(ctx, p, &D);
  if (st) return st;
  MP_CHECK(ctx, states_candi && paths_candi, "required pointer is NULL");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->ha_states_candi) { hipFree(ctx->ha_states_candi); ctx->ha_states_candi = nullptr; }
  if (ctx->ha_paths_candi) { hipFree(ctx->ha_paths_candi); ctx->ha_paths_candi = nullptr; }
  MP_HIP(ctx, hipMalloc(&ctx->ha_states_candi, sizeof(double) * 3 * p->n_prim));
  MP_HIP(ctx, hipMalloc(&ctx->ha_paths_candi, sizeof(double) * 3 * (size_t)p->n_prim * p->n_col));
  MP_HIP(ctx, hipMemcpy(ctx->ha_states_candi, states_candi, sizeof(double) * 3 * p->n_prim, hipMemcpyHostToDevice));
  MP_HIP(ctx, hipMemcpy(ctx->ha_paths_candi, paths_candi, sizeof(double) * 3 * (size_t)p->n_prim * p->n_col,
                        hipMemcpyHostToDevice));
  ctx->ha_n_prim = p->n_prim;
  ctx->ha_n_col = p->n_col;
  return MP_OK;
}

int mp_ha_neighbor_origin(mp_ctx* ctx, const mp_ha_params* p, int32_t n_steer, const double* steer_set,
                          int32_t n_gear, const double* gear_set, double* states_candi, double* paths_candi) {
  if (!ctx) return MP_ERR_INVALID;
  MP_CHECK(ctx, p && steer_set && gear_set && n_steer >= 1 && n_gear >= 1, "bad arguments");
  MP_CHECK(ctx, p->n_prim == n_steer * n_gear, "n_prim (%d) != n_gear*n_steer (%d)", p->n_prim, n_steer * n_gear);
  const double dt = 1e-2;
  const int ncol = (int)std::floor(p->expand_time / dt);
  MP_CHECK(ctx, ncol == p->n_col, "n_col (%d) != floor(expand_time/0.01) (%d)", p->n_col, ncol);
  std::vector<double> sc(3 * (size_t)p->n_prim), pc(3 * (size_t)p->n_prim * ncol);
  // hybrid_astar_utils.jl:483-503 (FDLIBM sin/cos on the host: setup-time, 62 x 250 steps)
  for (int g = 0; g < n_gear; g++)
    for (int k = 0; k < n_steer; k++) {
      const int id = g * n_steer + k;
      double s[3] = {0.0, 0.0, 0.0};
      for (int i = 0; i < ncol; i++) {
        const double v = gear_set[g], c = steer_set[k];
        const double d0 = v * mpj_cos(s[2]), d1 = v * mpj_sin(s[2]), d2 = c * v;
        s[0] = s[0] + d0 * dt;
        s[1] = s[1] + d1 * dt;
        s[2] = s[2] + d2 * dt;
        for (int r = 0; r < 3; r++) pc[((size_t)id * ncol + i) * 3 + r] = s[r];
      }
      for (int r = 0; r < 3; r++) sc[3 * id + r] = s[r];
    }
  if (states_candi) std::copy(sc.begin(), sc.end(), states_candi);
  if (paths_candi) std::copy(pc.begin(), pc.end(), paths_candi);
  return mp_ha_set_primitives(ctx, p, sc.data(), pc.data());
}

int mp_ha_expand(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* node, const double* goal,
                 const double* walls, double* nb_states, int64_t* idx, uint8_t* free_, double* h) {
  if (!ctx) return MP_ERR_INVALID;
  HaDev D;
  int st = make_ha(ctx, p, &D);
  if (st) return st;
  if ((st = need_prims(ctx, p))) return st;
  MP_CHECK(ctx, B >= 1 && node && goal && (walls || p->n_walls == 0) && nb_states && idx && free_ && h,
           "bad arguments");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const size_t np = p->n_prim;
  IterArgs A{};
  A.node = mp_upload(ctx, WS_IO0, node, 3 * (size_t)B, &st);
  A.goal = mp_upload(ctx, WS_IO1, goal, 3 * (size_t)B, &st);
  A.walls = p->n_walls ? mp_upload(ctx, WS_IO2, walls, 5 * (size_t)p->n_walls * B, &st) : nullptr;
  std::vector<int> so(B);
  for (int i = 0; i < B; i++) so[i] = i;
  A.scene_of = mp_upload(ctx, WS_IO3, so.data(), (size_t)B, &st);
  A.nb = mp_alloc_out(ctx, WS_IO4, nb_states, 3 * np * B, &st);
  A.idx = (long long*)mp_alloc_out(ctx, WS_IO5, idx, np * B, &st);
  A.fr = mp_alloc_out(ctx, WS_IO6, free_, np * B, &st);
  A.h = mp_alloc_out(ctx, WS_IO7, h, np * B, &st);
  if (st) return st;
  A.sc = ctx->ha_states_candi;
  A.pc = ctx->ha_paths_candi;
  A.n_active = B;
  A.do_rs = 0;
  A.do_exp = 1;
  if ((st = launch_iter(ctx, D, A))) return st;
  if ((st = mp_download(ctx, nb_states, (const double*)A.nb, 3 * np * B))) return st;
  if ((st = mp_download(ctx, (long long*)idx, (const long long*)A.idx, np * B))) return st;
  if ((st = mp_download(ctx, free_, (const uint8_t*)A.fr, np * B))) return st;
  if ((st = mp_download(ctx, h, (const double*)A.h, np * B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_ha_rs_connect(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* node, const double* goal,
                     const double* walls, uint8_t* ok, double* path, int32_t* path_len) {
  if (!ctx) return MP_ERR_INVALID;
  HaDev D;
  int st = make_ha(ctx, p, &D);
  if (st) return st;
  MP_CHECK(ctx, B >= 1 && node && goal && (walls || p->n_walls == 0) && ok && path && path_len, "bad arguments");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  IterArgs A{};
  A.node = mp_upload(ctx, WS_IO0, node, 3 * (size_t)B, &st);
  A.goal = mp_upload(ctx, WS_IO1, goal, 3 * (size_t)B, &st);
  A.walls = p->n_walls ? mp_upload(ctx, WS_IO2, walls, 5 * (size_t)p->n_walls * B, &st) : nullptr;
  std::vector<int> so(B);
  for (int i = 0; i < B; i++) so[i] = i;
  A.scene_of = mp_upload(ctx, WS_IO3, so.data(), (size_t)B, &st);
  A.rs_ok = mp_alloc_out(ctx, WS_IO4, ok, (size_t)B, &st);
  A.rs_path = mp_alloc_out(ctx, WS_IO5, path, (size_t)B * MAXPATH * 3, &st);
  A.rs_len = mp_alloc_out(ctx, WS_IO6, path_len, (size_t)B, &st);
  if (st) return st;
  A.n_active = B;
  A.do_rs = 1;
  A.do_exp = 0;
  if ((st = launch_iter(ctx, D, A))) return st;
  if ((st = mp_download(ctx, ok, (const uint8_t*)A.rs_ok, (size_t)B))) return st;
  if ((st = mp_download(ctx, path, (const double*)A.rs_path, (size_t)B * MAXPATH * 3))) return st;
  if ((st = mp_download(ctx, path_len, (const int32_t*)A.rs_len, (size_t)B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_ha_allpath(mp_ctx* ctx, int32_t B, const double* norm_states, double* cost, double* cmds, int32_t* best) {
  if (!ctx) return MP_ERR_INVALID;
  MP_CHECK(ctx, B >= 1 && norm_states && cost && cmds && best, "bad arguments");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  int st = MP_OK;
  const double* dns = mp_upload(ctx, WS_IO0, norm_states, 3 * (size_t)B, &st);
  double* dcost = mp_alloc_out(ctx, WS_IO1, cost, 48 * (size_t)B, &st);
  double* dcmds = mp_alloc_out(ctx, WS_IO2, cmds, 48 * 15 * (size_t)B, &st);
  int32_t* dbest = mp_alloc_out(ctx, WS_IO3, best, (size_t)B, &st);
  if (st) return st;
  mp_time_begin(ctx);
  hipLaunchKernelGGL(allpath_kernel, dim3((unsigned)((B + 15) / 16)), dim3(64), 0, ctx->stream, B, dns, dcost, dcmds,
                     (int*)dbest);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  if ((st = mp_download(ctx, cost, (const double*)dcost, 48 * (size_t)B))) return st;
  if ((st = mp_download(ctx, cmds, (const double*)dcmds, 48 * 15 * (size_t)B))) return st;
  if ((st = mp_download(ctx, best, (const int32_t*)dbest, (size_t)B))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

int mp_ha_plan(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* start, const double* goal,
               const double* walls, int32_t* found, int32_t* pops, int32_t* n_nodes, int64_t* pop_seq,
               int32_t* n_states, double* states_out, int32_t* rs_len, double* rs_path) {
  if (!ctx) return MP_ERR_INVALID;
  HaDev D;
  int st = make_ha(ctx, p, &D);
  if (st) return st;
  if ((st = need_prims(ctx, p))) return st;
  MP_CHECK(ctx, B >= 1 && start && goal && (walls || p->n_walls == 0) && found && pops && n_nodes && pop_seq &&
               n_states && states_out && rs_len && rs_path, "bad arguments");
  MP_CHECK(ctx, p->max_pops >= 1, "max_pops must be >= 1");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const int np = p->n_prim, mp = p->max_pops;
  IterArgs A{};
  A.goal = mp_upload(ctx, WS_HA0, goal, 3 * (size_t)B, &st);
  A.walls = p->n_walls ? mp_upload(ctx, WS_HA1, walls, 5 * (size_t)p->n_walls * B, &st) : nullptr;
  double* dnode = (double*)mp_ws(ctx, WS_IO0, sizeof(double) * 3 * B);
  int* dso = (int*)mp_ws(ctx, WS_IO1, sizeof(int) * B);
  A.rs_ok = (unsigned char*)mp_ws(ctx, WS_IO2, B);
  A.rs_path = (double*)mp_ws(ctx, WS_IO3, sizeof(double) * B * MAXPATH * 3);
  A.rs_len = (int*)mp_ws(ctx, WS_IO4, sizeof(int) * B);
  A.nb = (double*)mp_ws(ctx, WS_IO5, sizeof(double) * 3 * np * B);
  A.idx = (long long*)mp_ws(ctx, WS_IO6, sizeof(long long) * np * B);
  A.fr = (unsigned char*)mp_ws(ctx, WS_IO7, (size_t)np * B);
  A.h = (double*)mp_ws(ctx, WS_IO8, sizeof(double) * np * B);
  if (st || !dnode || !dso || !A.rs_ok || !A.rs_path || !A.rs_len || !A.nb || !A.idx || !A.fr || !A.h)
    return st ? st : MP_ERR_NOMEM;
  A.node = dnode;
  A.scene_of = dso;
  A.sc = ctx->ha_states_candi;
  A.pc = ctx->ha_paths_candi;
  A.do_rs = 1;
  A.do_exp = 1;
  // pinned staging: nodes + scene map in, results out
  const size_t in_bytes = sizeof(double) * 3 * B + sizeof(int) * B;
  const size_t out_bytes = (size_t)B * (1 + sizeof(int) + sizeof(double) * 3 * np + sizeof(long long) * np + np +
                                        sizeof(double) * np);
  char* pin = (char*)mp_pinned(ctx, in_bytes + out_bytes + 64);
  if (!pin) return mp_fail(ctx, MP_ERR_NOMEM, "pinned staging allocation failed");
  double* h_node = (double*)pin;
  int* h_so = (int*)(pin + sizeof(double) * 3 * B);
  char* q = pin + in_bytes;
  unsigned char* h_ok = (unsigned char*)q; q += B;
  int* h_len = (int*)q; q += sizeof(int) * B;
  double* h_nb = (double*)q; q += sizeof(double) * 3 * np * B;
  long long* h_idx = (long long*)q; q += sizeof(long long) * np * B;
  unsigned char* h_fr = (unsigned char*)q; q += (size_t)np * B;
  double* h_h = (double*)q;

  // per-scene search state (planHybridAstar!, hybrid_astar_utils.jl:235-296)
  std::vector<std::vector<HNode>> nodes(B);
  std::vector<std::unordered_map<long long, int>> dict(B);
  std::vector<std::vector<int>> open(B);
  std::vector<int> done(B, 0), cur(B, -1), loop(B, 0);
  std::vector<long long> start_index(B);
  for (int b = 0; b < B; b++) {
    found[b] = 0;
    n_states[b] = 0;
    rs_len[b] = 0;
    for (int i = 0; i < mp; i++) pop_seq[(size_t)b * mp + i] = -1;
    // starting node (setup.jl:112-121): Encode of the regulated start
    const double* s0 = start + 3 * b;
    const double* sbd = p->stbound;
    double x = std::fmax(std::fmin(s0[0], sbd[1]), sbd[0]), y = std::fmax(std::fmin(s0[1], sbd[3]), sbd[2]);
    double psi = std::fmax(std::fmin(mpj_modpi(s0[2]), sbd[5]), sbd[4]);
    const double xid = mpj_round((x - sbd[0]) / p->res[0]) + 1, yid = mpj_round((y - sbd[2]) / p->res[1]) + 1;
    const double pid = mpj_round((psi - sbd[4]) / p->res[2]) + 1;
    const double ynum = mpj_round((sbd[3] - sbd[2]) / p->res[1]) + 1, pnum = mpj_round((sbd[5] - sbd[4]) / p->res[2]) + 1;
    long long si = (long long)((xid - 1) * ynum * pnum + (yid - 1) * pnum + pid);
    if (s0[0] < sbd[0] || s0[0] > sbd[1] || s0[1] < sbd[2] || s0[1] > sbd[3]) si = 0;
    start_index[b] = si;
    nodes[b].push_back(HNode{-1, {s0[0], s0[1], s0[2]}, si, 0, 0, 0});
    dict[b][si] = 0;
    open[b].push_back(0);
  }
  auto less_f = [](const std::vector<HNode>& nd) {
    return [&nd](int a, int c) { return (bool)mpj_isless(nd[a].f, nd[c].f); };
  };
  std::vector<int> act;
  for (;;) {
    act.clear();
    for (int b = 0; b < B; b++) {
      if (done[b]) continue;
      if (open[b].empty() || loop[b] >= mp) { done[b] = 1; continue; }
      loop[b]++;
      std::stable_sort(open[b].begin(), open[b].end(), less_f(nodes[b]));
      cur[b] = open[b].front();
      open[b].erase(open[b].begin());
      pop_seq[(size_t)b * mp + loop[b] - 1] = nodes[b][cur[b]].index;
      const int slot = (int)act.size();
      act.push_back(b);
      for (int r = 0; r < 3; r++) h_node[3 * b + r] = nodes[b][cur[b]].st[r];
      h_so[slot] = b;
    }
    if (act.empty()) break;
    const int na = (int)act.size();
    MP_HIP(ctx, hipMemcpyAsync(dnode, h_node, sizeof(double) * 3 * B, hipMemcpyHostToDevice, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(dso, h_so, sizeof(int) * na, hipMemcpyHostToDevice, ctx->stream));
    A.n_active = na;
    if ((st = launch_iter(ctx, D, A))) return st;
    MP_HIP(ctx, hipMemcpyAsync(h_ok, A.rs_ok, B, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(h_len, A.rs_len, sizeof(int) * B, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(h_nb, A.nb, sizeof(double) * 3 * np * B, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(h_idx, A.idx, sizeof(long long) * np * B, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(h_fr, A.fr, (size_t)np * B, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipMemcpyAsync(h_h, A.h, sizeof(double) * np * B, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int b : act) {
      std::vector<HNode>& nd = nodes[b];
      if (h_ok[b]) {  // termination (:259-271)
        found[b] = 1;
        done[b] = 1;
        rs_len[b] = h_len[b];
        MP_HIP(ctx, hipMemcpy(rs_path + (size_t)b * MAXPATH * 3, A.rs_path + (size_t)b * MAXPATH * 3,
                              sizeof(double) * 3 * h_len[b], hipMemcpyDeviceToHost));
        int c = cur[b], ns = 0;
        double* so = states_out + (size_t)b * mp * 3;
        for (int r = 0; r < 3; r++) so[3 * ns + r] = nd[c].st[r];
        ns++;
        while (nd[c].parent >= 0 && nd[c].index != start_index[b] && ns < mp) {
          c = dict[b][nd[c].parent];
          for (int r = 0; r < 3; r++) so[3 * ns + r] = nd[c].st[r];
          ns++;
        }
        n_states[b] = ns;
        continue;
      }
      // FindNewNode bookkeeping (:418-446), neighbours in order
      const HNode cn = nd[cur[b]];
      for (int k = 0; k < np; k++) {
        const size_t o = (size_t)b * np + k;
        if (h_idx[o] == 0 || !h_fr[o]) continue;
        const double tg = cn.g + p->expand_time;
        double th = std::fmax(h_h[o], 0.0);
        if (h_h[o] != h_h[o]) th = h_h[o];
        const double tf = tg + th;
        auto it = dict[b].find(h_idx[o]);
        int id;
        bool upd = false;
        if (it != dict[b].end()) {
          id = it->second;
          if (tg < nd[id].g) {
            nd[id].g = tg; nd[id].h = th; nd[id].f = tf; nd[id].parent = cn.index;
            upd = true;
          }
        } else {
          id = (int)nd.size();
          nd.push_back(HNode{cn.index, {h_nb[3 * o], h_nb[3 * o + 1], h_nb[3 * o + 2]}, h_idx[o], tg, th, tf});
          dict[b][h_idx[o]] = id;
          upd = true;
        }
        if (upd) {
          bool in = false;
          for (int qd : open[b])
            if (nd[qd].index == nd[id].index) { in = true; break; }
          if (!in) open[b].push_back(id);
        }
      }
    }
  }
  for (int b = 0; b < B; b++) {
    pops[b] = loop[b];
    n_nodes[b] = (int)nodes[b].size();
  }
  return MP_OK;
}

}  // extern "C"
