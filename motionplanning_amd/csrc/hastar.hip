// hastar.hip — Hybrid A* hot path for gfx950 (PathPlanning/HybridAstar/src/hybrid_astar_utils.jl,
// ReedsSheppsCurves/src/ReedsSheppsUtils.jl, CollisionDetection/src/utils.jl) + C-ABI.
//
// ha_iter_kernel: one launch per search iteration for B scenes in lockstep.
//   block (s, 0)      RS_connected(node_s): the 48 Reeds–Shepp candidates on 48 lanes,
//                     Julia-argmin across the wave, the optimal command's 100-steps-per-
//                     segment Euler path (heading recurrence and x/y running sums on one
//                     lane, trigonometry on all lanes), then the SAT sweep of its poses.
//   block (s, 1+g)    FindNewNode for neighbours 16g..16g+15: transform + regulate + Encode
//                     on 16 lanes, the (neighbour, pose) SAT collision sweep across all
//                     lanes, then the 48-candidate rs_heuristic of all 16 neighbours at once
//                     (lanes 4j..4j+3 = the four variants of neighbour j, word loop uniform).
// ha_book_kernel: the open list / Dict bookkeeping of planHybridAstar! and the next pop, on the
// device (mp_ha_plan enqueues the whole search without host round trips).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

// the libm routines run under divergent control flow here (per-lane early returns, partial
// pose loops): lane-safe variants, no wave-level ballots inside them
#define MPJ_LANE_SAFE 1
#include "../../include/mp_jlmath.h"
#include "runtime.hpp"

namespace {

constexpr int MAXW = 16;    // walls per scene held in LDS
constexpr int MAXPATH = 501;
constexpr int NBG = 16;     // neighbours per expansion block (4 lanes = 4 RS variants each)
#define PI2 (MPJ_PI / 2)
#ifdef HA_DEBUG
// phase markers to host-mapped memory (tools/ha_dbg.cpp polls them while the kernel runs)
__device__ int* g_ha_dbg;
#define HMARK(ph) __hip_atomic_store(g_ha_dbg + (blockIdx.x * 64 + threadIdx.x), (ph), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
// phase timestamps (s_memtime) of block b at [b][16] after the 64x64 marker area
#define HTIME(i)                                                                                   \
  do {                                                                                             \
    if (threadIdx.x == 0)                                                                          \
      reinterpret_cast<unsigned long long*>(g_ha_dbg + 64 * 64)[blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// bookkeeping-kernel stamps of scene b at [b][16] after the iteration kernel's 4096 blocks, at
// iteration HA_DBG_IT
#ifndef HA_DBG_IT
#define HA_DBG_IT 20
#endif
#define BTIME(i)                                                                                   \
  do {                                                                                             \
    if (threadIdx.x == 0 && it == HA_DBG_IT)                                                       \
      reinterpret_cast<unsigned long long*>(g_ha_dbg + 64 * 64)[(4096 + b) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define HMARK(ph)
#define HTIME(i)
#define BTIME(i)
#endif

struct HaDev {
  double L2, W2, minR, expand_time;
  double res[3];
  double sb[6];
  int n_walls, n_prim, n_col;
  int cull;  // the SAT culls' rounding margins are proven for this call's coordinates (ha_cull_ok); else full SAT
};

// ------------------------------------------------------------ Reeds–Shepp
__device__ __forceinline__ void polar(double a, double b, double* r, double* th) {
  *r = mpj_sqrt(a * a + b * b);
  *th = mpj_atan2_bl(b, a);
}

struct Cmd {
  int n;
  double tr[5], ge[5], st[5];
};

// The two polar forms every RS word starts from (ReedsSheppsUtils.jl path1..12):
// A = polar(x - sin p, y - 1 + cos p), B = polar(x + sin p, y - 1 - cos p).  Computed once
// per candidate variant instead of once per word (same operands, same bits).
struct RsPre {
  double p, rA, tA, rB, tB;
};
__device__ __forceinline__ RsPre rs_pre(const double* q) {
  double sp, cp;
  mpj_sincos_bl(q[2], &sp, &cp);
  RsPre R;
  R.p = q[2];
  polar(q[0] - sp, q[1] - 1 + cp, &R.rA, &R.tA);
  polar(q[0] + sp, q[1] - 1 - cp, &R.rB, &R.tB);
  return R;
}

__device__ __forceinline__ double fin(double t, double u, double v, double cost) {
  if ((t < 0) || (v < 0) || (u < 0)) return __builtin_inf();
  return cost;
}

// Reeds–Shepp words path1..path12 (ReedsSheppsUtils.jl:48-380): rs_word below.

// One Reeds–Shepp word w (wave-uniform) as ONE straight-line program: each transcendental
// (sqrt, acos, sin, asin, atan2) and the three modπ appear once, guarded by uniform branches
// on w, with word-selected operands — the same operations on the same operands as the
// reference words and oracle/or_hastar.c rs_path (bit-identical), but one copy of the code
// instead of twelve inlined word bodies (which overflowed the instruction cache).
__constant__ signed char kRsGe[12][5] = {{1, 1, 1}, {1, 1, 1}, {1, -1, 1}, {1, -1, -1}, {1, 1, -1},
                                         {1, 1, -1, -1}, {1, -1, -1, 1}, {1, -1, -1, -1}, {1, 1, 1, -1},
                                         {1, -1, -1, -1}, {1, 1, 1, -1}, {1, -1, -1, -1, 1}};
__constant__ signed char kRsSt[12][5] = {{1, 0, 1}, {1, 0, -1}, {1, -1, 1}, {1, -1, 1}, {1, -1, 1},
                                         {1, -1, 1, -1}, {1, -1, 1, -1}, {1, -1, 0, 1}, {1, 0, -1, 1},
                                         {1, -1, 0, -1}, {1, 0, 1, -1}, {1, -1, 0, 1, -1}};
// command lengths as: 0 t, 1 u, 2 v, 3 π/2
__constant__ signed char kRsTr[12][5] = {{0, 1, 2}, {0, 1, 2}, {0, 1, 2}, {0, 1, 2}, {0, 1, 2},
                                         {0, 1, 1, 2}, {0, 1, 1, 2}, {0, 3, 1, 2}, {0, 1, 3, 2},
                                         {0, 3, 1, 2}, {0, 1, 3, 2}, {0, 3, 1, 3, 2}};
__constant__ signed char kRsN[12] = {3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 5};

// (A/B) HA_RS_NOINLINE=1: one out-of-line copy of rs_word instead of one per call site (the step
// kernel's instruction footprint)
#ifndef HA_RS_NOINLINE
#define HA_RS_NOINLINE 0
#endif
#if HA_RS_NOINLINE
#define RS_WORD_ATTR __attribute__((noinline))
#else
#define RS_WORD_ATTR __forceinline__
#endif
__device__ RS_WORD_ATTR double rs_word(int w_, const RsPre& R, Cmd* c, double* tuv = nullptr) {
  const int w = __builtin_amdgcn_readfirstlane(w_);  // wave-uniform word: scalar branches and table loads
  const double p = R.p;
  const bool useA = (w == 1) | (w == 3) | (w == 4) | (w == 5) | (w == 8) | (w == 9);
  const double rho = useA ? R.rA : R.rB, th = useA ? R.tA : R.tB;
  const double r2 = rho * rho;
  double sq = 0.0, ang = 0.0, ac = 0.0;
  if (w == 2 || w == 8 || w == 9 || w == 12) sq = mpj_sqrt(r2 - 4);
  double u;  // words 1, 2, 8-12: direct; 3-7: below
  if (w == 1) u = rho;
  else if (w == 2) u = sq;
  else if (w == 8 || w == 9) u = sq - 2;
  else if (w == 10 || w == 11) u = rho - 2;
  else if (w == 12) u = sq - 4;
  else u = 0.0;
  const double u1 = (20 - r2) / 16;
  if (w >= 3 && w <= 7) {
    double arg;
    if (w <= 4) arg = rho / 4;
    else if (w == 5) arg = 1 - r2 / 8;
    else if (w == 6) arg = rho <= 2 ? (rho + 2) / 4 : (rho - 2) / 4;
    else arg = u1;
    ac = mpj_acos(arg);
  }
  if (w == 5 || w == 7) {
    u = ac;
    ang = mpj_asin(2 * mpj_sin(u) / rho);
  } else if (w == 2 || w == 8 || w == 9 || w == 12) {
    double y, x;
    if (w == 2) { y = 2; x = u; }
    else if (w == 8) { y = 2; x = u + 2; }
    else if (w == 9) { y = u + 2; x = 2; }
    else { y = 2; x = u + 4; }
    ang = mpj_atan2_bl(y, x);
  } else if (w >= 3 && w <= 6) {
    ang = ac;
  }
  // t = modπ(targ)   (word 1: t = θ, and modπ(θ) == θ for θ = atan2(...) ∈ [-π, π])
  double targ;
  if (w == 1 || w == 11) targ = th;
  else if (w == 2) targ = th + ang;
  else if (w == 10) targ = th + PI2;
  else if (w == 5 || w == 9 || (w == 6 && !(rho <= 2))) targ = th + PI2 - ang;
  else targ = th + PI2 + ang;
  const double t = mpj_modpi_bl(targ);
  if (w == 3 || w == 4 || w == 6) {  // u = modπ(π - 2a) / modπ(a) / modπ(π - a)
    const double uarg = (w == 6) ? (rho <= 2 ? ang : MPJ_PI - ang) : MPJ_PI - 2 * ang;
    u = mpj_modpi_bl(uarg);
  }
  double varg;
  if (w == 1 || w == 10 || w == 11) varg = (w == 1) ? p - t : p - t - PI2;
  else if (w == 2 || w == 7 || w == 12) varg = t - p;
  else if (w == 3) varg = p - t - u;
  else if (w == 4) varg = t + u - p;
  else if (w == 5) varg = t - p - u;
  else if (w == 6) varg = p - t + 2 * u;
  else if (w == 8) varg = t - p + PI2;
  else varg = t - p - PI2;  // w == 9
  const double v = mpj_modpi_bl(varg);
  const double at = __builtin_fabs(t), au = __builtin_fabs(u), av = __builtin_fabs(v);
  double cost;
  if (w <= 5) cost = at + au + av;
  else if (w <= 7) cost = at + 2 * au + av;
  else if (w == 8) cost = at + PI2 + au + av;
  else if (w <= 11) cost = at + au + PI2 + av;
  else cost = at + PI2 + au + PI2 + av;
  bool valid;
  if (w == 1) valid = true;
  else if (w == 2 || (w >= 8 && w <= 11)) valid = rho >= 2;
  else if (w <= 6) valid = rho <= 4;
  else if (w == 7) valid = (rho <= 6) && (0 <= u1) && (u1 <= 1);
  else valid = rho >= 4;
  if (tuv) {  // the word's segment lengths: with (w, variant) they determine its commands (cmd_from_tuv)
    tuv[0] = t;
    tuv[1] = u;
    tuv[2] = v;
  }
  if (c) {
    const int wi = w - 1;
    c->n = kRsN[wi];
#pragma unroll
    for (int r = 0; r < 5; r++) {
      const int code = kRsTr[wi][r];
      c->tr[r] = code == 0 ? t : code == 1 ? u : code == 2 ? v : PI2;
      c->ge[r] = kRsGe[wi][r];
      c->st[r] = kRsSt[wi][r];
    }
  }
  return valid ? fin(t, u, v, cost) : __builtin_inf();
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

// changeBasis with sin/cos of init's heading given (the lattice-heading tables)
__device__ __forceinline__ void change_basis_sc(const double* init, const double* term, double minR, double s0,
                                                double c0, double* out) {
  const double p0 = init[2], pg = term[2];
  const double dx = (term[0] - init[0]) / minR, dy = (term[1] - init[1]) / minR;
  out[0] = dx * c0 + dy * s0;
  out[1] = -dx * s0 + dy * c0;
  out[2] = pg - p0;
}
__device__ __forceinline__ void change_basis(const double* init, const double* term, double minR, double* out) {
  const double p0 = init[2], pg = term[2];
  const double dx = (term[0] - init[0]) / minR, dy = (term[1] - init[1]) / minR;
  double s0, c0;
  mpj_sincos_bl(p0, &s0, &c0);
  out[0] = dx * c0 + dy * s0;
  out[1] = -dx * s0 + dy * c0;
  out[2] = pg - p0;
}

// ------------------------------------------------------------- collision
// The reference's two BLAS-dispatched products here round as Julia's OpenBLAS does (oracle/or_blas.h):
// GetRectanglePts' R*pts is dgemm (2x2 * 2x5, K = 2: fma(a1, b1, a0*b0)) and SAT's
// transpose(pts .- bg_pt)*normal_vec is dgemv 'T' on two rows (fma(m0, n0, m1*n1)).
__device__ __forceinline__ double sat_dp(double mx, double my, double nx, double ny) {
  return __builtin_fma(mx, nx, my * ny);
}
__device__ __forceinline__ void rect_pts(double ox, double oy, double c, double s, double l, double w, double* pts) {
  const double px[5] = {-l, -l, l, l, -l}, py[5] = {w, -w, -w, w, w};
#pragma unroll
  for (int j = 0; j < 5; j++) {
    pts[2 * j] = __builtin_fma(-s, py[j], c * px[j]) + ox;
    pts[2 * j + 1] = __builtin_fma(c, py[j], s * px[j]) + oy;
  }
}

// SeparatingAxisTheorem (CollisionDetection/src/utils.jl:37-62).  The fifth point of each
// polygon repeats the first, so projecting 4 points gives the same min/max.
__device__ __forceinline__ int sat(const double* base, const double* other) {
  for (int e = 0; e < 4; e++) {
    const double bx = base[2 * e], by = base[2 * e + 1];
    const double vx = base[2 * e + 2] - bx, vy = base[2 * e + 3] - by;
    const double nx = -vy, ny = vx;
    double mnb = 0, mxb = 0, mno = 0, mxo = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const double db = sat_dp(base[2 * j] - bx, base[2 * j + 1] - by, nx, ny);
      const double dq = sat_dp(other[2 * j] - bx, other[2 * j + 1] - by, nx, ny);
      if (j == 0 || db < mnb) mnb = db;
      if (j == 0 || db > mxb) mxb = db;
      if (j == 0 || dq < mno) mno = dq;
      if (j == 0 || dq > mxo) mxo = dq;
    }
    if ((mxo <= mnb) || (mxb <= mno)) return 1;
  }
  return 0;
}

// SAT with a wall as the base polygon, its pose-independent part precomputed once per block:
// per edge [bx, by, nx, ny, min, max] of the wall's own projections (same operations).
__device__ __forceinline__ void sat_base_pre(const double* base, double* pre /* [4][6] */) {
  for (int e = 0; e < 4; e++) {
    const double bx = base[2 * e], by = base[2 * e + 1];
    const double vx = base[2 * e + 2] - bx, vy = base[2 * e + 3] - by;
    const double nx = -vy, ny = vx;
    double mnb = 0, mxb = 0;
    for (int j = 0; j < 4; j++) {
      const double db = sat_dp(base[2 * j] - bx, base[2 * j + 1] - by, nx, ny);
      if (j == 0 || db < mnb) mnb = db;
      if (j == 0 || db > mxb) mxb = db;
    }
    double* o = pre + 6 * e;
    o[0] = bx; o[1] = by; o[2] = nx; o[3] = ny; o[4] = mnb; o[5] = mxb;
  }
}
__device__ __forceinline__ int sat_pre(const double* pre, const double* other) {
  for (int e = 0; e < 4; e++) {
    const double* o = pre + 6 * e;
    const double bx = o[0], by = o[1], nx = o[2], ny = o[3], mnb = o[4], mxb = o[5];
    double mno = 0, mxo = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const double dq = sat_dp(other[2 * j] - bx, other[2 * j + 1] - by, nx, ny);
      if (j == 0 || dq < mno) mno = dq;
      if (j == 0 || dq > mxo) mxo = dq;
    }
    if ((mxo <= mnb) || (mxb <= mno)) return 1;
  }
  return 0;
}

// Wall table row: corners (10) + wall-side SAT table (24) + [center x, center y, far²] (3) + cull bounds (3).
// far² = (√2 (r_vehicle + r_wall) + 1e-6)², r = a rectangle's circumradius.  When the vehicle's
// centre is farther than that from a wall's centre, ConvexCollision(wall, vehicle) is false for
// certain: each rectangle has an edge normal within 45° of the centre-to-centre direction d, along
// which the centres are >= |d|/√2 apart while each rectangle projects within its circumradius of
// its centre, so BOTH SeparatingAxisTheorem calls find a separating axis -- with a gap of >= 1e-6 m
// against rounding errors below 1e-12 m at these coordinates.  Such walls skip their SAT pair
// (the booleans, hence every planner decision, are unchanged; tests/test_oracle_hastar.py checks
// the bound against the oracle's SAT).
// round 4: + the per-direction cull bounds (3) of wall_cull, so a row is 40 doubles
constexpr int WT = 40;
// The culls' margin argument (1e-6 m, and 1e-6·|n| along an edge normal n) against the rounding of the
// computed projections: a projection fl((p - b)·n) of a computed corner p (|p|, |b| <= X, corner rounding
// <= 3ε(X + L)) is within ~15ε(X + L)·|n| of the exact one (the FMA forms above round once less per term).  ha_cull_ok enables the culls only when every
// input coordinate and length of the call (wall centres + extents, stbound, start, goal, minR, vehicle and
// primitive sizes) is <= HA_CULL_MAX = 1e6 m; every swept pose then lies within ~10 HA_CULL_MAX of the
// origin (a neighbour within expand_time of an in-bounds node, a Reeds-Shepp path within its length of
// the popped node), so the rounding is <= 15·1.1e-16·1e7·|n| = 1.7e-8·|n|, 60x below the margin.  Beyond
// it the culls are off (far² and the cull bounds +inf) and every SAT call runs, as the reference does.
constexpr double HA_CULL_MAX = 1e6;
// MAXW walls at 2 bits each in pose_free's 32-bit `need` mask
static_assert(2 * MAXW <= 32, "pose_free's need mask holds 2 bits per wall");
__device__ __forceinline__ double wall_far2(const HaDev& P, const double* wl) {
  if (!P.cull) return __builtin_inf();  // never "far": every wall's SAT pair runs
  const double rv = mpj_sqrt(P.L2 * P.L2 + P.W2 * P.W2), rw = mpj_sqrt(wl[3] * wl[3] + wl[4] * wl[4]);
  const double f = 1.4142135623730951 * (rv + rw) * (1 + 1e-12) + 1e-6;
  return f * f;
}

// Per-direction SAT cull, one wall (corners wp, SAT table pre, centre c) -> cl[3]:
//  cl[0], cl[1] = (r_vehicle + 1e-6)·|n_e|·(1 + 1e-12) for the wall's edges e = 0, 1 (n_e = the edge
//    normal of the wall-side SAT table): when the vehicle centre's projection on n_e lies more than
//    cl[e] beyond the wall's own projection interval [mnb, mxb], the vehicle's circumcircle -- hence
//    every vehicle corner -- is past the wall along that axis by >= 1e-6·|n_e|, so
//    SeparatingAxisTheorem(wall, vehicle) returns true (errors of the computed projections are
//    ~1e-13·|n_e| at these coordinates);
//  cl[2] = r_wall·(1 + 1e-12) + 1e-6 (r_wall = the largest corner-to-centre distance): when the wall
//    centre lies farther than L2 + cl[2] along the vehicle's heading or W2 + cl[2] across it, every wall
//    corner is past the vehicle's edge along that edge normal, so SeparatingAxisTheorem(vehicle, wall)
//    returns true.
// The booleans are the reference's either way (tests/test_oracle_hastar.py checks both bounds against
// the oracle's SAT); the cull only skips SAT calls whose result is certain.
__device__ __forceinline__ void wall_cull(const HaDev& P, const double* wp, const double* pre, const double* c,
                                          double* cl) {
  if (!P.cull) {  // no bound is certain: every SAT call runs
    cl[0] = cl[1] = cl[2] = __builtin_inf();
    return;
  }
  const double rv = mpj_sqrt(P.L2 * P.L2 + P.W2 * P.W2);
  for (int e = 0; e < 2; e++) {
    const double nx = pre[6 * e + 2], ny = pre[6 * e + 3];
    cl[e] = (rv + 1e-6) * mpj_sqrt(nx * nx + ny * ny) * (1 + 1e-12);
  }
  double r2 = 0;
  for (int j = 0; j < 4; j++) {
    const double dx = wp[2 * j] - c[0], dy = wp[2 * j + 1] - c[1];
    r2 = fmax(r2, dx * dx + dy * dy);
  }
  cl[2] = mpj_sqrt(r2) * (1 + 1e-12) + 1e-6;
}
// (A/B) -DHA_SAT_OVERLAP=1 enables class 2 below (proved in the oracle test; not yet measured on the GPU)
#ifndef HA_SAT_OVERLAP
#define HA_SAT_OVERLAP 0
#endif
// Wall-side class of a vehicle centred at (x, y), from its projections on the wall's edge normals 0, 1:
//  1: SAT(wall, vehicle) is certainly true (wall_cull's cl[0..1]);
//  2: the centre lies inside the wall, at least 1e-5 of the wall's extent from each side along both
//     normals: the centre is then interior to both rectangles by far more than any rounding error, so
//     on every axis the two projections overlap and both SeparatingAxisTheorem calls return false --
//     the pose collides (tests/test_oracle_hastar.py);
//  0: neither is certain.
__device__ __forceinline__ int wall_side_class(const double* pre, const double* cl, double x, double y) {
  const double d0 = (x - pre[0]) * pre[2] + (y - pre[1]) * pre[3];
  const double d1 = (x - pre[6]) * pre[8] + (y - pre[7]) * pre[9];
  if ((d0 - cl[0] > pre[5]) | (d0 + cl[0] < pre[4]) | (d1 - cl[1] > pre[11]) | (d1 + cl[1] < pre[10])) return 1;
  if (!HA_SAT_OVERLAP) return 0;
  const double m0 = (pre[5] - pre[4]) * 1e-5, m1 = (pre[11] - pre[10]) * 1e-5;
  return ((d0 > pre[4] + m0) & (d0 < pre[5] - m0) & (d1 > pre[10] + m1) & (d1 < pre[11] - m1)) ? 2 : 0;
}
// 1: SAT(vehicle, wall) is certainly true; (dx, dy) = vehicle centre - wall centre, (cy, sy) the
// vehicle rectangle's heading (wall_cull's cl[2])
__device__ __forceinline__ int cull_vehicle_side(const HaDev& P, const double* cl, double dx, double dy, double cy,
                                                 double sy) {
  const double u = dx * cy + dy * sy, v = dy * cy - dx * sy;
  return (__builtin_fabs(u) > P.L2 * (1 + 1e-12) + cl[2]) | (__builtin_fabs(v) > P.W2 * (1 + 1e-12) + cl[2]);
}

// The heading-only part of a pose's collision check: sin/cos of ψ (the centre offset) and of the
// rectangle's yaw modπ(ψ) (its own sin/cos only when it differs; when yaw == ψ bit for bit the two pairs
// are the same numbers).  A function of ψ alone, so the neighbour sweeps read it from a per-plan table
// (ha_pose_table_kernel) when the expanded node's heading is a lattice heading.
struct PoseTrig {
  double sq, cq, sy, cy;
};
__device__ __forceinline__ PoseTrig pose_trig(double psi) {
  PoseTrig t;
  mpj_sincos_bl(psi, &t.sq, &t.cq);
  const double yaw = mpj_modpi_bl(psi);
  t.sy = t.sq;
  t.cy = t.cq;
  if (MPJ_ANY(yaw != psi)) mpj_sincos_bl(yaw, &t.sy, &t.cy);  // |ψ| > π: the wrapped yaw's own sin/cos
  return t;
}

// vehicle pose q=[x,y,ψ] (rear axle) with its heading terms T against all walls (corners wp, SAT tables
// wpre, centres / far² wc and cull bounds wcl in LDS); 1 = free
__device__ __forceinline__ int pose_free_t(const HaDev& P, const double* q, const PoseTrig& T, const double* wp,
                                           const double* wpre, const double* wc, const double* wcl, int nw) {
  const double sq = T.sq, cq = T.cq, sy = T.sy, cy = T.cy;
  const double x = q[0] + P.L2 * cq, y = q[1] + P.L2 * sq;
  // the SAT calls whose result is not certain (bit 2i: SAT(wall i, vehicle), bit 2i+1: SAT(vehicle,
  // wall i)), collected before the rectangle is built so its corners are live only where needed
  unsigned need = 0;
  for (int i = 0; i < nw; i++) {
    const double dx = x - wc[3 * i], dy = y - wc[3 * i + 1];
    if (dx * dx + dy * dy > wc[3 * i + 2]) continue;  // far from this wall: separated for certain
    const int ws = wall_side_class(wpre + 24 * i, wcl + 3 * i, x, y);
#if HA_SAT_OVERLAP
    if (ws == 2) return 0;  // centre inside the wall: collides for certain
#endif
    need |= (unsigned)(ws != 1) << (2 * i);
    need |= (unsigned)!cull_vehicle_side(P, wcl + 3 * i, dx, dy, cy, sy) << (2 * i + 1);
  }
  if (!need) return 1;
  double vp[10];
  rect_pts(x, y, cy, sy, P.L2, P.W2, vp);
  for (int i = 0; i < nw; i++) {
    if (((need >> (2 * i)) & 1) && !sat_pre(wpre + 24 * i, vp)) return 0;
    if (((need >> (2 * i)) & 2) && !sat(vp, wp + 10 * i)) return 0;
  }
  return 1;
}
__device__ __forceinline__ int pose_free(const HaDev& P, const double* q, const double* wp, const double* wpre,
                                         const double* wc, const double* wcl, int nw) {
  return pose_free_t(P, q, pose_trig(q[2]), wp, wpre, wc, wcl, nw);
}

// one (wall, direction) term of pose_free: d = 0 SAT(wall, vehicle), d = 1 SAT(vehicle, wall); the pose
// is free iff every term of every wall is 1 (ConvexCollision = SAT(wall, veh) && SAT(veh, wall))
__device__ __forceinline__ int pose_free_part(const HaDev& P, const double* q, const double* wp, const double* wpre,
                                              const double* wc, const double* wcl, int w, int d) {
  double sq, cq;
  mpj_sincos_bl(q[2], &sq, &cq);
  const double x = q[0] + P.L2 * cq, y = q[1] + P.L2 * sq;
  const double fx = x - wc[3 * w], fy = y - wc[3 * w + 1];
  if (fx * fx + fy * fy > wc[3 * w + 2]) return 1;  // far from this wall: separated for certain
#if HA_SAT_OVERLAP
  const int ws = wall_side_class(wpre + 24 * w, wcl + 3 * w, x, y);
  if (ws == 2) return 0;  // centre inside the wall: both terms are false
  if (d == 0 && ws == 1) return 1;
#else
  if (d == 0 && wall_side_class(wpre + 24 * w, wcl + 3 * w, x, y) == 1) return 1;
#endif
  const double yaw = mpj_modpi_bl(q[2]);
  double sy = sq, cy = cq;
  if (MPJ_ANY(yaw != q[2])) mpj_sincos_bl(yaw, &sy, &cy);
  if (d == 1 && cull_vehicle_side(P, wcl + 3 * w, fx, fy, cy, sy)) return 1;
  double vp[10];
  rect_pts(x, y, cy, sy, P.L2, P.W2, vp);
  return d == 0 ? sat_pre(wpre + 24 * w, vp) : sat(vp, wp + 10 * w);
}
// the same term with the heading terms given (the pose table)
__device__ __forceinline__ int pose_free_part_t(const HaDev& P, const double* q, const PoseTrig& T, const double* wp,
                                                const double* wpre, const double* wc, const double* wcl, int w, int d) {
  const double x = q[0] + P.L2 * T.cq, y = q[1] + P.L2 * T.sq;
  const double fx = x - wc[3 * w], fy = y - wc[3 * w + 1];
  if (fx * fx + fy * fy > wc[3 * w + 2]) return 1;
#if HA_SAT_OVERLAP
  const int ws = wall_side_class(wpre + 24 * w, wcl + 3 * w, x, y);
  if (ws == 2) return 0;
  if (d == 0 && ws == 1) return 1;
#else
  if (d == 0 && wall_side_class(wpre + 24 * w, wcl + 3 * w, x, y) == 1) return 1;
#endif
  if (d == 1 && cull_vehicle_side(P, wcl + 3 * w, fx, fy, T.cy, T.sy)) return 1;
  double vp[10];
  rect_pts(x, y, T.cy, T.sy, P.L2, P.W2, vp);
  return d == 0 ? sat_pre(wpre + 24 * w, vp) : sat(vp, wp + 10 * w);
}

// transform (hybrid_astar_utils.jl:459-481) with the node's cos/sin given
__device__ __forceinline__ void transform_cs(const double* node, double c, double s, const double* q, double* o) {
  o[0] = q[0] * c - q[1] * s + node[0];
  o[1] = q[0] * s + q[1] * c + node[1];
  o[2] = q[2] + node[2];
}
__device__ __forceinline__ void transform1(const double* node, const double* q, double* o) {
  double s, c;
  mpj_sincos_bl(node[2], &s, &c);
  transform_cs(node, c, s, q, o);
}

__device__ __forceinline__ void regulate(const HaDev& P, const double* s, double* o) {
  o[0] = mpj_round(s[0] / P.res[0]) * P.res[0];
  o[1] = mpj_round(s[1] / P.res[1]) * P.res[1];
  const double psi = mpj_modpi_bl(s[2]);
  o[2] = mpj_round(psi / P.res[2]) * P.res[2];
}

// Encode's heading index (hybrid_astar_utils.jl:316-350): a function of the heading alone
__device__ __forceinline__ double encode_pid(const HaDev& P, double h) {
  const double* b = P.sb;
  double psi = mpj_modpi_bl(h);
  psi = __builtin_fmax(__builtin_fmin(psi, b[5]), b[4]);
  return mpj_round((psi - b[4]) / P.res[2]) + 1;
}
// Encode with the heading index given
__device__ __forceinline__ long long encode_p(const HaDev& P, const double* s, double pid) {
  const double* b = P.sb;
  double x = s[0], y = s[1];
  x = __builtin_fmax(__builtin_fmin(x, b[1]), b[0]);
  y = __builtin_fmax(__builtin_fmin(y, b[3]), b[2]);
  const double xid = mpj_round((x - b[0]) / P.res[0]) + 1;
  const double yid = mpj_round((y - b[2]) / P.res[1]) + 1;
  const double ynum = mpj_round((b[3] - b[2]) / P.res[1]) + 1;
  const double pnum = mpj_round((b[5] - b[4]) / P.res[2]) + 1;
  const double idx = (xid - 1) * ynum * pnum + (yid - 1) * pnum + pid;
  if (s[0] < b[0] || s[0] > b[1] || s[1] < b[2] || s[1] > b[3]) return 0;
  return (long long)idx;
}
__device__ __forceinline__ long long encode(const HaDev& P, const double* s) {
  return encode_p(P, s, encode_pid(P, s[2]));
}

struct IterArgs {
  const double* node;    // [B][3]
  const double* goal;    // [B][3]
  const double* walls;   // [B][nw][5]
  const double* sc;      // [n_prim][3]
  const double* pc;      // [n_prim][n_col][3]
  const int* scene_of;   // active slot -> scene index (nullptr: slot = scene)
  const int* active;     // per-scene live flag (device-resident search), nullptr = all
  const double* wtab;    // [B][nw][WT] wall corners (10) + SAT tables (24) + centre, far², nullptr = compute
  const int* n_live;     // device count of the scene_of list (nullptr: n_active)
  int n_active;
  int do_rs, do_exp;
  int rs_path_free_only;  // RS_connected writes its path only when it is collision-free (the planner
                          // reads it only then); the standalone entry point writes every path
  int coherent;           // ha_step_kernel: the per-scene outputs the same launch's bookkeeping reads
                          // (neighbour records, rs_ok / rs_len) are stored agent-coherent (st_ag)
  // the search's Dict (mp_ha_plan; nullptr elsewhere): a neighbour group skips rs_heuristic when no
  // neighbour of it can use the value (its Encode cell already holds a node with g <= the tentative g)
  const int* dnid;        // [B][C] cell -> node id (-1 absent)
  const double* dg;       // [B][C] node g
  const double* cur_g;    // [B] the popped node's g
  int C;
  // MPGPU_HA_STAMPS=1 (diagnostics): s_memrealtime stamps of every block of every STAMP_EVERY-th
  // iteration, [slot][block][6]: entry, body done, role decided, bookkeeping done, finish done, role
  unsigned long long* stamps;
  int stamp_blocks;
  // RS_connected outputs (per scene)
  unsigned char* rs_ok;  // [B]
  double* rs_path;       // [B][501][3]
  int* rs_len;           // [B]
  // FindNewNode outputs (per scene, per neighbour)
  double* nb;            // [B][n_prim][3]
  long long* idx;        // [B][n_prim]
  unsigned char* fr;     // [B][n_prim]
  double* h;             // [B][n_prim]
  // (mp_ha_plan, HA_RS_WINNER) rs_heuristic's winning Reeds-Shepp candidate (0..47) per neighbour, -1 when
  // the group did not evaluate it; and the popped node's stored winner per scene (-1: unknown -> RS_connected
  // runs the full 48-candidate search).  A node's states never change after its creation (FindNewNode's
  // update branch, hybrid_astar_utils.jl:425-430, touches g/h/f/parent only), and RS_connected (:229-230)
  // runs the same changeBasis + allpath on them as rs_heuristic (:365-366) did at the creation, so the
  // stored candidate is RS_connected's argmin and only its word needs evaluating for the commands.
  int* hw;               // [B][n_prim]
  const int* node_rw;    // [B]
  // (tail launches of mp_ha_plan, ha_step_kernel<..., RSH = true>) rs_heuristic per neighbour in four word
  // chunks: the chunk's best (cost, candidate id), [B][n_prim][4]; the bookkeeping combines them
  double* hp_c;
  int* hp_i;
  double* hp_t;          // [B][n_prim][4][3] the chunk winner's (t, u, v) (its RS_connected commands)
  const double* node_tuv;  // [B][3] the popped node's stored (t, u, v) when node_rw has RW_TUV
  // (mp_ha_plan) the pose table: PoseTrig of every swept primitive pose (1:5:n_col) for every lattice
  // heading m·res[2], m = pt_mlo .. pt_mlo + pt_nm - 1: [pt_nm][n_prim][pt_nsw][4]; nullptr = compute
  const double* ptab;
  int pt_mlo, pt_nm, pt_nsw;
  // (mp_ha_plan) lattice-heading tables over the same m: htn [pt_nm][2] = sin, cos of m·res[2] (transform's
  // and changeBasis's of the node); htk [pt_nm][n_prim][4] = neighbour k's regulated heading, its sin and cos
  // (changeBasis from the neighbour), Encode's heading index -- the heading-only terms of FindNewNode's
  // transform / regulate_states / Encode (:396-405), nullptr = compute
  const double* htn;
  const double* htk;
  int no_pre;  // (A/B, MPGPU_HA_PRESCAN=0) the prescan block only marks its record stale: the bookkeeping scans
  int rs_last;  // ha_step_kernel dispatches the RS_connected blocks last ((A/B) MPGPU_HA_RS_LAST=0: first)
  int node_ag;  // read the node agent-coherently (written in this launch), once node_flag[s] >= node_flag_min
  // (tail pipe / persistent launches) the node as tagged granules instead: [B][HA_NGR] of {tag, 32-bit value},
  // this parity's, complete once every tag equals ngr_tag (see ha_publish_node)
  const unsigned long long* ngr;
  unsigned ngr_tag;
  int ngr_pub;  // the tail's bookkeeping publishes granules (else the node buffers + a drained flag); (A/B) MPGPU_HA_NGR
  const int* node_flag;
  int node_flag_min;
  int* node_flag_err;  // the wait is bounded: past HA_SPIN_MAX polls it sets *node_flag_err and gives up
  // (full-width ha_pipe_kernel) the popped node's g and the scene's node count before its FindNewNode, published
  // with the node: the Dict pre-check then runs beside FindNewNode's writes (see ha_iter_body)
  const double* node_g;
  const int* node_nn;
  int full_tuv;  // the full-width groups store their winners' (t, u, v) (hp_t chunk 0) and the books flag them
  unsigned long long* mirror;  // (host-coherent) launch it's first block writes (it - 1) << 32 | live(it - 1)
  // [B][n_prim][HA_DREC] (full-width / middle step launches) each neighbour's Dict entry as the group found it:
  // cell's node id, then its g, pos, f, seq, Encode index, rs winner, state -- the bookkeeping reads them with
  // the other records instead of looking them up after them
  long long* drec;
  const int* dpos;
  const double* df;
  const long long* dseq;
  const long long* dindex;
  const int* drw;
  const double* dst;
  int no_tuv;  // (A/B, MPGPU_HA_TUV=0) nodes keep only their winner id: RS_connected evaluates its word
};

// Agent-coherent relaxed stores / loads (global_store / global_load with the sc1 policy: they reach
// and read the device coherence point, past the per-XCD L2).  ha_step_kernel hands per-scene records
// from one block to another inside a launch with these, ordered by s_waitcnt + an arrival ticket,
// so no block needs an agent-scope release fence (an L2 write-back of the whole XCD).
template <class T>
__device__ __forceinline__ void st_ag(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_ag(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_out(bool coh, T* p, T v) {
  if (coh) st_ag(p, v);
  else *p = v;
}

// the lattice-heading index of heading h into the per-plan tables (IterArgs::htn), or -1 when h is not
// m·res[2] bit for bit for a tabulated m (e.g. an unregulated start) -- then every term is computed
__device__ __forceinline__ int lattice_m(const HaDev& P, const IterArgs& A, double h) {
  if (!A.htn) return -1;
  const double m = mpj_round(h / P.res[2]);
  if (__double_as_longlong(m * P.res[2]) == __double_as_longlong(h) && m >= A.pt_mlo && m < A.pt_mlo + A.pt_nm)
    return (int)m - A.pt_mlo;
  return -1;
}
// transform + regulate_states + Encode of neighbour k of `node` (:396-405), the heading terms from the
// lattice tables when tabm >= 0 (the same values: the tables hold what these operations give); if sn, also
// sin / cos of the regulated heading (changeBasis from the neighbour)
__device__ __forceinline__ long long expand_nb(const HaDev& P, const IterArgs& A, const double* node, int tabm, int k,
                                               double* nb, double* sn = nullptr, double* cn = nullptr) {
  double t[3];
  if (tabm >= 0) {
    const double* hn = A.htn + 2 * tabm;
    const double* hk = A.htk + ((size_t)tabm * P.n_prim + k) * 4;
    transform_cs(node, hn[1], hn[0], A.sc + 3 * k, t);
    nb[0] = mpj_round(t[0] / P.res[0]) * P.res[0];
    nb[1] = mpj_round(t[1] / P.res[1]) * P.res[1];
    nb[2] = hk[0];
    if (sn) {
      *sn = hk[1];
      *cn = hk[2];
    }
    return encode_p(P, nb, hk[3]);
  }
  transform1(node, A.sc + 3 * k, t);
  regulate(P, t, nb);
  if (sn) mpj_sincos_bl(nb[2], sn, cn);
  return encode(P, nb);
}

// The live count of the previous iteration (final: written by the previous launch) to the host, packed with
// the iteration, by the launch's first thread (a vector store to fine-grained host memory); mp_ha_plan sizes
// its next launches from it instead of a stream copy every 16 iterations.
__device__ __forceinline__ void ha_mirror(const IterArgs& A, int it) {
  if (A.mirror && A.n_live && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(A.mirror, ((unsigned long long)(it - 1) << 32) | (unsigned)*A.n_live, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int HA_DREC = 10;
// (A/B build -DHA_DREC_CODE=1 + MPGPU_HA_DREC=1) the step launches' groups copy their neighbours' Dict entries
// into the records: bit-exact but 0.3-0.5 ms slower per 256-plan (r05zf: the groups' extra loads / stores and
// registers cost more than the bookkeeping's saved round trip), so compiled out by default
#ifndef HA_DREC_CODE
#define HA_DREC_CODE 0
#endif

// Bounded cross-block wait (ha_pipe_kernel, ha_persist_kernel): poll *p until it is >= v; past HA_SPIN_MAX
// polls (~1 s) set *err and return HA_DONE (every waiter then leaves its loop: a wrong result, not a hang)
constexpr int HA_DONE = 0x3ffffffe;  // a scene's flag once its search ended (even: no next node)
constexpr long long HA_SPIN_MAX = 1LL << 24;
__device__ __forceinline__ int wait_ge(const int* p, int v, int* err) {
  int f = ld_ag(p);
  for (long long n = 0; f < v; n++) {
    if (n >= HA_SPIN_MAX) {
      if (err) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return HA_DONE;
    }
    __builtin_amdgcn_s_sleep(2);
    f = ld_ag(p);
  }
  return f;
}

// The popped node handed to the expansion and RS_connected blocks of the same launch as tagged granules (the
// data IS the flag): 14 one-word {tag = iteration + 1, value} records -- the state's and the stored commands'
// six double halves each, the winner word, the go bit -- each written by ONE agent-scope 8-byte store of its
// own lane, so the bookkeeping neither drains its stores nor raises a separate flag, and a consumer wave polls
// the 14 words until every tag matches (one round trip instead of flag + node).  HA_NGR_DONE in the go word's
// tag: the scene's search ended.  The go word's value: bit 0 go (a node follows), bit 1 skip (the consumer has
// nothing to do this round: the node's expansion was made speculatively, or no runner-up exists; HA_SPEC).
constexpr int HA_NGR = 16;
// granule slots by iteration (it & 7): a slot is rewritten by the bookkeeping seven iterations on -- its consumers
// (the expansion groups, and one of the scene's two RS_connected blocks) take it as soon as it appears and run at
// most a couple of iterations behind; a consumer that found its slot overwritten would wait out its bounded spin
// and fail the plan (Q.err), not read another iteration's node
constexpr int HA_NGR_SLOTS = 8;
constexpr unsigned HA_NGR_DONE = 0xffffffffu;
__device__ __forceinline__ void ha_publish_node(unsigned long long* g, unsigned tag, int lane, const long long* w,
                                                unsigned go) {
  if (lane >= 14) return;
  unsigned v;
  if (lane < 6) v = (unsigned)((unsigned long long)w[3 + (lane >> 1)] >> (32 * (lane & 1)));  // state
  else if (lane < 12) v = (unsigned)((unsigned long long)w[7 + ((lane - 6) >> 1)] >> (32 * (lane & 1)));  // tuv
  else if (lane == 12) v = (unsigned)(int)w[6];  // rs winner word
  else v = go;
  __hip_atomic_store(g + lane, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0 of a consumer block; returns the go word (0: the search ended or the wait ran out; bit 1: skip), the
// node in st / tuv / rw
__device__ __forceinline__ int ha_consume_node(const unsigned long long* g, unsigned tag, int lane, double* st,
                                               double* tuv, int* rw, int* err) {
  unsigned long long x = 0;
  for (long long n = 0;; n++) {
    x = lane < 14 ? __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    const unsigned t = (unsigned)(x >> 32);
    const unsigned tg = __shfl(t, 13);
    if (tg == HA_NGR_DONE) return 0;
    if (__all(lane >= 14 || t == tag)) break;
    if (n >= HA_SPIN_MAX) {
      if (lane == 0 && err) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  const unsigned v = (unsigned)x;
  const int go = (int)__shfl(v, 13);
#pragma unroll
  for (int e = 0; e < 3; e++) {
    const unsigned lo = __shfl(v, 2 * e), hi = __shfl(v, 2 * e + 1);
    const unsigned tlo = __shfl(v, 6 + 2 * e), thi = __shfl(v, 7 + 2 * e);
    if (lane == 0) {
      st[e] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
      tuv[e] = __longlong_as_double((long long)(((unsigned long long)thi << 32) | tlo));
    }
  }
  const int w = (int)__shfl(v, 12);
  if (lane == 0) *rw = w;
  return go;
}

// output addressing: per scene
struct OutRef {
  double* h;
  double* nb;
  long long* idx;
  int* len;
  unsigned char* ok;
  unsigned char* fr;
  double* path;
};
__device__ __forceinline__ OutRef out_ref(const IterArgs& A, int s, int n_prim) {
  OutRef r;
  r.h = A.h ? A.h + (size_t)s * n_prim : nullptr;
  r.nb = A.nb ? A.nb + (size_t)s * n_prim * 3 : nullptr;
  r.idx = A.idx ? A.idx + (size_t)s * n_prim : nullptr;
  r.len = A.rs_len ? A.rs_len + s : nullptr;
  r.ok = A.rs_ok ? A.rs_ok + s : nullptr;
  r.fr = A.fr ? A.fr + (size_t)s * n_prim : nullptr;
  r.path = A.rs_path ? A.rs_path + (size_t)s * MAXPATH * 3 : nullptr;
  return r;
}

// threads per block of ha_iter_kernel: 4 waves, three Reeds–Shepp words per wave (HA_WAVES=6 or 12:
// two words or one per wave: measured slower, 55 / 53 ms vs 45 ms per 256-scenario plan -- the
// per-wave Reeds–Shepp set-up is repeated and the launch is already issue-bound).
#ifndef HA_WAVES
#define HA_WAVES 4
#endif
constexpr int HW = HA_WAVES;
constexpr int HT = 64 * HW;
static_assert(12 % HW == 0, "HA_WAVES must divide the 12 Reeds-Shepp words");
// Tail shape, for iterations with few scenes still searching (the latency-bound end of a batched
// plan): 12 waves per block (one Reeds-Shepp word per wave) and 4 neighbours per expansion block
// (16 blocks per scene: the collision sweep is one pose per thread), so a lone scene's iteration
// spreads over 17 CUs instead of 5.
// diagnostics: -DHA_STAMP_CODE=1 compiles the per-block phase stamps in (MPGPU_HA_STAMPS=1 then turns
// them on; tools/ha_stamps.py reads them) -- out by default: the code alone cost 0.4 ms per plan (r04zb)
#ifndef HA_STAMP_CODE
#define HA_STAMP_CODE 0
#endif
#ifndef HA_NBG_TAIL
#define HA_NBG_TAIL 4
#endif
constexpr int HW_TAIL = 12, NBG_TAIL = HA_NBG_TAIL;
// the middle shape's waves per block (MPGPU_HA_MID_BLOCKS): 16 neighbours each, 12 / HA_MID_HW Reeds-Shepp
// words per wave (12-wave blocks measured 38 ms per 256-plan at MID 1024, r05q; 6-wave ones 24.9, r05x)
#ifndef HA_MID_HW
#define HA_MID_HW 6
#endif
// (A/B) -DHA_TAIL_OVERLAP=1: the tail shape's neighbour groups evaluate rs_heuristic for all their
// neighbours, overlapped with the sweep, instead of sweeping first and evaluating it only when a neighbour
// needs it (as the full-width shape does).  Measured slower (r05e, lone 729-pop scenario: 29.1 vs 28.3 us
// per iteration): with 4 neighbours per group a word fills 16 of a wave's 64 lanes, and the group's 12
// waves (3 per SIMD) are issue-bound -- the word search takes ~10 us on every group instead of ~8.5 us on
// the groups that need it.
#ifndef HA_TAIL_RSH
#define HA_TAIL_RSH 1
#endif
// (A/B build, -DHA_FULL_TUV_CODE=1 + MPGPU_HA_FULL_TUV=1) the full-width groups' winners' (t, u, v) carried
// through the full-width bookkeeping too (see the host's ftuv_env)
#ifndef HA_FULL_TUV_CODE
#define HA_FULL_TUV_CODE 0
#endif
#ifndef HA_TAIL_OVERLAP
#define HA_TAIL_OVERLAP 0
#endif

// allpath + findmin split over the block's HW waves: wave w evaluates words WPW·w+1..WPW·(w+1) for
// its lanes' candidates (lane&3 = variant of the state in `s`), the per-wave winners are
// combined in LDS in word order with the same total order (rs_before).  Every wave returns
// the block-wide winner for its lanes; *best_id is the winning candidate id.
struct NoMid {
  __device__ void operator()() const {}
};
// mid(): work the block does between its word loop and the cross-wave reduction (the tail shape's collision
// sweep), so the waves' Reeds-Shepp chains and that work overlap on the SIMDs instead of following each other
// TUV (the full-width groups): every lane also keeps its best word's (t, u, v) through the word loop and the
// variant reduction, into tv_out; the lanes of wave (id / 4) / WPW then hold the block winner's
template <bool CMD, int HWt, class Mid = NoMid, bool TUV = false>
__device__ __forceinline__ double rs_best_split(const double* s, int tid, int* best_id, double* sh_c, int* sh_i,
                                                double* cmd_out = nullptr, const Mid& mid = Mid(),
                                                double* tv_out = nullptr) {
  constexpr int WPW = 12 / HWt;  // Reeds–Shepp words per wave
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, var = lane & 3;
  double q[3];
  rs_variant(s, var, q);
  const RsPre R = rs_pre(q);
  HTIME(12);
  double bc = __builtin_inf();
  int bi = 1 << 20;
  // CMD with one word per wave (the tail shape): that word's commands are kept from its one evaluation;
  // with more (the full-width shape) carrying every lane's best commands through the loop set the kernel's
  // register peak, so the winning word is evaluated again below
  constexpr bool KEEP = CMD && WPW == 1;
  Cmd cb;
  double tb[3] = {0.0, 0.0, 0.0};
#pragma unroll 1
  for (int w = WPW * wave + 1; w <= WPW * wave + WPW; w++) {
    double tw[3];
    const double cost = rs_word(w, R, KEEP ? &cb : nullptr, TUV ? tw : nullptr);
    const int id = 4 * (w - 1) + var;
    if (rs_before(cost, id, bc, bi)) {
      bc = cost;
      bi = id;
      if (TUV)
#pragma unroll
        for (int e = 0; e < 3; e++) tb[e] = tw[e];
    }
  }
#pragma unroll
  for (int o = 2; o >= 1; o >>= 1) {
    const double ov = __shfl_xor(bc, o);
    const int oi = __shfl_xor(bi, o);
    double ot[3];
    if (TUV)
#pragma unroll
      for (int e = 0; e < 3; e++) ot[e] = __shfl_xor(tb[e], o);
    if (rs_before(ov, oi, bc, bi)) {
      bc = ov;
      bi = oi;
      if (TUV)
#pragma unroll
        for (int e = 0; e < 3; e++) tb[e] = ot[e];
    }
  }
  if (TUV)
#pragma unroll
    for (int e = 0; e < 3; e++) tv_out[e] = tb[e];
  HTIME(13);
  sh_c[tid] = bc;
  sh_i[tid] = bi;
  mid();
  __syncthreads();
  double v = sh_c[lane];
  int ix = sh_i[lane];
  for (int w = 1; w < HWt; w++) {
    const double ov = sh_c[64 * w + lane];
    const int oi = sh_i[64 * w + lane];
    if (rs_before(ov, oi, v, ix)) { v = ov; ix = oi; }
  }
  *best_id = ix;
  // CMD: the wave that evaluated the winning word evaluates it again for its commands (the same
  // operations on the same operands: the same bits) -- cheaper than carrying every lane's best
  // commands through the word loop, which set the kernel's register peak -- and the lane of the
  // winning variant stores them with allpath's gear/steer flips (timeflip: gear, reflect: steer,
  // reverse: both), as rs_commands does
  if (CMD && wave == (ix / 4) / WPW) {  // wave-uniform
    if (!KEEP) rs_word(ix / 4 + 1, R, &cb);
    const int n = v < __builtin_inf() ? cb.n : 0;
#pragma unroll
    for (int r = 0; r < 5; r++) {
      double ge = 0.0, st = 0.0, tr = 0.0;
      if (r < n) {
        tr = cb.tr[r];
        ge = cb.ge[r];
        st = cb.st[r];
        if (var == 1 || var == 3) ge = -1 * ge;
        if (var == 2 || var == 3) st = -1 * st;
      }
      if (lane == (ix & 3)) {
        cmd_out[r * 3 + 0] = tr;
        cmd_out[r * 3 + 1] = ge;
        cmd_out[r * 3 + 2] = st;
      }
    }
  }
  return v;
}

// RS_connected's allpath + findmin when the winning candidate id is already known (the popped node's
// rs_heuristic winner, IterArgs::node_rw): wave 0 evaluates only that word, lane v = variant v, and the
// lane of the winning variant stores the commands as rs_best_split does.  The same operations on the same
// operands as that candidate's evaluation inside the full search, so the same cost and commands.
__device__ __forceinline__ void rs_known_cmd(const double* s, int tid, int id, double* cmd_out) {
  if (tid >= 64) return;  // wave-uniform
  const int lane = tid & 63, var = lane & 3;
  double q[3];
  rs_variant(s, var, q);
  const RsPre R = rs_pre(q);
  Cmd cb;
  const double cost = rs_word(id / 4 + 1, R, &cb);
  const int n = cost < __builtin_inf() ? cb.n : 0;  // the winner's own cost is the search's minimum
#pragma unroll
  for (int r = 0; r < 5; r++) {
    double ge = 0.0, st = 0.0, tr = 0.0;
    if (r < n) {
      tr = cb.tr[r];
      ge = cb.ge[r];
      st = cb.st[r];
      if (var == 1 || var == 3) ge = -1 * ge;
      if (var == 2 || var == 3) st = -1 * st;
    }
    if (lane == (id & 3)) {
      cmd_out[r * 3 + 0] = tr;
      cmd_out[r * 3 + 1] = ge;
      cmd_out[r * 3 + 2] = st;
    }
  }
}

// A node's stored RS_connected commands (IterArgs::node_rw with RW_TUV): candidate id = 4(w-1) + variant, the
// word's (t, u, v) as rs_word computed them for that variant, ok = its cost < Inf.  The commands rs_known_cmd's
// winning lane writes, from the word tables, without evaluating the word again.
enum { RW_ID = 0xff, RW_TUV = 1 << 8, RW_OK = 1 << 9 };
__device__ __forceinline__ void cmd_from_tuv(int rw, const double* tuv, double* cmd_out) {
  const int id = rw & RW_ID, wi = id / 4, var = id & 3;
  const int n = (rw & RW_OK) ? kRsN[wi] : 0;
#pragma unroll
  for (int r = 0; r < 5; r++) {
    double ge = 0.0, st = 0.0, tr = 0.0;
    if (r < n) {
      const int code = kRsTr[wi][r];
      tr = code == 0 ? tuv[0] : code == 1 ? tuv[1] : code == 2 ? tuv[2] : PI2;
      ge = kRsGe[wi][r];
      st = kRsSt[wi][r];
      if (var == 1 || var == 3) ge = -1 * ge;
      if (var == 2 || var == 3) st = -1 * st;
    }
    cmd_out[r * 3 + 0] = tr;
    cmd_out[r * 3 + 1] = ge;
    cmd_out[r * 3 + 2] = st;
  }
}

// One search iteration's device work for the block (role by blockIdx: RS_connected or a
// 16-neighbour group).  Returns false (block-uniformly) when the block has nothing to do.
template <int HWt, int NBGt, bool RSH = false>
__device__ __forceinline__ bool ha_iter_body(const HaDev& P, const IterArgs& A, unsigned long long* hstp = nullptr,
                                             int slot_ = -1, int item_ = -1) {
// (diagnostics, -DHA_STAMP_CODE=1) phase stamps of the block's thread 0 into ha_step_kernel's slots 12..
#define HSTAMP(i) if (HA_STAMP_CODE && hstp) __hip_atomic_store(hstp + (i), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
  constexpr int HT = 64 * HWt, NBG = NBGt;
  __shared__ double wp[MAXW * 10];
  __shared__ double wpre[MAXW * 24];
  __shared__ double wc[MAXW * 3];
  __shared__ double wcl[MAXW * 3];
  __shared__ double cmd[15];
  __shared__ double psi_s[MAXPATH], ix_s[MAXPATH], iy_s[MAXPATH];
  __shared__ double path_s[MAXPATH * 3];
  __shared__ double red_c[HT];
  __shared__ int red_i[HT];
  __shared__ double red_t[RSH ? 3 : 1][RSH ? 192 : 1];  // RSH units: the word waves' (t, u, v)
  __shared__ double g_nb[NBG][3];
  __shared__ double g_sc[NBG][2];  // sin, cos of the regulated heading (changeBasis of rs_heuristic)
  __shared__ long long g_ix[NBG];
  __shared__ int g_free[NBG];
  __shared__ int g_need[NBG];
  __shared__ int sh_n;
  const int per = 1 + (P.n_prim + NBG - 1) / NBG + (RSH ? 1 : 0);  // RSH: the prescan block is the last item
  // (ha_pipe_kernel passes its own slot / role numbering)
  const int slot = slot_ >= 0 ? slot_ : blockIdx.x / per, item = item_ >= 0 ? item_ : blockIdx.x % per;
  // the live count and the slot's scene are independent loads (slot < the grid's bound <= B keeps the
  // list read in bounds); a scene on the bookkeeping's list (n_live set) is live, so its flag is not
  // read: the node and goal loads then follow one round trip instead of three
  const int n_live = A.n_live ? *A.n_live : A.n_active;
  const int s = A.scene_of ? A.scene_of[slot] : slot;
  if (slot >= n_live) return false;  // past the live-scene list
  if (item == 0 && !A.do_rs) return false;
  if (item > 0 && !A.do_exp) return false;
  const bool rs = item == 0;  // block-uniform role: RS_connected, else a 16-neighbour group
  if (!A.n_live && A.active && !A.active[s]) return false;  // scene finished (device-resident search)
  const int tid = threadIdx.x, lane = tid & 63;
  HMARK(1);
  HTIME(0);
  const int nw = P.n_walls;
  const double* node = A.node + 3 * s;
  const double* goal = A.goal + 3 * s;
  __shared__ double nd_s[3], nd_g, nd_tuv[3];
  __shared__ int nd_go, nd_nn, nd_rw;
  const OutRef R = out_ref(A, s, P.n_prim);
  const int k0 = rs ? 0 : (item - 1) * NBG, nk = rs ? 0 : min(NBG, P.n_prim - k0);
  // wall corners (Block2Pts) and their SAT tables in LDS: precomputed once per plan
  // (ha_wall_kernel) or evaluated here
  if (A.wtab) {
    for (int i = tid; i < nw * WT; i += HT) {
      const double v = A.wtab[(size_t)s * nw * WT + i];
      const int w = i / WT, e = i - WT * w;
      if (e < 10) wp[10 * w + e] = v;
      else if (e < 34) wpre[24 * w + e - 10] = v;
      else if (e < 37) wc[3 * w + e - 34] = v;
      else wcl[3 * w + e - 37] = v;
    }
  } else {
    for (int i = tid; i < nw; i += HT) {
      const double* wl = A.walls + ((size_t)s * nw + i) * 5;
      rect_pts(wl[0], wl[1], mpj_cos(wl[2]), mpj_sin(wl[2]), wl[3], wl[4], wp + 10 * i);
      sat_base_pre(wp + 10 * i, wpre + 24 * i);
      wc[3 * i] = wl[0];
      wc[3 * i + 1] = wl[1];
      wc[3 * i + 2] = wall_far2(P, wl);
      wall_cull(P, wp + 10 * i, wpre + 24 * i, wl, wcl + 3 * i);
    }
  }
  if (tid < NBG) g_free[tid] = 1;
  if (A.node_ag) {  // the node comes from another block of this launch (ha_pipe_kernel's bookkeeping): wait for
    // its ready flag (the walls are staged meanwhile), then read it agent-coherently
    if (A.ngr) {  // tagged granules: the node and its ready state in one poll (ha_consume_node)
      if (tid < 64) {
        const int go = ha_consume_node(A.ngr + (size_t)s * HA_NGR, A.ngr_tag, tid, nd_s, nd_tuv, &nd_rw,
                                       A.node_flag_err);
        if (tid == 0) nd_go = go;
      }
      __syncthreads();
      if (!nd_go) return false;  // block-uniform: the search ended, nothing to expand
      if (nd_go & 2) return true;  // block-uniform: nothing to do this round (HA_SPEC: expanded speculatively)
    } else {
      if (tid == 0) nd_go = wait_ge(A.node_flag + s, A.node_flag_min, A.node_flag_err) & 1;
      __syncthreads();
      if (!nd_go) return false;  // block-uniform: the search ended, nothing to expand
      if (tid < 3) nd_s[tid] = ld_ag(A.node + 3 * s + tid);
      if (tid == 3 && A.node_g) nd_g = ld_ag(A.node_g + s);
      if (tid == 4 && A.node_g) nd_nn = ld_ag(A.node_nn + s);
      __syncthreads();
    }
    node = nd_s;
  }
  // the tail shape (threads to spare): the collision sweep splits every pose into its 2·n_walls SAT terms,
  // one per thread, and a neighbour group evaluates rs_heuristic for all its neighbours at once
  constexpr bool SPLIT = HWt == HW_TAIL;
  int hit = -1;  // (groups with a Dict) the neighbour's node id in the scene's Dict
  // the expanded node's heading is a lattice heading m·res[2] (bit for bit; every regulated state's is): its
  // neighbours' heading terms and its poses' come from the per-plan tables
  const int tabm = lattice_m(P, A, node[2]);
  if (tid < nk) {  // transform + regulate_states + Encode of the group's neighbours (:396-405)
    const int k = k0 + tid;
    double nb[3], sn, cn;
    const long long ix = expand_nb(P, A, node, tabm, k, nb, &sn, &cn);
    g_sc[tid][0] = sn;
    g_sc[tid][1] = cn;
    if (!rs && !RSH && !(SPLIT && HA_TAIL_OVERLAP) && A.dnid) hit = ix > 0 && ix < A.C ? A.dnid[(size_t)s * A.C + ix] : -1;
    st_out(A.coherent, R.nb + 3 * k, nb[0]);
    st_out(A.coherent, R.nb + 3 * k + 1, nb[1]);
    st_out(A.coherent, R.nb + 3 * k + 2, nb[2]);
    st_out(A.coherent, R.idx + k, ix);
    g_nb[tid][0] = nb[0];
    g_nb[tid][1] = nb[1];
    g_nb[tid][2] = nb[2];
    g_ix[tid] = ix;
  }
  HMARK(6);
  HTIME(1);
  HSTAMP(12);
  __syncthreads();
  const int j = lane >> 2;
  // (A/B build -DHA_SWEEP_PROBE=1, non-RSH groups) the last swept pose of every neighbour first: a neighbour that
  // collides there (the far end of its primitive) skips its other poses -- whole waves of them, as a wave covers
  // about one neighbour's poses.  Same result (an OR over poses); measured 0.3-0.4 ms slower per 256-plan
  // (r05zt: the extra phase and barrier cost more than the skipped rounds), so off.
#ifndef HA_SWEEP_PROBE
#define HA_SWEEP_PROBE 0
#endif
  auto sweep = [&](int npose, int nthr = 64 * HWt) {
    double nsn = 0.0, ncs = 1.0;
    if (!rs) {
      if (tabm >= 0) {
        nsn = A.htn[2 * tabm];
        ncs = A.htn[2 * tabm + 1];
      } else {
        mpj_sincos_bl(node[2], &nsn, &ncs);
      }
    }
    const int parts = SPLIT ? 2 * nw : 1;
    auto item = [&](int jn, int jp, int part) {
      double q[3];
      if (rs) {
        q[0] = path_s[3 * (jp * 5)];
        q[1] = path_s[3 * (jp * 5) + 1];
        q[2] = path_s[3 * (jp * 5) + 2];
      } else {
        transform_cs(node, ncs, nsn, A.pc + ((size_t)(k0 + jn) * P.n_col + jp * 5) * 3, q);
      }
      int fr;
      if (!rs && tabm >= 0 && A.ptab) {  // block-uniform (the RS path's poses have their own headings)
        const double2* e =
            reinterpret_cast<const double2*>(A.ptab + (((size_t)tabm * P.n_prim + k0 + jn) * A.pt_nsw + jp) * 4);
        const double2 a = e[0], c = e[1];
        const PoseTrig T{a.x, a.y, c.x, c.y};
        fr = SPLIT ? pose_free_part_t(P, q, T, wp, wpre, wc, wcl, part >> 1, part & 1)
                   : pose_free_t(P, q, T, wp, wpre, wc, wcl, nw);
      } else {
        fr = SPLIT ? pose_free_part(P, q, wp, wpre, wc, wcl, part >> 1, part & 1) : pose_free(P, q, wp, wpre, wc, wcl, nw);
      }
      if (!fr) g_free[jn] = 0;  // every writer stores 0
    };
    constexpr bool PROBE = HA_SWEEP_PROBE && !RSH && !SPLIT;
    if (PROBE && !rs && npose > 1) {  // block-uniform
      for (int t = tid; t < nk; t += nthr)
        if (g_ix[t] != 0 && g_free[t]) item(t, npose - 1, 0);
      __syncthreads();
    }
    const int total = (rs ? npose : nk * npose) * parts;
    for (int t = tid; t < total; t += nthr) {
      const int tp = SPLIT ? t / parts : t, part = SPLIT ? t - tp * parts : 0;
      const int jn = rs ? 0 : tp / npose, jp = rs ? tp : tp - jn * npose;
      if (!rs && g_ix[jn] == 0) continue;  // Encode 0: skipped before the collision check (:406-408)
      if (!g_free[jn]) continue;  // already colliding: block_collision_check stops at its first hit
      if (PROBE && !rs && npose > 1 && jp == npose - 1) continue;  // (probed above)
      item(jn, jp, part);
    }
  };
  double cb = 0.0;
  int best = -1;
  if (rs) {
    // allpath + findmin: RS_connected's optimal command from the popped node
    double ns[3];
    // the popped node's stored rs_heuristic winner (agent-coherently when published in this launch)
    const int known =
        A.node_rw ? (A.node_ag ? (A.ngr ? nd_rw : ld_ag(A.node_rw + s)) : A.node_rw[s]) : -1;
    if (tabm >= 0)
      change_basis_sc(node, goal, P.minR, A.htn[2 * tabm], A.htn[2 * tabm + 1], ns);
    else
      change_basis(node, goal, P.minR, ns);
    HTIME(2);
    HSTAMP(12);
    if (known >= 0 && (known & RW_TUV)) {  // block-uniform: the commands stored at the node's creation
      if (tid == 0) {
        double tv[3];
        for (int e = 0; e < 3; e++)
          tv[e] = A.node_ag ? (A.ngr ? nd_tuv[e] : ld_ag(A.node_tuv + 3 * s + e)) : A.node_tuv[3 * s + e];
        cmd_from_tuv(known, tv, cmd);
      }
    } else if (known >= 0 && known < 48)
      rs_known_cmd(ns, tid, known, cmd);
    else
      cb = rs_best_split<true, HWt>(ns, tid, &best, red_c, red_i, cmd);
    HSTAMP(13);
    HTIME(3);
    // createActPath (ReedsSheppsUtils.jl:440-466): 100 Euler steps per segment -- per segment the
    // heading recurrence ψ_{t+1} = ψ_t + (st*v)*dt, the per-step increments, then the x and y
    // running sums -- software-pipelined over the segments: stage k runs segment k's heading, segment
    // k-1's increments and segment k-2's running sums, each on its own threads, so the serial chains
    // of different segments overlap.  The same operations in the same order per value.
    __syncthreads();  // cmd (written by the winning lane) visible
    int nseg = 0;
    for (int i = 0; i < 5; i++) {
      if (cmd[i * 3 + 1] == 0) break;
      nseg++;
    }
    const int nst = 100 * nseg;
    constexpr int TP = 128, TW = 192;  // the serial heading's thread; the first increment thread
    static_assert(HT > TW, "the pipelined createActPath needs four waves");
    if (tid == 0) {
      psi_s[0] = node[2];
      path_s[0] = node[0];
      path_s[1] = node[1];
    }
    __syncthreads();
    for (int st = 0; st < nseg + 2; st++) {
      {  // segment st: the heading recurrence, all 100 steps at once when the closed form of repeated
         // addition applies (mpj_rep_add_ok: same bits, block-uniform), else on thread TP
        const int seg = st;
        if (seg < nseg) {
          const double q0 = psi_s[seg * 100];
          const double dt = __builtin_fabs(cmd[seg * 3]) / 100;
          const double c = (cmd[seg * 3 + 2] * cmd[seg * 3 + 1]) * dt;
          double d;
          if (mpj_rep_add_ok(q0, c, 100, &d)) {
            for (int k = tid - TW; k >= 0 && k < 100; k += HT - TW)
              psi_s[seg * 100 + k + 1] = c == 0.0 ? q0 + c : mpj_fma(k + 1, d, q0);
          } else if (tid == TP) {
            double q = q0;
            for (int k = 0; k < 100; k++) {
              q = q + c;
              psi_s[seg * 100 + k + 1] = q;
            }
          }
        }
      }
      {  // segment st-1: the per-step increments
        const int seg = st - 1;
        if (seg >= 0 && seg < nseg) {
          const double dt = __builtin_fabs(cmd[seg * 3]) / 100, v = cmd[seg * 3 + 1];
          for (int k = tid - TW; k >= 0 && k < 100; k += HT - TW) {
            const int t = seg * 100 + k;
            double sn, cs;
            mpj_sincos_bl(psi_s[t], &sn, &cs);
            double d0 = v * cs, d1 = v * sn;
            d0 = d0 * P.minR;
            d1 = d1 * P.minR;
            ix_s[t] = d0 * dt;
            iy_s[t] = d1 * dt;
            path_s[3 * (t + 1) + 2] = psi_s[t + 1];
          }
        }
      }
      {  // segment st-2: the running sums in order, a straight segment (every increment the same bits)
         // in closed form, else x on thread 0 and y on thread 64
        const int seg = st - 2;
        if (seg >= 0 && seg < nseg) {
          const int t0 = seg * 100;
          const double x0 = path_s[3 * t0], y0 = path_s[3 * t0 + 1];
          const double ix = ix_s[t0], iy = iy_s[t0];
          const bool same = __double_as_longlong(psi_s[t0]) == __double_as_longlong(psi_s[t0 + 1]) &&
                            cmd[seg * 3 + 2] * cmd[seg * 3 + 1] == 0.0;  // ψ constant over the segment
          double dx, dy;
          const bool cx = same && mpj_rep_add_ok(x0, ix, 100, &dx), cy = same && mpj_rep_add_ok(y0, iy, 100, &dy);
          for (int k = tid - TW; k >= 0 && k < 100; k += HT - TW) {
            if (cx) path_s[3 * (t0 + k + 1)] = ix == 0.0 ? x0 + ix : mpj_fma(k + 1, dx, x0);
            if (cy) path_s[3 * (t0 + k + 1) + 1] = iy == 0.0 ? y0 + iy : mpj_fma(k + 1, dy, y0);
          }
          if ((tid == 0 && !cx) || (tid == 64 && !cy)) {
            const int c = tid == 0 ? 0 : 1;
            const double* inc = c == 0 ? ix_s : iy_s;
            double acc = c == 0 ? x0 : y0;
            // batches of 20 increments into registers first: the LDS reads then pipeline instead of
            // each waiting behind the previous path store (the compiler cannot disprove aliasing)
            for (int u0 = t0; u0 < t0 + 100; u0 += 20) {
              double v[20];
#pragma unroll
              for (int u = 0; u < 20; u++) v[u] = inc[u0 + u];
#pragma unroll
              for (int u = 0; u < 20; u++) {
                acc = acc + v[u];
                path_s[3 * (u0 + u + 1) + c] = acc;
              }
            }
          }
        }
      }
      __syncthreads();
    }
    HTIME(8);
    HSTAMP(14);
    if (tid == 0) path_s[2] = node[2];
    __syncthreads();
    const int n = nst + 1;
    if (!A.rs_path_free_only)
      for (int i = tid; i < 3 * n; i += HT) st_out(A.coherent, R.path + i, path_s[i]);
    if (tid == 0) sh_n = n;
    HTIME(4);
    sweep(n > 5 ? (n - 1) / 5 + 1 : 1);  // block_collision_check on poses 1:5:end
    HTIME(5);
  } else if (RSH) {
    // tail shape, rs_heuristic in word units (IterArgs::hp_c): waves 0 .. HWt-4 sweep the group's own
    // neighbours; waves HWt-3 .. HWt-1 each evaluate one Reeds-Shepp word, 3c+1 .. 3c+3, for the 16 neighbours
    // 16g .. 16g+15 (g = (item-1)/4, c = (item-1)%4; 64 lanes = 16 neighbours x 4 variants, every lane used),
    // whatever the sweep finds.  Per SIMD at most one such wave: the word chains run side by side on the
    // scene's 16 group CUs (a group's 12-wave word search with 16 lanes per word was issue-bound, ~8.5 us).
    // The scene's bookkeeping combines the four word chunks of each neighbour (rs_before is a total order).
    static_assert(HWt >= 4, "three word waves beside the sweep");
    constexpr int SWT = 64 * (HWt - 3);
    const int g = (item - 1) >> 2, c = (item - 1) & 3;
    const int npose = P.n_col > 5 ? (P.n_col - 1) / 5 + 1 : 1;
    if (tid < SWT) {
      sweep(npose, SWT);
    } else {
      const int w = 3 * c + ((tid - SWT) >> 6) + 1;  // wave-uniform
      const int k = min(16 * g + (lane >> 2), P.n_prim - 1);
      double nb[3], ns[3], q[3], sn, cn;
      expand_nb(P, A, node, tabm, k, nb, &sn, &cn);  // the owner group's operations: the same regulated state
      change_basis_sc(nb, goal, P.minR, sn, cn, ns);
      rs_variant(ns, lane & 3, q);
      const RsPre Rp = rs_pre(q);
      double tv[3];
      double bc = rs_word(w, Rp, nullptr, tv);
      int bi = 4 * (w - 1) + (lane & 3);
#pragma unroll
      for (int o = 2; o >= 1; o >>= 1) {
        const double ov = __shfl_xor(bc, o);
        const int oi = __shfl_xor(bi, o);
        double ot[3];
#pragma unroll
        for (int e = 0; e < 3; e++) ot[e] = __shfl_xor(tv[e], o);
        if (rs_before(ov, oi, bc, bi)) {
          bc = ov;
          bi = oi;
#pragma unroll
          for (int e = 0; e < 3; e++) tv[e] = ot[e];
        }
      }
      red_c[tid] = bc;
      red_i[tid] = bi;
#pragma unroll
      for (int e = 0; e < 3; e++) red_t[e][tid - SWT] = tv[e];
    }
    HSTAMP(13);
    __syncthreads();
    if (tid >= SWT && tid < SWT + 64 && (lane & 3) == 0) {  // the chunk's three words, per neighbour
      double v = red_c[tid];
      int ix = red_i[tid], wu = 0;
#pragma unroll
      for (int u = 1; u < 3; u++) {
        const double ov = red_c[tid + 64 * u];
        const int oi = red_i[tid + 64 * u];
        if (rs_before(ov, oi, v, ix)) { v = ov; ix = oi; wu = u; }
      }
      const int k = 16 * g + (lane >> 2);
      if (k < P.n_prim) {
        const size_t q = ((size_t)s * P.n_prim + k) * 4 + c;
        st_out(A.coherent, A.hp_c + q, v);
        st_out(A.coherent, A.hp_i + q, ix);
#pragma unroll
        for (int e = 0; e < 3; e++) st_out(A.coherent, A.hp_t + 3 * q + e, red_t[e][tid - SWT + 64 * wu]);
      }
    }
    HSTAMP(14);
    HSTAMP(15);
  } else if (SPLIT && HA_TAIL_OVERLAP) {
    // tail shape (latency-bound: CUs to spare, one scene's chain): rs_heuristic of every neighbour of the
    // group, whether or not FindNewNode will read it, without waiting for the collision sweep; the sweep
    // runs between each wave's Reeds-Shepp word and the cross-wave reduction, so the two overlap
    double ns[3];
    const int jj = j < nk ? j : 0;
    change_basis_sc(g_nb[jj], goal, P.minR, g_sc[jj][0], g_sc[jj][1], ns);
    const int npose = P.n_col > 5 ? (P.n_col - 1) / 5 + 1 : 1;
    cb = rs_best_split<false, HWt>(ns, tid, &best, red_c, red_i, nullptr, [&] { sweep(npose); });
    HSTAMP(13);
    HSTAMP(14);
    HSTAMP(15);
  } else {
    // dg_cost first (primitive poses 1:5:n_col): rs_heuristic is only used for neighbours that
    // are collision-free and in bounds, so a group without one skips the 48 RS candidates.
    // FindNewNode (:418-446) also leaves a neighbour alone whose cell already holds a node with
    // g <= tg = g(popped) + expand_time (the same tg for every neighbour): its heuristic is never read.
    // The Dict at this launch is the one this iteration's FindNewNode starts from (the bookkeeping
    // that changes it runs after every neighbour group of the scene, ha_step_kernel / ha_book_kernel).
    double gd = 0.0;
    if (hit >= 0) gd = A.dg[(size_t)s * A.C + hit];  // loaded now, used after the sweep (a node newer than
    // the pipelined launch's nn_lim below may be half-written: its g is loaded but never used)
    // (step launches) the rest of the neighbour's Dict entry for the bookkeeping, loaded beside gd and stored
    // after the sweep (the Dict is the one this iteration's FindNewNode starts from: it runs after every group)
    const bool drec = HA_DREC_CODE && A.drec && A.dnid && !A.node_ag && tid < nk;
    long long dv[HA_DREC - 2];
    if (drec && hit >= 0) {
      const size_t q = (size_t)s * A.C + hit;
      dv[0] = A.dpos[q];
      dv[1] = __double_as_longlong(A.df[q]);
      dv[2] = A.dseq[q];
      dv[3] = A.dindex[q];
      dv[4] = A.drw[q];
#pragma unroll
      for (int e = 0; e < 3; e++) dv[5 + e] = __double_as_longlong(A.dst[q * 3 + e]);
    }
    sweep(P.n_col > 5 ? (P.n_col - 1) / 5 + 1 : 1);
    if (drec) {
      long long* o = A.drec + ((size_t)s * P.n_prim + k0 + tid) * HA_DREC;
      st_out(A.coherent, o, (long long)hit);
      if (hit >= 0) {
        st_out(A.coherent, o + 1, __double_as_longlong(gd));
#pragma unroll
        for (int e = 0; e < HA_DREC - 2; e++) st_out(A.coherent, o + 2 + e, dv[e]);
      }
    }
    HTIME(4);
    HSTAMP(13);
    // (full-width ha_pipe_kernel) this iteration's FindNewNode writes the Dict meanwhile: only nodes older than
    // it (id < its starting node count) are trusted, and their g only decreases, so the g read (the old or the
    // new value) >= the g FindNewNode(n_{it+1}) compares with: a skip stays a skip
    const bool pub = A.node_ag && A.node_g;
    const int nn_lim = pub ? nd_nn : 0x7fffffff;
    if (tid < nk)  // (A.cur_g only with a Dict: mp_ha_expand has neither)
      g_need[tid] = !A.dnid || !(hit >= 0 && hit < nn_lim && !((pub ? nd_g : A.cur_g[s]) + P.expand_time < gd));
    __syncthreads();
    HTIME(5);
    HSTAMP(14);
    int any = 0;
    for (int q = 0; q < nk; q++) any |= (g_ix[q] != 0) & g_free[q] & g_need[q];
    if (any) {  // block-uniform
      double ns[3];
      const int jj = j < nk ? j : 0;
      change_basis_sc(g_nb[jj], goal, P.minR, g_sc[jj][0], g_sc[jj][1], ns);
      HTIME(2);
      if (HA_FULL_TUV_CODE && A.full_tuv && A.hp_t) {  // (t, u, v) of each neighbour's winner, for RS_connected
        double tv[3];
        cb = rs_best_split<false, HWt, NoMid, true>(ns, tid, &best, red_c, red_i, nullptr, NoMid(), tv);
        if ((lane & 3) == 0 && j < nk && (tid >> 6) == (best / 4) / (12 / HWt))
#pragma unroll
          for (int e = 0; e < 3; e++)
            st_out(A.coherent, A.hp_t + ((size_t)s * P.n_prim + k0 + j) * 12 + e, tv[e]);
      } else {
        cb = rs_best_split<false, HWt>(ns, tid, &best, red_c, red_i);
      }
      HSTAMP(15);
      HTIME(3);
    }
  }
  HMARK(20);
  HTIME(10);
  HSTAMP(16);
  __syncthreads();
  if (rs) {
    if (tid == 0) {
      st_out(A.coherent, R.ok, (unsigned char)g_free[0]);
      st_out(A.coherent, R.len, sh_n);
    }
    if (A.rs_path_free_only && g_free[0])  // block-uniform (after the barrier above)
      for (int i = tid; i < 3 * sh_n; i += HT) st_out(A.coherent, R.path + i, path_s[i]);  // (read by ha_persist_kernel)
  } else if (tid < 64 && (lane & 3) == 0 && j < nk) {
    const int fr = g_ix[j] != 0 && g_free[j];
    st_out(A.coherent, R.fr + k0 + j, (unsigned char)fr);
    if (!RSH) {  // (RSH: the bookkeeping forms h and the winner from the word chunks)
      st_out(A.coherent, R.h + k0 + j, fr ? cb * P.minR : 0.0);
      if (A.hw) st_out(A.coherent, A.hw + (size_t)s * P.n_prim + k0 + j, fr ? best : -1);
    }
  }
  return true;
}

template <int HWt, int NBGt>
__global__ __launch_bounds__(64 * HWt) void ha_iter_kernel(HaDev P, IterArgs A) {
  ha_iter_body<HWt, NBGt>(P, A);
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
  const RsPre R = rs_pre(q);
  double bc = __builtin_inf();
  int bi = 1 << 20;
#pragma unroll 1
  for (int w = 1; w <= 12; w++) {
    Cmd c;
    const double cst = rs_word(w, R, &c);
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
  D->cull = 0;  // set per call by ha_cull_ok
  return MP_OK;
}

// the coordinate-magnitude guard of the SAT culls (HA_CULL_MAX above): walls [B][n_walls][5] (x, y, ψ,
// half length, half width), a and b [B][3] (nodes / starts, goals)
void ha_cull_ok(const mp_ctx* ctx, const mp_ha_params* p, HaDev* D, int B, const double* walls, const double* a,
                const double* b) {
  // the largest magnitude, and whether any input is NaN or infinite (std::max drops a NaN operand, so it is
  // tracked separately: a non-finite coordinate or length turns the culls off, every SAT call then runs)
  double m = 0.0;
  bool finite = true;
  auto see = [&](double v) {
    finite &= std::isfinite(v);
    m = std::max(m, std::fabs(v));
  };
  for (double v : {p->minR, p->vehicle_len, p->vehicle_wid, p->expand_time, ctx->ha_prim_ext}) see(v);
  for (int i = 0; i < 6; i++) see(p->stbound[i]);
  for (size_t i = 0; walls && i < (size_t)B * p->n_walls; i++) {
    const double* w = walls + 5 * i;
    see(w[2]);
    see(std::fabs(w[0]) + std::fabs(w[3]) + std::fabs(w[4]));
    see(std::fabs(w[1]) + std::fabs(w[3]) + std::fabs(w[4]));
  }
  for (size_t i = 0; i < 3 * (size_t)B; i++) {
    if (a) i % 3 != 2 ? see(a[i]) : (void)(finite &= std::isfinite(a[i]));
    if (b) i % 3 != 2 ? see(b[i]) : (void)(finite &= std::isfinite(b[i]));
  }
  D->cull = finite && m <= HA_CULL_MAX;
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
  hipLaunchKernelGGL((ha_iter_kernel<HW, NBG>), dim3((unsigned)(A.n_active * (1 + (D.n_prim + NBG - 1) / NBG))), dim3(HT), 0,
                     ctx->stream, D, A);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  return MP_OK;
}

// Block2Pts + the wall-side SAT tables (pose independent) + centre / far² + the cull bounds once per plan:
// [B][nw][WT]
// the pose table (IterArgs::ptab): thread = (m, primitive k, swept pose j); the heading m·res[2] + the
// primitive pose's heading, as transform computes it, and its PoseTrig
__global__ __launch_bounds__(256) void ha_pose_table_kernel(HaDev P, const double* pc, int mlo, int nm, int nsw,
                                                            double* tab) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= nm * P.n_prim * nsw) return;
  const int j = t % nsw, k = (t / nsw) % P.n_prim, m = t / (nsw * P.n_prim);
  const double head = (double)(mlo + m) * P.res[2];
  const double psi = pc[((size_t)k * P.n_col + j * 5) * 3 + 2] + head;
  const PoseTrig T = pose_trig(psi);
  double* o = tab + (size_t)t * 4;
  o[0] = T.sq;
  o[1] = T.cq;
  o[2] = T.sy;
  o[3] = T.cy;
}

// the lattice-heading tables (IterArgs::htn / htk): thread = (m, neighbour k)
__global__ __launch_bounds__(256) void ha_head_table_kernel(HaDev P, const double* sc, int mlo, int nm, double* htn,
                                                            double* htk) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= nm * P.n_prim) return;
  const int k = t % P.n_prim, m = t / P.n_prim;
  const double head = (double)(mlo + m) * P.res[2];
  if (k == 0) {
    double sh, ch;
    mpj_sincos_bl(head, &sh, &ch);
    htn[2 * m] = sh;
    htn[2 * m + 1] = ch;
  }
  const double t2 = sc[3 * k + 2] + head;  // transform's heading (o[2] = q[2] + node[2])
  const double psi = mpj_modpi_bl(t2);       // regulate_states
  const double nb2 = mpj_round(psi / P.res[2]) * P.res[2];
  double sn, cn;
  mpj_sincos_bl(nb2, &sn, &cn);
  double* o = htk + (size_t)t * 4;
  o[0] = nb2;
  o[1] = sn;
  o[2] = cn;
  o[3] = encode_pid(P, nb2);
}

__global__ __launch_bounds__(64) void ha_wall_kernel(HaDev P, int B, const double* walls, double* wtab) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= B * P.n_walls) return;
  const double* wl = walls + (size_t)i * 5;
  double* o = wtab + (size_t)i * WT;
  rect_pts(wl[0], wl[1], mpj_cos(wl[2]), mpj_sin(wl[2]), wl[3], wl[4], o);
  sat_base_pre(o, o + 10);
  o[34] = wl[0];
  o[35] = wl[1];
  o[36] = wall_far2(P, wl);
  wall_cull(P, o, o + 10, wl, o + 37);
}

// ------------------------------------------------ device-resident search state
// planHybridAstar! (hybrid_astar_utils.jl:235-296) bookkeeping on the device, one scene per
// block, all arrays scene-major.  Nodes are numbered in creation order (as Dict insertion in
// the reference / the oracle); nid is nodes_collection (Encode index -> node id).  The open
// list is a compact array of (f, seq, id) entries; its order is the reference's: a stable
// sort by f every iteration (`sort!` + `popfirst!`, :242-244) keeps equal-f nodes in list
// order, i.e. the key (f, seq) where seq is the node's rank in the list order -- nodes whose
// f decreased in place get fresh seqs in their previous list order, then the nodes appended
// by push! in push order (FindNewNode :418-446).  popfirst! = the least (f, seq) key.
struct HaSearch {
  int C;                 // Encode cells per scene (ncell + 1: cell 0 holds an out-of-bounds start)
  int mp;                // max_pops
  long long* parent;     // [B][C] per node id: parent Encode index (-1: none)
  double* st;            // [B][C][3]
  long long* index;      // [B][C]
  double *g, *h, *f;     // [B][C]
  long long* seq;        // [B][C]
  int* pos;              // [B][C] open-list position, -1 = not in the open list
  int* nid;              // [B][C] cell -> node id, -1 = absent
  double* of;            // [B][C] open entries: f, seq, node id, and the node's g, Encode
  long long* oseq;       // index and state (so popfirst! needs no second dependent load)
  int* oid;
  double* og;
  long long* oix;
  double* ost;           // [B][C][3]
  double* cur_g;         // [B] popped node's g and Encode index
  long long* cur_ix;
  int* sc_i;             // [8][B] per-scene ints: n_nodes, n_open, loop, cur, active, found, n_states, rs_len
  long long* ctr;        // [B] seq counter
  long long* start_index;// [B]
  long long* pop_seq;    // [B][mp]
  double* states;        // [B][mp][3] hybrid_astar_states (goal side first)
  double* node;          // [2][B][3] popped node state: the next iteration's input (iteration i pops into
                         // buffer i & 1 while its blocks read buffer (i - 1) & 1)
  int* live;             // [mp + 2] scenes still searching after iteration i
  int* lst;              // [2][B] those scenes' indices (iteration i writes list i & 1, in any order)
  int* tk;               // [2][B] ha_step_kernel arrival tickets: neighbour groups, then (RS block, bookkeeping)
  long long* rec;        // [B][8] ha_step_kernel: the bookkeeping's record for the scene's finisher
  int* rw;               // [B][C] per node id: rs_heuristic's winning candidate at the node's creation (-1: unknown)
  int* orw;              // [B][C] open entries: the same, so popfirst! hands it to RS_connected with the state
  int* node_rw;          // [2][B] popped node's winner, double-buffered like node
  double* tuv;           // [B][C][3] per node id: the winner's (t, u, v) when rw has RW_TUV
  double* otuv;          // [B][C][3] open entries: the same
  double* node_tuv;      // [2][B][3] popped node's, double-buffered like node
  long long* pre;        // [B][PRE_W] (RSH tail) the prescan's record: popfirst!'s K least entries before FindNewNode
  double* node_g;        // [2][B] (full-width ha_pipe_kernel) the popped node's g, double-buffered like node
  int* node_nn;          // [2][B] the scene's node count before the FindNewNode that published the node
  unsigned long long* ngr;  // [HA_NGR_SLOTS][B][HA_NGR] the popped node as tagged granules (ha_publish_node), by it & 3
  int* nx;               // [B] (ha_pipe_kernel) 2·it + 2 + go once iteration it's bookkeeping has popped the next node
  int* ex;               // [B] (ha_persist_kernel) expansions finished (neighbour groups, cumulative)
  int* rsr;              // [2][B] (ha_persist_kernel) 2·it + 2 once RS_connected(n_it) has run, by it & 1 (its RS block)
  int* err;              // [1] (ha_persist_kernel) a bounded wait ran out (the search is then not trusted)
  // (ha_persist_kernel, HA_SPEC) the runner-up: popfirst!'s second-least entry when n_{it+1} is popped, the
  // candidate for n_{it+2}, expanded (and RS_connected) speculatively
  unsigned long long* ngr2;  // [HA_NGR_SLOTS][B][HA_NGR] the runner-up as tagged granules, by it & 3
  int* exs;              // [2][B] speculative expansions finished (neighbour groups, cumulative), by the parity of the runner-up's iteration
  int* rsrs;             // [2][B] 2·it + 2 once RS_connected(r_it) has run, by it & 1
  int* nhit;             // [2][B] (diagnostics) pops that were the runner-up, runner-ups published
};
// prescan record: [0] iteration tag, [1] kc = min(K, n_open), then K entries of 13 words: f (bits), seq, position,
// node id, g (bits), Encode index, state (3, bits), rw, (t, u, v) (3, bits)
constexpr int PRE_K = 4, PRE_E = 13, PRE_W = 2 + PRE_E * PRE_K;
enum { SI_NNODES = 0, SI_NOPEN, SI_LOOP, SI_CUR, SI_ACTIVE, SI_FOUND, SI_NSTATES, SI_RSLEN, SI_N };

// open-list order: a before c (Julia isless on f, then list position)
__device__ __forceinline__ bool key_before(double af, long long as, double cf, long long cs) {
  if (mpj_isless(af, cf)) return true;
  if (mpj_isless(cf, af)) return false;
  return as < cs;
}

// lane exchanges without LDS round trips: DPP row operations, v_readlane
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ long long dpp_l(long long x) {
  const int lo = dpp_i<CTRL>((int)x), hi = dpp_i<CTRL>((int)(x >> 32));
  return ((long long)hi << 32) | (unsigned int)lo;
}
__device__ __forceinline__ long long readlane_l(long long x, int l) {
  const int lo = __builtin_amdgcn_readlane((int)x, l), hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return ((long long)hi << 32) | (unsigned int)lo;
}
// (f, seq, pos) <- the open-list-order minimum of itself and the DPP partner's (pos < 0: none)
template <int CTRL>
__device__ __forceinline__ void key_min_dpp(double& f, long long& sq, int& p) {
  const double of = __longlong_as_double(dpp_l<CTRL>(__double_as_longlong(f)));
  const long long os = dpp_l<CTRL>(sq);
  const int op = dpp_i<CTRL>(p);
  if (op >= 0 && (p < 0 || key_before(of, os, f, sq))) {
    f = of;
    sq = os;
    p = op;
  }
}

// popfirst! for scene b (a 256-thread block): the least (f, seq) open entry, found by a
// strided scan (4 independent entry loads in flight per thread) and a wave then block
// reduction (the key order is total, so the reduction order does not matter); wave 0 removes
// it by moving the last entry into its place.  Returns false (block-uniform) when the search
// ends here (open list empty / max_pops).
// NT threads (a multiple of 64).  The popped state goes to node_out[3 * b]; direct: the pop count and
// pop_seq are written here (ha_init_kernel, ha_book_kernel), else they are left to the scene's finisher
// in ha_step_kernel and the popped Encode index is returned in *iw_out (lane 0 of wave 0).
constexpr int BKT = 256;
// TUV: the open entries carry the (t, u, v) of RSH-tail nodes (only the tail's launches can meet them: the shapes
// go full width -> tail, never back)
template <int NT, bool TUV = true>
__device__ __forceinline__ bool ha_pop(const HaSearch& Q, int B, int b, int n_open, int loop, int tid,
                                       double* node_out, int* rw_out, double* tuv_out, bool direct, long long* iw_out,
                                       unsigned long long* stp = nullptr) {
  static_assert(NT % 64 == 0, "whole waves");
  __shared__ double r_f[NT / 64];
  __shared__ long long r_s[NT / 64];
  __shared__ int r_p[NT / 64];
  __shared__ double r_pay[NT / 64][5];  // the wave winner's entry: g, Encode index, state
  __shared__ int r_id[NT / 64];
  __shared__ int r_rw[NT / 64];
  __shared__ double r_tuv[NT / 64][3];
  const size_t base = (size_t)b * Q.C;
  if (n_open == 0 || loop >= Q.mp) return false;
  const int lane = tid & 63, wave = tid >> 6;
  const int last = n_open - 1;
  // the last entry (moved into the winner's place) does not depend on the scan: loaded first
  double fl = 0.0, gl = 0.0, stl = 0.0, tuvl = 0.0;
  long long sl = 0, il = 0;
  int lid = 0, rwl = -1;
  if (tid < 64) {
    fl = Q.of[base + last];
    gl = Q.og[base + last];
    sl = Q.oseq[base + last];
    il = Q.oix[base + last];
    lid = Q.oid[base + last];
    rwl = Q.orw[base + last];
    if (lane < 3) {
      stl = Q.ost[(base + last) * 3 + lane];
      if (TUV) tuvl = Q.otuv[(base + last) * 3 + lane];
    }
  }
  double bf = __builtin_inf();
  long long bs = 0x7fffffffffffffffLL;
  int bp = -1;
  int pid = 0, prw = -1;
  double pg = 0.0, pix = 0.0, p0s = 0.0, p1s = 0.0, p2s = 0.0, pt0 = 0.0, pt1 = 0.0, pt2 = 0.0;
  for (int p0 = tid; p0 < n_open; p0 += 4 * NT) {
    double fv[4];
    long long sv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int p = p0 + u * NT;
      fv[u] = p < n_open ? Q.of[base + p] : 0.0;
      sv[u] = p < n_open ? Q.oseq[base + p] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int p = p0 + u * NT;
      if (p < n_open && (bp < 0 || key_before(fv[u], sv[u], bf, bs))) { bf = fv[u]; bs = sv[u]; bp = p; }
    }
  }
  // the thread's own best entry's payload, loaded now so that its latency hides behind the reductions
  // (no dependent load after the winner is known)
  if (bp >= 0) {
    pid = Q.oid[base + bp];
    prw = Q.orw[base + bp];
    pg = Q.og[base + bp];
    pix = __longlong_as_double(Q.oix[base + bp]);
    p0s = Q.ost[(base + bp) * 3];
    p1s = Q.ost[(base + bp) * 3 + 1];
    p2s = Q.ost[(base + bp) * 3 + 2];
    if (TUV) {
      pt0 = Q.otuv[(base + bp) * 3];
      pt1 = Q.otuv[(base + bp) * 3 + 1];
      pt2 = Q.otuv[(base + bp) * 3 + 2];
    }
  }
  if (HA_STAMP_CODE && stp) {  // diagnostics: the scan's loads returned (the payload waited for)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(stp + 10, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int own = bp;
  // wave minimum: quad xor 1 / xor 2, half-row and row mirrors, then the four rows by v_readlane
  key_min_dpp<0xB1>(bf, bs, bp);
  key_min_dpp<0x4E>(bf, bs, bp);
  key_min_dpp<0x141>(bf, bs, bp);
  key_min_dpp<0x140>(bf, bs, bp);
  {
    double wf = __longlong_as_double(readlane_l(__double_as_longlong(bf), 0));
    long long ws = readlane_l(bs, 0);
    int wp_ = __builtin_amdgcn_readlane(bp, 0);
#pragma unroll
    for (int r = 1; r < 4; r++) {
      const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(bf), 16 * r));
      const long long os = readlane_l(bs, 16 * r);
      const int op = __builtin_amdgcn_readlane(bp, 16 * r);
      if (op >= 0 && (wp_ < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wp_ = op; }
    }
    bf = wf;
    bs = ws;
    bp = wp_;
  }
  if (lane == 0) { r_f[wave] = bf; r_s[wave] = bs; r_p[wave] = bp; }
  if (bp >= 0 && own == bp) {  // the one lane that scanned the wave's winning position
    r_id[wave] = pid;
    r_rw[wave] = prw;
    if (TUV) {
      r_tuv[wave][0] = pt0;
      r_tuv[wave][1] = pt1;
      r_tuv[wave][2] = pt2;
    }
    r_pay[wave][0] = pg;
    r_pay[wave][1] = pix;
    r_pay[wave][2] = p0s;
    r_pay[wave][3] = p1s;
    r_pay[wave][4] = p2s;
  }
  __syncthreads();
  if (HA_STAMP_CODE && stp)
    __hip_atomic_store(stp + 11, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid >= 64) return true;
  // the block minimum: wave w's winner on lane w of wave 0 (one LDS read per lane, all at once), reduced
  // within the row by the same DPP steps -- not a serial pass over the NT/64 winners (2.9 us for 12 of
  // them in the r04zk stamps)
  static_assert(NT / 64 <= 16, "the wave winners fit one row");
  double cf = __builtin_inf();
  long long cs = 0x7fffffffffffffffLL;
  int cp = -1;
  if (lane < NT / 64) {
    cp = r_p[lane];
    cf = r_f[lane];
    cs = r_s[lane];
  }
  const int mine = cp;
  key_min_dpp<0xB1>(cf, cs, cp);
  key_min_dpp<0x4E>(cf, cs, cp);
  key_min_dpp<0x141>(cf, cs, cp);
  key_min_dpp<0x140>(cf, cs, cp);
  bp = __builtin_amdgcn_readlane(cp, 0);
  const int ww = __builtin_ctzll(__ballot(lane < NT / 64 && mine == bp));
  const int id = r_id[ww];
  const int rww = r_rw[ww];
  const double gw = r_pay[ww][0];
  const long long iw = __double_as_longlong(r_pay[ww][1]);
  const double stw = lane < 3 ? r_pay[ww][2 + lane] : 0.0;
  const double tuvw = TUV && lane < 3 ? r_tuv[ww][lane] : 0.0;
  if (bp != last) {
    if (lane == 0) {
      Q.of[base + bp] = fl;
      Q.oseq[base + bp] = sl;
      Q.oid[base + bp] = lid;
      Q.og[base + bp] = gl;
      Q.oix[base + bp] = il;
      Q.orw[base + bp] = rwl;
      Q.pos[base + lid] = bp;
    }
    if (lane < 3) {
      Q.ost[(base + bp) * 3 + lane] = stl;
      if (TUV) Q.otuv[(base + bp) * 3 + lane] = tuvl;
    }
  }
  if (lane == 0) {
    Q.pos[base + id] = -1;
    Q.sc_i[SI_NOPEN * B + b] = last;
    Q.sc_i[SI_CUR * B + b] = id;
    if (direct) {
      Q.sc_i[SI_LOOP * B + b] = loop + 1;
      Q.pop_seq[(size_t)b * Q.mp + loop] = iw;
    } else {
      *iw_out = iw;
    }
    Q.cur_g[b] = gw;
    Q.cur_ix[b] = iw;
    rw_out[b] = rww;
  }
  if (lane < 3) {
    node_out[3 * b + lane] = stw;
    if (TUV) tuv_out[3 * b + lane] = tuvw;
  }
  return true;
}

// starting node (setup.jl:112-121) and the first popfirst!; block b = scene b
__global__ __launch_bounds__(256) void ha_init_kernel(HaDev P, HaSearch Q, int B, const double* start) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t base = (size_t)b * Q.C;
  for (int c = tid; c < Q.C; c += 256) Q.nid[base + c] = -1;
  const double* s0 = start + 3 * b;
  if (tid == 0) {
    const long long si = encode(P, s0);  // 0 when the start is outside stbound
    Q.parent[base] = -1;
    for (int r = 0; r < 3; r++) Q.st[base * 3 + r] = s0[r];
    Q.index[base] = si;
    Q.g[base] = 0.0; Q.h[base] = 0.0; Q.f[base] = 0.0;
    Q.seq[base] = 0;
    Q.pos[base] = 0;
    Q.of[base] = 0.0; Q.oseq[base] = 0; Q.oid[base] = 0;
    Q.rw[base] = -1; Q.orw[base] = -1;  // the start node: RS_connected runs the full search once
    Q.og[base] = 0.0; Q.oix[base] = si;
    for (int r = 0; r < 3; r++) Q.ost[base * 3 + r] = s0[r];
    Q.ctr[b] = 1;
    Q.start_index[b] = si;
    Q.sc_i[SI_NNODES * B + b] = 1;
    Q.sc_i[SI_FOUND * B + b] = 0;
    Q.sc_i[SI_NSTATES * B + b] = 0;
    Q.sc_i[SI_RSLEN * B + b] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    const long long si = Q.start_index[b];
    if (si >= 0 && si < Q.C) Q.nid[base + si] = 0;
  }
  __syncthreads();
  const bool go = ha_pop<256>(Q, B, b, 1, 0, tid, Q.node, Q.node_rw, Q.node_tuv, true, nullptr);  // node buffer 0: iteration 1 reads it
  if (tid == 0) Q.sc_i[SI_ACTIVE * B + b] = go;
}

// One search iteration's bookkeeping for scene b, after ha_iter_kernel wrote the scene's
// RS_connected result and the 62 neighbours (array mode): termination (:259-271) or
// FindNewNode's Dict/open-list updates (:418-446) on wave 0 (neighbour k on lane k), then the
// next popfirst! (whole block).
__device__ void ha_book(const HaDev& P, const HaSearch& Q, const IterArgs& A, int B, int it, int b) {
  __shared__ int s_nopen;
  const int tid = threadIdx.x, lane = tid & 63;
  BTIME(0);
  const size_t base = (size_t)b * Q.C;
  const int np = P.n_prim;
  // one round of independent loads: the scene's counters and wave 0's neighbour record (lane k)
  const int active = Q.sc_i[SI_ACTIVE * B + b];
  const int rs_ok = A.rs_ok[b];
  const int loop = Q.sc_i[SI_LOOP * B + b];
  const int n_open0 = Q.sc_i[SI_NOPEN * B + b];
  const int nn0 = Q.sc_i[SI_NNODES * B + b];
  const long long ctr = Q.ctr[b];
  const double cur_g = Q.cur_g[b];
  const long long cidx = Q.cur_ix[b];
  long long ix = 0;
  int frk = 0, hwk = -1;
  double hk = 0.0, nb0 = 0.0, nb1 = 0.0, nb2 = 0.0;
  double tuvk[3] = {0.0, 0.0, 0.0};
  if (tid < np) {
    ix = A.idx[(size_t)b * np + tid];
    frk = A.fr[(size_t)b * np + tid];
    hk = A.h[(size_t)b * np + tid];
    if (A.hw) hwk = A.hw[(size_t)b * np + tid];
    nb0 = A.nb[((size_t)b * np + tid) * 3];
    nb1 = A.nb[((size_t)b * np + tid) * 3 + 1];
    nb2 = A.nb[((size_t)b * np + tid) * 3 + 2];
  }
  if (!active) return;
  BTIME(1);
  if (rs_ok) {  // RS_connected: path found -> hybrid_astar_states by the parent chain
    if (tid == 0) {
      Q.sc_i[SI_FOUND * B + b] = 1;
      Q.sc_i[SI_ACTIVE * B + b] = 0;
      Q.sc_i[SI_RSLEN * B + b] = A.rs_len[b];
      double* so = Q.states + (size_t)b * Q.mp * 3;
      int c = Q.sc_i[SI_CUR * B + b], ns = 0;
      for (int r = 0; r < 3; r++) so[r] = Q.st[(base + c) * 3 + r];
      ns++;
      while (Q.parent[base + c] >= 0 && Q.index[base + c] != Q.start_index[b] && ns < Q.mp) {
        const long long pc = Q.parent[base + c];
        c = (pc >= 0 && pc < Q.C) ? Q.nid[base + pc] : -1;
        if (c < 0) break;
        for (int r = 0; r < 3; r++) so[3 * ns + r] = Q.st[(base + c) * 3 + r];
        ns++;
      }
      Q.sc_i[SI_NSTATES * B + b] = ns;
    }
    return;
  }
  BTIME(2);
  // ---- FindNewNode (:391-447): only the first valid occurrence of an Encode index in this
  // expansion can change anything (every neighbour has the same tentative g).  Lane k of wave 0 is
  // neighbour k; it is a duplicate when an earlier valid lane holds the same Encode index.  The 64
  // comparisons per lane are split over the block's four waves (wave w: earlier lanes 16w..16w+15,
  // broadcast LDS reads), while wave 0 already loads the Dict entries of its valid lanes (loads
  // only: the Dict changes after the check), so their latency overlaps the check.
  __shared__ long long s_vix[64];
  __shared__ int s_dup[BKT / 64][64];
  static_assert(BKT == 256, "the duplicate check below ORs four wave partials");
  const bool valid = tid < np && ix != 0 && frk;
  if (tid < 64) s_vix[tid] = valid ? ix : 0;
  __syncthreads();
  {
    const int w = tid >> 6;
    const long long key = s_vix[lane];  // lane's own index if valid, else 0 (never a duplicate then)
    bool d = false;
#pragma unroll
    for (int jj = 0; jj < 16; jj++) {  // unconditional reads: no exec-masked branch per j
      const int j = 16 * w + jj;
      const long long oj = s_vix[j];
      d = d | ((oj == key) & (j < lane) & (key != 0));
    }
    s_dup[w][lane] = d;
  }
  int hit = -1;
  double gd = 0.0, fo_ = 0.0, dst0 = 0.0, dst1 = 0.0, dst2 = 0.0;
  int po = 0, drw = -1;
  double dtuv[3] = {0.0, 0.0, 0.0};
  long long so0 = 0, io = 0;
  if (valid) {  // wave 0: the Dict entry of every valid lane (used by the first occurrences below)
    hit = (ix >= 0 && ix < Q.C) ? Q.nid[base + ix] : -1;
    if (hit >= 0) {
      gd = Q.g[base + hit];
      po = Q.pos[base + hit];
      fo_ = Q.f[base + hit];
      so0 = Q.seq[base + hit];
      io = Q.index[base + hit];
      drw = Q.rw[base + hit];
#pragma unroll
      for (int e = 0; e < 3; e++) dtuv[e] = 0.0;  // (no RSH units in the split shape: no node has (t, u, v))
      dst0 = Q.st[(base + hit) * 3];
      dst1 = Q.st[(base + hit) * 3 + 1];
      dst2 = Q.st[(base + hit) * 3 + 2];
    }
  }
  BTIME(8);
  __syncthreads();
  if (tid < 64) {
    int n_open = n_open0;
    const int k = lane;
    const bool dup = s_dup[0][k] | s_dup[1][k] | s_dup[2][k] | s_dup[3][k];
    const bool first = valid && !dup;
    BTIME(3);
    const double tg = cur_g + P.expand_time;
    double th = 0.0, tf = 0.0;
    int id = -1;
    bool chg = false, app = false, isnew = false;
    double fo = 0.0;
    long long so_ = 0;
    double nst0 = 0.0, nst1 = 0.0, nst2 = 0.0;  // the node's state and Encode index (its open entry)
    long long nix = ix;
    int nrw = hwk;  // the node's stored rs_heuristic winner (its open entry carries it)
    double nt0 = tuvk[0], nt1 = tuvk[1], nt2 = tuvk[2];
    if (first) {
      th = __builtin_fmax(hk, 0.0);
      if (hk != hk) th = hk;
      tf = tg + th;
      if (hit >= 0) {
        id = hit;
        nst0 = dst0;
        nst1 = dst1;
        nst2 = dst2;
        nix = io;
        nrw = drw;
        nt0 = dtuv[0];
        nt1 = dtuv[1];
        nt2 = dtuv[2];
        if (tg < gd) {
          if (po >= 0) {
            chg = true;
            fo = fo_;
            so_ = so0;
          } else {
            app = true;
          }
        }
      } else {
        isnew = true;
        app = true;
        nst0 = nb0;
        nst1 = nb1;
        nst2 = nb2;
      }
    }
    BTIME(4);
    const unsigned long long m_new = __ballot(isnew), m_chg = __ballot(chg), m_app = __ballot(app);
    const unsigned long long below = (1ull << k) - 1;  // lanes < k
    const int n_new = __popcll(m_new), n_chg = __popcll(m_chg), n_app = __popcll(m_app);
    if (isnew) id = nn0 + __popcll(m_new & below);
    // in-place updates keep their previous list order: rank by the old key among the changed
    int r = 0;
    for (unsigned long long m = m_chg; m; m &= m - 1) {
      const int j = __builtin_ctzll(m);
      const double fj = __shfl(fo, j);
      const long long sj = __shfl(so_, j);
      r += chg && key_before(fj, sj, fo, so_);
    }
    long long nseq = 0;
    if (chg) nseq = ctr + r;
    else if (app) nseq = ctr + n_chg + __popcll(m_app & below);  // then push! in neighbour order
    if (chg || app) {
      const size_t q = base + id;
      if (isnew) {
        Q.st[q * 3] = nst0;
        Q.st[q * 3 + 1] = nst1;
        Q.st[q * 3 + 2] = nst2;
        Q.index[q] = ix;
        Q.rw[q] = nrw;
        if (ix > 0 && ix < Q.C) Q.nid[base + ix] = id;
      }
      Q.g[q] = tg;
      Q.h[q] = th;
      Q.f[q] = tf;
      Q.parent[q] = cidx;
      Q.seq[q] = nseq;
      const int p = chg ? Q.pos[q] : n_open + __popcll(m_app & below);
      Q.of[base + p] = tf;
      Q.oseq[base + p] = nseq;
      Q.og[base + p] = tg;
      if (!chg) {
        Q.oid[base + p] = id;
        Q.oix[base + p] = nix;
        Q.orw[base + p] = nrw;
        Q.ost[(base + p) * 3] = nst0;
        Q.ost[(base + p) * 3 + 1] = nst1;
        Q.ost[(base + p) * 3 + 2] = nst2;
        Q.pos[q] = p;
      }
    }
    n_open += n_app;
    if (lane == 0) {
      Q.sc_i[SI_NNODES * B + b] = nn0 + n_new;
      Q.ctr[b] = ctr + n_chg + n_app;
      s_nopen = n_open;
    }
  }
  BTIME(5);
  __syncthreads();  // the open-list writes of wave 0 before the block-wide scan
  BTIME(6);
  const int n_open = s_nopen;
  // ---- next popfirst!
  const bool go = ha_pop<BKT, false>(Q, B, b, n_open, loop, tid, Q.node + (size_t)(it & 1) * 3 * B, Q.node_rw + (size_t)(it & 1) * B,
                            Q.node_tuv + (size_t)(it & 1) * 3 * B, true,
                            nullptr);
  BTIME(7);
  if (tid == 0) {
    if (go) Q.lst[(it & 1) * B + atomicAdd(Q.live + it, 1)] = b;
    else {
      Q.sc_i[SI_ACTIVE * B + b] = 0;
      Q.sc_i[SI_NOPEN * B + b] = n_open;
    }
  }
}

__global__ __launch_bounds__(BKT) void ha_book_kernel(HaDev P, HaSearch Q, IterArgs A, int B, int it) {
  // the scenes live entering this iteration: the list the previous iteration's bookkeeping wrote
  // (iteration 1: every scene, inactive ones return at once)
  if (A.n_live && (int)blockIdx.x >= *A.n_live) return;
  ha_book(P, Q, A, B, it, A.scene_of ? A.scene_of[blockIdx.x] : (int)blockIdx.x);
}

// ---------------------------------------------------------------- fused iteration (ha_step_kernel)
// One launch per search iteration does the expansion AND the bookkeeping.  FindNewNode (:418-446) and
// the next popfirst! need only the 62 neighbour records, not RS_connected's answer, so the last of a
// scene's neighbour-group blocks to finish runs them at once, speculatively, beside the scene's
// RS_connected block (the iteration's longest chain).  Whichever of the two arrives second at the
// scene's final ticket finishes the iteration: RS_connected found a path -> the termination of
// :259-271 (the speculative pop is undone: its pop count, node count and pop_seq entry are never
// published, and the Dict changes of a finished scene are never read again; the parent chain it walks
// cannot have changed: FindNewNode only re-parents nodes whose g exceeds the popped node's, and every
// ancestor's g is below it); else the pop's results are published and the scene re-listed.  Records
// cross blocks through agent-coherent stores (st_ag), each writer's stores acknowledged (s_waitcnt)
// before its arrival ticket.

// every store of this thread acknowledged at the device coherence point; also a compiler barrier
__device__ __forceinline__ void ha_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

enum { RC_GO = 0, RC_LOOP, RC_NN0, RC_NNEW, RC_NOPEN, RC_CUR, RC_IW, RC_N = 8 };
#ifndef HA_FIN_SHORTCUT
#define HA_FIN_SHORTCUT 1  // the bookkeeping block arriving second finishes with its own values
#endif
// the bookkeeping's results for the scene's finisher (valid in thread 0)
struct BookRec {
  long long v[RC_N];
};

// FindNewNode + popfirst! for scene b on an NT-thread block (ha_book without its termination branch):
// the neighbour records are read agent-coherently; the node count, the pop count and pop_seq go to the
// scene's record (Q.rec) for the finisher instead of the scene's counters.
template <int NT, bool RSH = false>
__device__ __forceinline__ BookRec ha_book_spec(const HaDev& P, const HaSearch& Q, const IterArgs& A, int B, int it,
                                                int b, unsigned long long* stp = nullptr) {
#define BSTAMP(i) if (stp) __hip_atomic_store(stp + (i), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
  __shared__ int s_nopen, s_nnew, s_merged;
  __shared__ long long s_iw;
  __shared__ long long s_vix[64];
  __shared__ int s_dup[4][64];
  static_assert(NT >= 256, "the duplicate check below runs on four waves");
  const int tid = threadIdx.x, lane = tid & 63;
  const size_t base = (size_t)b * Q.C;
  const int np = P.n_prim;
  const int loop = Q.sc_i[SI_LOOP * B + b];
  const int n_open0 = Q.sc_i[SI_NOPEN * B + b];
  const int nn0 = Q.sc_i[SI_NNODES * B + b];
  const int cur0 = Q.sc_i[SI_CUR * B + b];
  const long long ctr = Q.ctr[b];
  const double cur_g = Q.cur_g[b];
  const long long cidx = Q.cur_ix[b];
  long long ix = 0;
  int frk = 0, hwk = -1;
  double hk = 0.0, nb0 = 0.0, nb1 = 0.0, nb2 = 0.0;
  double tuvk[3] = {0.0, 0.0, 0.0};
  if (tid < np) {
    const size_t q = (size_t)b * np + tid;
    ix = ld_ag(A.idx + q);
    frk = ld_ag(A.fr + q);
    if (RSH) {  // rs_heuristic from its four word chunks (ha_iter_body's RSH units): the least (cost, id)
      double cv[4], ct[4][3];
      int ci[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        cv[c] = ld_ag(A.hp_c + q * 4 + c);
        ci[c] = ld_ag(A.hp_i + q * 4 + c);
#pragma unroll
        for (int e = 0; e < 3; e++) ct[c][e] = ld_ag(A.hp_t + (q * 4 + c) * 3 + e);
      }
      double v = cv[0];
      int id = ci[0], wc = 0;
#pragma unroll
      for (int c = 1; c < 4; c++)
        if (rs_before(cv[c], ci[c], v, id)) { v = cv[c]; id = ci[c]; wc = c; }
      hk = v * P.minR;  // rs_heuristic = opt_cost * minR (:365-367), as the groups form it
      // the winner and its (t, u, v): RS_connected's commands when this neighbour becomes a node and is popped
      hwk = A.no_tuv ? id : id | RW_TUV | (v < __builtin_inf() ? RW_OK : 0);
#pragma unroll
      for (int e = 0; e < 3; e++) tuvk[e] = ct[0][e];
#pragma unroll
      for (int c = 1; c < 4; c++)
        if (wc == c)
#pragma unroll
          for (int e = 0; e < 3; e++) tuvk[e] = ct[c][e];
    } else {
      hk = ld_ag(A.h + q);
      if (A.hw) hwk = ld_ag(A.hw + q);
      if (A.full_tuv && hwk >= 0) {  // (the groups stored the winner's (t, u, v))
        hwk |= RW_TUV | (hk < __builtin_inf() ? RW_OK : 0);
#pragma unroll
        for (int e = 0; e < 3; e++) tuvk[e] = ld_ag(A.hp_t + q * 12 + e);
      }
    }
    nb0 = ld_ag(A.nb + 3 * q);
    nb1 = ld_ag(A.nb + 3 * q + 1);
    nb2 = ld_ag(A.nb + 3 * q + 2);
  }
  // (RSH) the prescan record (wave 0, one word per lane) and the last old open entry (lane f: field f), both
  // read now so their latency hides behind the Dict loads and FindNewNode
  long long recw = 0, lastw = 0;
  if (RSH && tid < 64) {
    if (lane < PRE_W) recw = ld_ag(Q.pre + (size_t)b * PRE_W + lane);
    if (n_open0 > 0 && lane < PRE_E) {
      const size_t L = base + n_open0 - 1;
      switch (lane) {
        case 0: lastw = __double_as_longlong(Q.of[L]); break;
        case 1: lastw = Q.oseq[L]; break;
        case 2: lastw = L - base; break;
        case 3: lastw = Q.oid[L]; break;
        case 4: lastw = __double_as_longlong(Q.og[L]); break;
        case 5: lastw = Q.oix[L]; break;
        case 6: case 7: case 8: lastw = __double_as_longlong(Q.ost[L * 3 + lane - 6]); break;
        case 9: lastw = Q.orw[L]; break;
        default: lastw = __double_as_longlong(Q.otuv[L * 3 + lane - 10]); break;
      }
    }
  }
  // duplicates: lane k of wave 0 is neighbour k; an earlier valid lane with the same Encode index makes
  // it one (the comparisons split over four waves, as in ha_book)
  const bool valid = tid < np && ix != 0 && frk;
  if (tid < 64) s_vix[tid] = valid ? ix : 0;
  __syncthreads();
  if (tid < 256) {
    const int w = tid >> 6;
    const long long key = s_vix[lane];
    bool d = false;
#pragma unroll
    for (int jj = 0; jj < 16; jj++) {
      const int j = 16 * w + jj;
      const long long oj = s_vix[j];
      d = d | ((oj == key) & (j < lane) & (key != 0));
    }
    s_dup[w][lane] = d;
  }
  int hit = -1;
  double gd = 0.0, fo_ = 0.0, dst0 = 0.0, dst1 = 0.0, dst2 = 0.0;
  int po = 0, drw = -1;
  double dtuv[3] = {0.0, 0.0, 0.0};
  long long so0 = 0, io = 0;
  if (HA_DREC_CODE && valid && !RSH && A.drec && A.dnid) {  // the groups' copies of the Dict entries
    const long long* r = A.drec + ((size_t)b * np + tid) * HA_DREC;
    long long w[HA_DREC];
#pragma unroll
    for (int e = 0; e < HA_DREC; e++) w[e] = ld_ag(r + e);
    hit = (int)w[0];
    if (hit >= 0) {
      gd = __longlong_as_double(w[1]);
      po = (int)w[2];
      fo_ = __longlong_as_double(w[3]);
      so0 = w[4];
      io = w[5];
      drw = (int)w[6];
      dst0 = __longlong_as_double(w[7]);
      dst1 = __longlong_as_double(w[8]);
      dst2 = __longlong_as_double(w[9]);
    }
  } else if (valid) {
    hit = (ix >= 0 && ix < Q.C) ? Q.nid[base + ix] : -1;
    if (hit >= 0) {
      gd = Q.g[base + hit];
      po = Q.pos[base + hit];
      fo_ = Q.f[base + hit];
      so0 = Q.seq[base + hit];
      io = Q.index[base + hit];
      drw = Q.rw[base + hit];
#pragma unroll
      for (int e = 0; e < 3; e++) dtuv[e] = (RSH || HA_FULL_TUV_CODE) ? Q.tuv[(base + hit) * 3 + e] : 0.0;
      dst0 = Q.st[(base + hit) * 3];
      dst1 = Q.st[(base + hit) * 3 + 1];
      dst2 = Q.st[(base + hit) * 3 + 2];
    }
  }
  __syncthreads();
  BSTAMP(6);
  if (tid < 64) {
    int n_open = n_open0;
    const int k = lane;
    const bool dup = s_dup[0][k] | s_dup[1][k] | s_dup[2][k] | s_dup[3][k];
    const bool first = valid && !dup;
    const double tg = cur_g + P.expand_time;
    double th = 0.0, tf = 0.0;
    int id = -1;
    bool chg = false, app = false, isnew = false;
    double fo = 0.0;
    long long so_ = 0;
    double nst0 = 0.0, nst1 = 0.0, nst2 = 0.0;
    long long nix = ix;
    int nrw = hwk;  // the node's stored rs_heuristic winner (its open entry carries it)
    double nt0 = tuvk[0], nt1 = tuvk[1], nt2 = tuvk[2];
    if (first) {
      th = __builtin_fmax(hk, 0.0);
      if (hk != hk) th = hk;
      tf = tg + th;
      if (hit >= 0) {
        id = hit;
        nst0 = dst0;
        nst1 = dst1;
        nst2 = dst2;
        nix = io;
        nrw = drw;
        nt0 = dtuv[0];
        nt1 = dtuv[1];
        nt2 = dtuv[2];
        if (tg < gd) {
          if (po >= 0) {
            chg = true;
            fo = fo_;
            so_ = so0;
          } else {
            app = true;
          }
        }
      } else {
        isnew = true;
        app = true;
        nst0 = nb0;
        nst1 = nb1;
        nst2 = nb2;
      }
    }
    const unsigned long long m_new = __ballot(isnew), m_chg = __ballot(chg), m_app = __ballot(app);
    const unsigned long long below = (1ull << k) - 1;
    const int n_new = __popcll(m_new), n_chg = __popcll(m_chg), n_app = __popcll(m_app);
    if (isnew) id = nn0 + __popcll(m_new & below);
    int r = 0;
    for (unsigned long long m = m_chg; m; m &= m - 1) {
      const int j = __builtin_ctzll(m);
      const double fj = __shfl(fo, j);
      const long long sj = __shfl(so_, j);
      r += chg && key_before(fj, sj, fo, so_);
    }
    long long nseq = 0;
    if (chg) nseq = ctr + r;
    else if (app) nseq = ctr + n_chg + __popcll(m_app & below);
    if (chg || app) {
      const size_t q = base + id;
      if (isnew) {
        Q.st[q * 3] = nst0;
        Q.st[q * 3 + 1] = nst1;
        Q.st[q * 3 + 2] = nst2;
        Q.index[q] = ix;
        Q.rw[q] = nrw;
        if (RSH || HA_FULL_TUV_CODE) {
          Q.tuv[q * 3] = nt0;
          Q.tuv[q * 3 + 1] = nt1;
          Q.tuv[q * 3 + 2] = nt2;
        }
        if (ix > 0 && ix < Q.C) Q.nid[base + ix] = id;
      }
      Q.g[q] = tg;
      Q.h[q] = th;
      Q.f[q] = tf;
      Q.parent[q] = cidx;
      Q.seq[q] = nseq;
      const int p = chg ? po : n_open + __popcll(m_app & below);  // po = Q.pos[q] (nothing moved it yet)
      Q.of[base + p] = tf;
      Q.oseq[base + p] = nseq;
      Q.og[base + p] = tg;
      if (!chg) {
        Q.oid[base + p] = id;
        Q.oix[base + p] = nix;
        Q.orw[base + p] = nrw;
        if (RSH || HA_FULL_TUV_CODE) {
          Q.otuv[(base + p) * 3] = nt0;
          Q.otuv[(base + p) * 3 + 1] = nt1;
          Q.otuv[(base + p) * 3 + 2] = nt2;
        }
        Q.ost[(base + p) * 3] = nst0;
        Q.ost[(base + p) * 3 + 1] = nst1;
        Q.ost[(base + p) * 3 + 2] = nst2;
        Q.pos[q] = p;
      }
    }
    n_open += n_app;
    if (lane == 0) {
      Q.ctr[b] = ctr + n_chg + n_app;
      s_nopen = n_open;
      s_nnew = nn0 + n_new;
    }
    if (RSH) {
      // ---- popfirst! merged from the prescan (ha_prescan): the least of the record entries FindNewNode left
      // alone, the changed entries (new keys, same positions) and the appended ones
      const int tag = (int)readlane_l(recw, 0), kc = (int)readlane_l(recw, 1);
      // this lane's own candidate: a changed or appended entry
      const int myp = chg ? po : app ? n_open0 + __popcll(m_app & below) : -1;
      double bf = tf;
      long long bs = nseq;
      int bp = myp;
      int bl = myp >= 0 ? lane : -1;  // the lane holding the winner (-1: a record entry)
      // the record's entries FindNewNode left alone (wave-uniform)
      bool any_left = false;
      double rf = 0.0;
      long long rsq = 0;
      int rp = -1, re = -1;
#pragma unroll
      for (int e = 0; e < PRE_K; e++) {
        if (e >= kc) break;
        const int pe = (int)readlane_l(recw, 2 + PRE_E * e + 2);
        if (__ballot(chg && po == pe)) continue;  // changed in place: its new key is a lane candidate
        const double fe = __longlong_as_double(readlane_l(recw, 2 + PRE_E * e));
        const long long se = readlane_l(recw, 2 + PRE_E * e + 1);
        any_left = true;
        if (rp < 0 || key_before(fe, se, rf, rsq)) { rf = fe; rsq = se; rp = pe; re = e; }
      }
      const bool ok_merge = tag == it && (any_left || n_open0 <= kc);
      if (ok_merge) {
        // the lanes' minimum
        int bpl = bp;
        key_min_dpp<0xB1>(bf, bs, bpl);
        key_min_dpp<0x4E>(bf, bs, bpl);
        key_min_dpp<0x141>(bf, bs, bpl);
        key_min_dpp<0x140>(bf, bs, bpl);
        double wf = __longlong_as_double(readlane_l(__double_as_longlong(bf), 0));
        long long ws = readlane_l(bs, 0);
        int wpos = __builtin_amdgcn_readlane(bpl, 0);
#pragma unroll
        for (int q = 1; q < 4; q++) {
          const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(bf), 16 * q));
          const long long os = readlane_l(bs, 16 * q);
          const int op = __builtin_amdgcn_readlane(bpl, 16 * q);
          if (op >= 0 && (wpos < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wpos = op; }
        }
        // vs the record's least untouched entry
        bool from_rec = false;
        if (rp >= 0 && (wpos < 0 || key_before(rf, rsq, wf, ws))) { wpos = rp; from_rec = true; }
        const bool go_ = !(n_open == 0 || loop >= Q.mp);
        if (go_) {
          // the winner's payload: id, g, Encode index, state, rw, (t, u, v)
          int wid, wrw;
          double wg, ws0, ws1, ws2, wt0, wt1, wt2;
          long long wix;
          if (from_rec) {
            const int o = 2 + PRE_E * re;
            wid = (int)readlane_l(recw, o + 3);
            wg = __longlong_as_double(readlane_l(recw, o + 4));
            wix = readlane_l(recw, o + 5);
            ws0 = __longlong_as_double(readlane_l(recw, o + 6));
            ws1 = __longlong_as_double(readlane_l(recw, o + 7));
            ws2 = __longlong_as_double(readlane_l(recw, o + 8));
            wrw = (int)readlane_l(recw, o + 9);
            wt0 = __longlong_as_double(readlane_l(recw, o + 10));
            wt1 = __longlong_as_double(readlane_l(recw, o + 11));
            wt2 = __longlong_as_double(readlane_l(recw, o + 12));
          } else {
            const int wl = __builtin_ctzll(__ballot(myp == wpos && myp >= 0));
            wid = __builtin_amdgcn_readlane(id, wl);
            wg = __longlong_as_double(readlane_l(__double_as_longlong(tg), wl));
            wix = readlane_l(nix, wl);
            ws0 = __longlong_as_double(readlane_l(__double_as_longlong(nst0), wl));
            ws1 = __longlong_as_double(readlane_l(__double_as_longlong(nst1), wl));
            ws2 = __longlong_as_double(readlane_l(__double_as_longlong(nst2), wl));
            wrw = __builtin_amdgcn_readlane(nrw, wl);
            wt0 = __longlong_as_double(readlane_l(__double_as_longlong(nt0), wl));
            wt1 = __longlong_as_double(readlane_l(__double_as_longlong(nt1), wl));
            wt2 = __longlong_as_double(readlane_l(__double_as_longlong(nt2), wl));
          }
          // popfirst!: the last entry moves into the winner's place (ha_pop's removal)
          const int last = n_open - 1;
          if (wpos != last) {
            double lf, lg, l0, l1, l2, lt0, lt1, lt2;
            long long ls, lix;
            int lid, lrw;
            // the last entry is held by a lane when it was appended (the highest appended lane: appends go in
            // lane order) or changed in place by FindNewNode; else it is the old last entry, loaded at the start
            const unsigned long long mlast = __ballot(chg && po == last);
            if (last >= n_open0 || mlast) {  // wave-uniform
              const int hl = last >= n_open0 ? 63 - __builtin_clzll(m_app) : __builtin_ctzll(mlast);
              lf = __longlong_as_double(readlane_l(__double_as_longlong(tf), hl));
              ls = readlane_l(nseq, hl);
              lg = __longlong_as_double(readlane_l(__double_as_longlong(tg), hl));
              lid = __builtin_amdgcn_readlane(id, hl);
              lix = readlane_l(nix, hl);
              l0 = __longlong_as_double(readlane_l(__double_as_longlong(nst0), hl));
              l1 = __longlong_as_double(readlane_l(__double_as_longlong(nst1), hl));
              l2 = __longlong_as_double(readlane_l(__double_as_longlong(nst2), hl));
              lrw = __builtin_amdgcn_readlane(nrw, hl);
              lt0 = __longlong_as_double(readlane_l(__double_as_longlong(nt0), hl));
              lt1 = __longlong_as_double(readlane_l(__double_as_longlong(nt1), hl));
              lt2 = __longlong_as_double(readlane_l(__double_as_longlong(nt2), hl));
            } else {  // the old last entry, untouched by FindNewNode (loaded at the start)
              lf = __longlong_as_double(readlane_l(lastw, 0));
              ls = readlane_l(lastw, 1);
              lid = (int)readlane_l(lastw, 3);
              lg = __longlong_as_double(readlane_l(lastw, 4));
              lix = readlane_l(lastw, 5);
              l0 = __longlong_as_double(readlane_l(lastw, 6));
              l1 = __longlong_as_double(readlane_l(lastw, 7));
              l2 = __longlong_as_double(readlane_l(lastw, 8));
              lrw = (int)readlane_l(lastw, 9);
              lt0 = __longlong_as_double(readlane_l(lastw, 10));
              lt1 = __longlong_as_double(readlane_l(lastw, 11));
              lt2 = __longlong_as_double(readlane_l(lastw, 12));
            }
            if (lane == 0) {
              Q.of[base + wpos] = lf;
              Q.oseq[base + wpos] = ls;
              Q.oid[base + wpos] = lid;
              Q.og[base + wpos] = lg;
              Q.oix[base + wpos] = lix;
              Q.orw[base + wpos] = lrw;
              Q.pos[base + lid] = wpos;
            }
            if (lane < 3) {
              Q.ost[(base + wpos) * 3 + lane] = lane == 0 ? l0 : lane == 1 ? l1 : l2;
              Q.otuv[(base + wpos) * 3 + lane] = lane == 0 ? lt0 : lane == 1 ? lt1 : lt2;
            }
          }
          if (lane == 0) {
            Q.pos[base + wid] = -1;
            Q.sc_i[SI_NOPEN * B + b] = last;
            Q.sc_i[SI_CUR * B + b] = wid;
            Q.cur_g[b] = wg;
            Q.cur_ix[b] = wix;
            Q.node_rw[(size_t)(it & 1) * B + b] = wrw;
            s_iw = wix;
          }
          if (lane < 3) {
            Q.node[(size_t)(it & 1) * 3 * B + 3 * b + lane] = lane == 0 ? ws0 : lane == 1 ? ws1 : ws2;
            Q.node_tuv[(size_t)(it & 1) * 3 * B + 3 * b + lane] = lane == 0 ? wt0 : lane == 1 ? wt1 : wt2;
          }
        }
        if (lane == 0) s_merged = go_ ? 1 : 2;  // 2: popfirst! ends the search here
      } else if (lane == 0) {
        s_merged = 0;
      }
    }
  }
  __syncthreads();  // the open-list writes of wave 0 before the block-wide scan
  BSTAMP(7);
  const int n_open = s_nopen;
  long long iw = 0;
  bool go;
  if (RSH && s_merged) {  // block-uniform
    go = s_merged == 1;
    iw = s_iw;
  } else {
    // (HA_FULL_TUV_CODE: the commands travel with the entry in both shapes, a full-width winner's rw carries RW_TUV)
    go = ha_pop<NT, RSH || HA_FULL_TUV_CODE>(Q, B, b, n_open, loop, tid, Q.node + (size_t)(it & 1) * 3 * B, Q.node_rw + (size_t)(it & 1) * B,
                    Q.node_tuv + (size_t)(it & 1) * 3 * B, false, &iw, stp);
  }
  BSTAMP(8);
  BookRec br;
  br.v[RC_GO] = go;
  br.v[RC_LOOP] = loop;
  br.v[RC_NN0] = nn0;
  br.v[RC_NNEW] = s_nnew;
  br.v[RC_NOPEN] = n_open;
  br.v[RC_CUR] = cur0;
  br.v[RC_IW] = iw;
  br.v[RC_N - 1] = 0;
  if (stp) __hip_atomic_store(stp + 9, (unsigned long long)n_open, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#undef BSTAMP
  return br;
}

// the scene's iteration ends (one thread): the termination of :259-271 when RS_connected found a path,
// else the speculative pop's results published and the scene listed for the next iteration
__device__ __forceinline__ void ha_finish(const HaSearch& Q, const IterArgs& A, int B, int it, int b,
                                          const BookRec& br, bool list = true) {
  const long long* rc = br.v;
  const int go = (int)rc[RC_GO], loop = (int)rc[RC_LOOP];
  const int rs_ok = ld_ag(A.rs_ok + b);
  if (rs_ok) {
    const size_t base = (size_t)b * Q.C;
    Q.sc_i[SI_FOUND * B + b] = 1;
    Q.sc_i[SI_ACTIVE * B + b] = 0;
    Q.sc_i[SI_RSLEN * B + b] = ld_ag(A.rs_len + b);
    Q.sc_i[SI_LOOP * B + b] = loop;
    Q.sc_i[SI_NNODES * B + b] = (int)rc[RC_NN0];
    double* so = Q.states + (size_t)b * Q.mp * 3;
    int c = (int)rc[RC_CUR], ns = 0;
    for (int r = 0; r < 3; r++) so[r] = Q.st[(base + c) * 3 + r];
    ns++;
    while (Q.parent[base + c] >= 0 && Q.index[base + c] != Q.start_index[b] && ns < Q.mp) {
      const long long pc = Q.parent[base + c];
      c = (pc >= 0 && pc < Q.C) ? Q.nid[base + pc] : -1;
      if (c < 0) break;
      for (int r = 0; r < 3; r++) so[3 * ns + r] = Q.st[(base + c) * 3 + r];
      ns++;
    }
    Q.sc_i[SI_NSTATES * B + b] = ns;
    return;
  }
  Q.sc_i[SI_NNODES * B + b] = (int)rc[RC_NNEW];
  if (go) {
    Q.sc_i[SI_LOOP * B + b] = loop + 1;
    Q.pop_seq[(size_t)b * Q.mp + loop] = rc[RC_IW];
    if (list) Q.lst[(it & 1) * B + atomicAdd(Q.live + it, 1)] = b;  // (ha_persist_kernel keeps no list)
  } else {
    Q.sc_i[SI_ACTIVE * B + b] = 0;
    Q.sc_i[SI_NOPEN * B + b] = (int)rc[RC_NOPEN];
  }
}

// (RSH tail) popfirst!'s scan ahead of FindNewNode, on its own block of the scene: the PRE_K least entries of
// the open list as this iteration starts (stream order: the previous bookkeeping's writes are complete), with
// their payloads, into the scene's record (Q.pre).  FindNewNode then changes some entries in place and appends
// others; the least entry after it is the least of the record's entries it left alone, the changed and the
// appended ones -- unless it changed every record entry while more remain (the bookkeeping then scans).
// Every entry outside the record has a key above the record's, so the merge is exact (the key order is total).
// Per thread its PRE_K least entries (insertion), per wave PRE_K rounds of a DPP minimum, then wave 0 over the
// waves' PRE_K each.  Returns false (block-uniform) past the live list.
template <int NT>
__device__ __forceinline__ bool ha_prescan(const HaSearch& Q, const IterArgs& A, int B, int it, int slot,
                                           unsigned long long* hstp = nullptr) {
  static_assert(NT % 64 == 0 && NT / 64 * PRE_K <= 64, "the waves' candidates fit wave 0");
  __shared__ double c_f[NT / 64][PRE_K];
  __shared__ long long c_s[NT / 64][PRE_K];
  __shared__ int c_p[NT / 64][PRE_K];
  const int n_live = A.n_live ? *A.n_live : A.n_active;
  const int b = A.scene_of ? A.scene_of[slot] : slot;
  if (slot >= n_live) return false;
  if (!A.n_live && A.active && !A.active[b]) return false;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = (size_t)b * Q.C;
  if (A.no_pre) {
    if (tid == 0) st_ag(Q.pre + (size_t)b * PRE_W, -1LL);
    return true;
  }
  const int n0 = Q.sc_i[SI_NOPEN * B + b];
  HSTAMP(12);
  double tf[PRE_K];
  long long ts[PRE_K];
  int tp[PRE_K];
#pragma unroll
  for (int e = 0; e < PRE_K; e++) { tf[e] = __builtin_inf(); ts[e] = 0x7fffffffffffffffLL; tp[e] = -1; }
  for (int p0 = tid; p0 < n0; p0 += 2 * NT) {  // two independent entry loads in flight per thread
    double fv[2];
    long long sv[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int p = p0 + u * NT;
      fv[u] = p < n0 ? Q.of[base + p] : 0.0;
      sv[u] = p < n0 ? Q.oseq[base + p] : 0;
    }
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int p = p0 + u * NT;
      if (p >= n0) continue;
      // insertion into the sorted PRE_K (the key order is total: positions are distinct entries)
      double f = fv[u];
      long long sq = sv[u];
      int pp = p;
#pragma unroll
      for (int e = 0; e < PRE_K; e++) {
        if (tp[e] < 0 || key_before(f, sq, tf[e], ts[e])) {
          const double f2 = tf[e];
          const long long s2 = ts[e];
          const int p2 = tp[e];
          tf[e] = f; ts[e] = sq; tp[e] = pp;
          f = f2; sq = s2; pp = p2;
          if (pp < 0) break;
        }
      }
    }
  }
  if (HA_STAMP_CODE && hstp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HSTAMP(13);
  }
  // the wave's PRE_K least: PRE_K rounds of the minimum of the lanes' heads, the owner lane shifting its list
#pragma unroll 1
  for (int r = 0; r < PRE_K; r++) {
    double bf = tf[0];
    long long bs = ts[0];
    int bp = tp[0];
    key_min_dpp<0xB1>(bf, bs, bp);
    key_min_dpp<0x4E>(bf, bs, bp);
    key_min_dpp<0x141>(bf, bs, bp);
    key_min_dpp<0x140>(bf, bs, bp);
    double wf = __longlong_as_double(readlane_l(__double_as_longlong(bf), 0));
    long long ws = readlane_l(bs, 0);
    int wp_ = __builtin_amdgcn_readlane(bp, 0);
#pragma unroll
    for (int q = 1; q < 4; q++) {
      const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(bf), 16 * q));
      const long long os = readlane_l(bs, 16 * q);
      const int op = __builtin_amdgcn_readlane(bp, 16 * q);
      if (op >= 0 && (wp_ < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wp_ = op; }
    }
    if (lane == 0) { c_f[wave][r] = wf; c_s[wave][r] = ws; c_p[wave][r] = wp_; }
    if (wp_ >= 0 && tp[0] == wp_) {  // the owner lane drops its head
#pragma unroll
      for (int e = 0; e + 1 < PRE_K; e++) { tf[e] = tf[e + 1]; ts[e] = ts[e + 1]; tp[e] = tp[e + 1]; }
      tf[PRE_K - 1] = __builtin_inf(); ts[PRE_K - 1] = 0x7fffffffffffffffLL; tp[PRE_K - 1] = -1;
    }
  }
  HSTAMP(14);
  __syncthreads();
  if (tid >= 64) return true;
  // wave 0: the block's PRE_K least of the waves' candidates (lane = wave * PRE_K + rank)
  double cf = __builtin_inf();
  long long cs = 0x7fffffffffffffffLL;
  int cp = -1;
  if (lane < NT / 64 * PRE_K) {
    cf = c_f[lane / PRE_K][lane % PRE_K];
    cs = c_s[lane / PRE_K][lane % PRE_K];
    cp = c_p[lane / PRE_K][lane % PRE_K];
  }
  int mine = -1;  // lane e < kc: the e-th least entry's position
#pragma unroll 1
  for (int r = 0; r < PRE_K; r++) {
    double bf = cf;
    long long bs = cs;
    int bp = cp;
    key_min_dpp<0xB1>(bf, bs, bp);
    key_min_dpp<0x4E>(bf, bs, bp);
    key_min_dpp<0x141>(bf, bs, bp);
    key_min_dpp<0x140>(bf, bs, bp);
    double wf = __longlong_as_double(readlane_l(__double_as_longlong(bf), 0));
    long long ws = readlane_l(bs, 0);
    int wp_ = __builtin_amdgcn_readlane(bp, 0);
#pragma unroll
    for (int q = 1; q < 4; q++) {
      const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(bf), 16 * q));
      const long long os = readlane_l(bs, 16 * q);
      const int op = __builtin_amdgcn_readlane(bp, 16 * q);
      if (op >= 0 && (wp_ < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wp_ = op; }
    }
    if (lane == r) mine = wp_;
    if (wp_ >= 0 && cp == wp_) { cf = __builtin_inf(); cs = 0x7fffffffffffffffLL; cp = -1; }
  }
  const int kc = min(PRE_K, n0);
  HSTAMP(15);
  long long* rec = Q.pre + (size_t)b * PRE_W;
  if (lane < kc && mine >= 0) {  // lane e: entry e and its payload
    const size_t q = base + mine;
    long long w[PRE_E];
    w[0] = __double_as_longlong(Q.of[q]);
    w[1] = Q.oseq[q];
    w[2] = mine;
    w[3] = Q.oid[q];
    w[4] = __double_as_longlong(Q.og[q]);
    w[5] = Q.oix[q];
#pragma unroll
    for (int e = 0; e < 3; e++) w[6 + e] = __double_as_longlong(Q.ost[q * 3 + e]);
    w[9] = Q.orw[q];
#pragma unroll
    for (int e = 0; e < 3; e++) w[10 + e] = __double_as_longlong(Q.otuv[q * 3 + e]);
#pragma unroll
    for (int e = 0; e < PRE_E; e++) st_ag(rec + 2 + PRE_E * lane + e, w[e]);
  }
  if (lane == 0) {
    st_ag(rec + 1, (long long)kc);
    st_ag(rec + 0, (long long)it);
  }
  HSTAMP(16);
  return true;
}


// ---------------------------------------------------------------- pipelined tail (ha_pipe_kernel)
// The expansion of a node (its 62 neighbour records) is a function of the node's state alone, and the next
// popfirst! is a function of the records, the Dict and the open list as they stand before FindNewNode writes:
// the least of the entries FindNewNode leaves alone, the ones it changes in place (new keys) and the ones it
// appends.  So launch it of the pipelined tail runs, per scene:
//   item 0   RS_connected(n_it), as before;
//   item 1   the bookkeeping: the records of n_it (expanded by the previous launch, E[it & 1]), FindNewNode's
//            decisions, the open list scan excluding the positions it changes, the pop of n_{it+1} -- published
//            (state, stored commands, a ready flag) before FindNewNode's writes -- then the writes, the removal,
//            and the final ticket with RS_connected, as ha_step_kernel's bookkeeping block;
//   items 2+ the expansion of n_{it+1} (the RSH groups and word units), into E[(it + 1) & 1] for launch it+1,
//            started as soon as the pop is published (they spin on the flag: their blocks follow the
//            bookkeeping's in dispatch order, so it is running or done).
// The chain per iteration is the bookkeeping's pop decision + the expansion, instead of the expansion + the
// whole bookkeeping.  Same operations on the same values as ha_step_kernel: the same search, bit for bit.
// A bootstrap launch (boot = 1) expands the current nodes only, for the first pipelined launch.

// E[par]: the expansion-record buffers hold two parities of [B][n_prim][...]
__device__ __forceinline__ IterArgs e_par(const IterArgs& A, int B, int np, int par) {
  IterArgs E = A;
  const size_t n = (size_t)B * np * par;
  E.idx = A.idx + n;
  E.fr = A.fr + n;
  E.nb = A.nb + 3 * n;
  E.hp_c = A.hp_c + 4 * n;
  E.hp_i = A.hp_i + 4 * n;
  E.hp_t = A.hp_t + 12 * n;
  E.h = A.h + n;  // (full-width pipe) rs_heuristic and its winner per neighbour
  E.hw = A.hw ? A.hw + n : nullptr;
  return E;
}

// pre_wait (ha_persist_kernel): the wait for this iteration's expansion records, run after the open list's loads
// are issued (the list stands as the previous iteration's bookkeeping left it) so they land meanwhile.
// SPEC (ha_persist_kernel, HA_SPEC): also the runner-up -- the second-least of popfirst!'s candidates, which is
// the next pop unless one of the popped node's children beats it (87 % of the pops of configs[3]) -- published
// as Q.ngr2 granules after the writes; sr (LDS, kept by the caller across iterations) holds the previous one
// (10 payload words + valid), and the pop's go word carries skip = hit (the popped node IS the previous
// runner-up, identical id, state and stored commands: its expansion and RS_connected were made speculatively);
// *hit_out returns it.
template <int NT, bool RSH = true, class Wait = NoMid, bool SPEC = false>
__device__ __forceinline__ BookRec ha_book_pipe(const HaDev& P, const HaSearch& Q, const IterArgs& E, int B, int it,
                                                int b, unsigned long long* stp = nullptr, const Wait& pre_wait = Wait(),
                                                long long* sr = nullptr, int* hit_out = nullptr) {
#define PSTAMP(i) if (stp) __hip_atomic_store(stp + (i), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
  constexpr int SC = 4;  // open entries per thread held in registers (more are re-read)
  __shared__ int s_nopen, s_nnew, s_nchg, s_go;
  __shared__ int s_chg[64];  // positions FindNewNode changes in place
  __shared__ long long s_vix[64];
  __shared__ int s_dup[4][64];
  __shared__ double r_f[NT / 64];
  __shared__ long long r_s[NT / 64];
  __shared__ int r_p[NT / 64];
  __shared__ long long r_pay[NT / 64][11];  // each wave winner's payload: id, g, ix, st[3], rw, tuv[3]
  __shared__ long long s_win[12];           // the pop's winner: payload as r_pay, position, (SPEC) hit
  // (SPEC) the runner-up: each wave's candidate and its payload (staged by the candidate's owner thread)
  __shared__ double u_f[SPEC ? NT / 64 : 1];
  __shared__ long long u_s[SPEC ? NT / 64 : 1];
  __shared__ int u_p[SPEC ? NT / 64 : 1];
  __shared__ long long u_pay[SPEC ? NT / 64 : 1][10];
  static_assert(NT >= 256 && NT / 64 <= 16, "four waves for the duplicate check, the wave winners fit a row");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = (size_t)b * Q.C;
  const int np = P.n_prim;
  const int loop = Q.sc_i[SI_LOOP * B + b];
  const int n_open0 = Q.sc_i[SI_NOPEN * B + b];
  const int nn0 = Q.sc_i[SI_NNODES * B + b];
  const int cur0 = Q.sc_i[SI_CUR * B + b];
  const long long ctr = Q.ctr[b];
  const double cur_g = Q.cur_g[b];
  const long long cidx = Q.cur_ix[b];
  // the open list as it stands (loads in flight while the records and the Dict come in)
  double fv[SC];
  long long sv[SC];
  // (loaded before n_open0 is known: positions past it are read -- inside the scene's C entries -- and masked)
#pragma unroll
  for (int u = 0; u < SC; u++) {
    const int p = tid + u * NT;
    fv[u] = p < Q.C ? Q.of[base + p] : 0.0;
    sv[u] = p < Q.C ? Q.oseq[base + p] : 0;
  }
  pre_wait();
  // n_it's neighbour records (expanded by the previous launch)
  long long ix = 0;
  int frk = 0, hwk = -1;
  double hk = 0.0, nb0 = 0.0, nb1 = 0.0, nb2 = 0.0;
  double tuvk[3] = {0.0, 0.0, 0.0};
  if (tid < np) {
    const size_t q = (size_t)b * np + tid;
    ix = ld_ag(E.idx + q);
    frk = ld_ag(E.fr + q);
    if (RSH) {
      double cv[4], ct[4][3];
      int ci[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        cv[c] = ld_ag(E.hp_c + q * 4 + c);
        ci[c] = ld_ag(E.hp_i + q * 4 + c);
#pragma unroll
        for (int e = 0; e < 3; e++) ct[c][e] = ld_ag(E.hp_t + (q * 4 + c) * 3 + e);
      }
      double v = cv[0];
      int id = ci[0], wc = 0;
#pragma unroll
      for (int c = 1; c < 4; c++)
        if (rs_before(cv[c], ci[c], v, id)) { v = cv[c]; id = ci[c]; wc = c; }
      hk = v * P.minR;
      hwk = E.no_tuv ? id : id | RW_TUV | (v < __builtin_inf() ? RW_OK : 0);
#pragma unroll
      for (int e = 0; e < 3; e++) tuvk[e] = ct[0][e];
#pragma unroll
      for (int c = 1; c < 4; c++)
        if (wc == c)
#pragma unroll
          for (int e = 0; e < 3; e++) tuvk[e] = ct[c][e];
    } else {  // the full-width groups' own rs_heuristic and winner (as ha_book_spec<NT, false>)
      hk = ld_ag(E.h + q);
      if (E.hw) hwk = ld_ag(E.hw + q);
      if (E.full_tuv && hwk >= 0) {
        hwk |= RW_TUV | (hk < __builtin_inf() ? RW_OK : 0);
#pragma unroll
        for (int e = 0; e < 3; e++) tuvk[e] = ld_ag(E.hp_t + q * 12 + e);
      }
    }
    nb0 = ld_ag(E.nb + 3 * q);
    nb1 = ld_ag(E.nb + 3 * q + 1);
    nb2 = ld_ag(E.nb + 3 * q + 2);
  }
  const bool valid = tid < np && ix != 0 && frk;
  if (tid < 64) s_vix[tid] = valid ? ix : 0;
  __syncthreads();
  if (tid < 256) {
    const int w = tid >> 6;
    const long long key = s_vix[lane];
    bool d = false;
#pragma unroll
    for (int jj = 0; jj < 16; jj++) {
      const int j = 16 * w + jj;
      const long long oj = s_vix[j];
      d = d | ((oj == key) & (j < lane) & (key != 0));
    }
    s_dup[w][lane] = d;
  }
  int hit = -1;
  double gd = 0.0, fo_ = 0.0, dst0 = 0.0, dst1 = 0.0, dst2 = 0.0;
  int po = 0, drw = -1;
  double dtuv[3] = {0.0, 0.0, 0.0};
  long long so0 = 0, io = 0;
  if (valid) {
    hit = (ix >= 0 && ix < Q.C) ? Q.nid[base + ix] : -1;
    if (hit >= 0) {
      gd = Q.g[base + hit];
      po = Q.pos[base + hit];
      fo_ = Q.f[base + hit];
      so0 = Q.seq[base + hit];
      io = Q.index[base + hit];
      drw = Q.rw[base + hit];
#pragma unroll
      for (int e = 0; e < 3; e++) dtuv[e] = Q.tuv[(base + hit) * 3 + e];
      dst0 = Q.st[(base + hit) * 3];
      dst1 = Q.st[(base + hit) * 3 + 1];
      dst2 = Q.st[(base + hit) * 3 + 2];
    }
  }
  __syncthreads();
  PSTAMP(6);
  // ---- FindNewNode's decisions (:418-446) on wave 0 (lane k = neighbour k), no writes yet
  const double tg = cur_g + P.expand_time;
  double th = 0.0, tf = 0.0;
  int id = -1;
  bool chg = false, app = false, isnew = false;
  double nst0 = 0.0, nst1 = 0.0, nst2 = 0.0;
  long long nix = ix, nseq = 0;
  int nrw = hwk, myp = -1;
  double nt0 = tuvk[0], nt1 = tuvk[1], nt2 = tuvk[2];
  unsigned long long m_new = 0, m_chg = 0, m_app = 0;
  int n_app = 0, n_open = n_open0;
  if (tid < 64) {
    const int k = lane;
    const bool dup = s_dup[0][k] | s_dup[1][k] | s_dup[2][k] | s_dup[3][k];
    const bool first = valid && !dup;
    double fo = 0.0;
    long long so_ = 0;
    if (first) {
      th = __builtin_fmax(hk, 0.0);
      if (hk != hk) th = hk;
      tf = tg + th;
      if (hit >= 0) {
        id = hit;
        nst0 = dst0; nst1 = dst1; nst2 = dst2;
        nix = io;
        nrw = drw;
        nt0 = dtuv[0]; nt1 = dtuv[1]; nt2 = dtuv[2];
        if (tg < gd) {
          if (po >= 0) { chg = true; fo = fo_; so_ = so0; }
          else app = true;
        }
      } else {
        isnew = true;
        app = true;
        nst0 = nb0; nst1 = nb1; nst2 = nb2;
      }
    }
    m_new = __ballot(isnew);
    m_chg = __ballot(chg);
    m_app = __ballot(app);
    const unsigned long long below = (1ull << k) - 1;
    const int n_chg = __popcll(m_chg);
    n_app = __popcll(m_app);
    if (isnew) id = nn0 + __popcll(m_new & below);
    int r = 0;
    for (unsigned long long m = m_chg; m; m &= m - 1) {
      const int j = __builtin_ctzll(m);
      const double fj = __shfl(fo, j);
      const long long sj = __shfl(so_, j);
      r += chg && key_before(fj, sj, fo, so_);
    }
    if (chg) nseq = ctr + r;
    else if (app) nseq = ctr + n_chg + __popcll(m_app & below);
    myp = chg ? po : app ? n_open0 + __popcll(m_app & below) : -1;
    if (chg) s_chg[__popcll(m_chg & below)] = po;
    n_open = n_open0 + n_app;
    if (lane == 0) {
      s_nchg = n_chg;
      s_nopen = n_open;
      s_nnew = nn0 + __popcll(m_new);
    }
  }
  __syncthreads();
  // ---- the old entries FindNewNode leaves alone: each thread's least (positions it changes excluded)
  const int nchg = s_nchg;
  auto changed = [&](int p) {
    bool c = false;
    for (int i = 0; i < nchg; i++) c |= s_chg[i] == p;
    return c;
  };
  double bf = __builtin_inf(), bf2 = __builtin_inf();
  long long bs = 0x7fffffffffffffffLL, bs2 = 0x7fffffffffffffffLL;
  int bp = -1, bp2 = -1;  // (SPEC) the thread's second-least too
  auto consider = [&](double f, long long sq, int p) {
    if (bp < 0 || key_before(f, sq, bf, bs)) {
      if (SPEC) { bf2 = bf; bs2 = bs; bp2 = bp; }
      bf = f; bs = sq; bp = p;
    } else if (SPEC && (bp2 < 0 || key_before(f, sq, bf2, bs2))) {
      bf2 = f; bs2 = sq; bp2 = p;
    }
  };
#pragma unroll
  for (int u = 0; u < SC; u++) {
    const int p = tid + u * NT;
    if (p < n_open0 && !changed(p)) consider(fv[u], sv[u], p);
  }
  for (int p = tid + SC * NT; p < n_open0; p += NT) {  // long lists: the rest re-read
    const double f = Q.of[base + p];
    const long long sq = Q.oseq[base + p];
    if (!changed(p)) consider(f, sq, p);
  }
  const double own_f = bf;  // (SPEC) the thread's least, before the reductions overwrite bf / bs / bp
  const long long own_s = bs;
  // the thread's own best entry's payload, its latency behind the reductions
  long long pay[11];
#pragma unroll
  for (int e = 0; e < 11; e++) pay[e] = 0;
  if (bp >= 0) {
    const size_t q = base + bp;
    pay[0] = Q.oid[q];
    pay[1] = __double_as_longlong(Q.og[q]);
    pay[2] = Q.oix[q];
#pragma unroll
    for (int e = 0; e < 3; e++) pay[3 + e] = __double_as_longlong(Q.ost[q * 3 + e]);
    pay[6] = Q.orw[q];
#pragma unroll
    for (int e = 0; e < 3; e++) pay[7 + e] = __double_as_longlong(Q.otuv[q * 3 + e]);
  }
  const int own = bp;
  key_min_dpp<0xB1>(bf, bs, bp);
  key_min_dpp<0x4E>(bf, bs, bp);
  key_min_dpp<0x141>(bf, bs, bp);
  key_min_dpp<0x140>(bf, bs, bp);
  {
    double wf = __longlong_as_double(readlane_l(__double_as_longlong(bf), 0));
    long long ws = readlane_l(bs, 0);
    int wp_ = __builtin_amdgcn_readlane(bp, 0);
#pragma unroll
    for (int q = 1; q < 4; q++) {
      const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(bf), 16 * q));
      const long long os = readlane_l(bs, 16 * q);
      const int op = __builtin_amdgcn_readlane(bp, 16 * q);
      if (op >= 0 && (wp_ < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wp_ = op; }
    }
    if (lane == 0) { r_f[wave] = wf; r_s[wave] = ws; r_p[wave] = wp_; }
    if (wp_ >= 0 && own == wp_) {
#pragma unroll
      for (int e = 0; e < 10; e++) r_pay[wave][e] = pay[e];
    }
  }
  __syncthreads();
  PSTAMP(7);
  // ---- popfirst! (wave 0): the least of the waves' winners (lanes < NT/64) and the lanes' changed / appended
  // entries -- a lane offers the better of the two it holds
  if (tid < 64) {
    double cf = __builtin_inf();
    long long cs = 0x7fffffffffffffffLL;
    int cp = -1, src = -1;  // src: wave index of an old winner, 64 + lane for a lane candidate
    if (lane < NT / 64 && r_p[lane] >= 0) { cf = r_f[lane]; cs = r_s[lane]; cp = r_p[lane]; src = lane; }
    if (myp >= 0 && (cp < 0 || key_before(tf, nseq, cf, cs))) { cf = tf; cs = nseq; cp = myp; src = 64 + lane; }
    const int mine = cp, msrc = src;
    key_min_dpp<0xB1>(cf, cs, cp);
    key_min_dpp<0x4E>(cf, cs, cp);
    key_min_dpp<0x141>(cf, cs, cp);
    key_min_dpp<0x140>(cf, cs, cp);
    double wf = __longlong_as_double(readlane_l(__double_as_longlong(cf), 0));
    long long ws = readlane_l(cs, 0);
    int wpos = __builtin_amdgcn_readlane(cp, 0);
#pragma unroll
    for (int q = 1; q < 4; q++) {
      const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(cf), 16 * q));
      const long long os = readlane_l(cs, 16 * q);
      const int op = __builtin_amdgcn_readlane(cp, 16 * q);
      if (op >= 0 && (wpos < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wpos = op; }
    }
    const bool go = !(n_open == 0 || loop >= Q.mp);
    // the winner's lane writes its payload to LDS (an old entry's from its wave record, a lane's own values)
    if (go && mine == wpos && mine >= 0) {
      if (msrc < 64) {
#pragma unroll
        for (int e = 0; e < 10; e++) s_win[e] = r_pay[msrc][e];
      } else {
        s_win[0] = id;
        s_win[1] = __double_as_longlong(tg);
        s_win[2] = nix;
        s_win[3] = __double_as_longlong(nst0);
        s_win[4] = __double_as_longlong(nst1);
        s_win[5] = __double_as_longlong(nst2);
        s_win[6] = nrw;
        s_win[7] = __double_as_longlong(nt0);
        s_win[8] = __double_as_longlong(nt1);
        s_win[9] = __double_as_longlong(nt2);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the winner's LDS writes before the wave reads them
    // (SPEC) the pop is the previous runner-up: same node id, state and stored commands (the inputs of its
    // expansion and of RS_connected), so both were made speculatively
    bool hit = false;
    if (SPEC && go && sr[10]) {
      hit = s_win[0] == sr[0];
#pragma unroll
      for (int e = 3; e < 10; e++) hit = hit && s_win[e] == sr[e];
    }
    if (RSH && E.ngr_pub) {
      // publish the next node as tagged granules (ha_publish_node): no drain, no separate flag; the node
      // buffers too, for the next launch's RS_connected (a launch boundary orders those)
      long long wv[10];
#pragma unroll
      for (int e = 0; e < 10; e++) wv[e] = go ? s_win[e] : 0;
      ha_publish_node(Q.ngr + ((size_t)(it & (HA_NGR_SLOTS - 1)) * B + b) * HA_NGR, (unsigned)it + 1, lane, wv,
                      go ? 1u | (hit ? 2u : 0u) : 0u);
      if (go && lane < 3) {
        Q.node[(size_t)(it & 1) * 3 * B + 3 * b + lane] = __longlong_as_double(s_win[3 + lane]);
        Q.node_tuv[(size_t)(it & 1) * 3 * B + 3 * b + lane] = __longlong_as_double(s_win[7 + lane]);
      }
      if (go && lane == 0) Q.node_rw[(size_t)(it & 1) * B + b] = (int)s_win[6];
    } else {
      if (go) {
        // publish the next node: state, stored commands, then the ready flag (the expansion blocks spin on it)
        if (lane < 3) {
          st_ag(Q.node + (size_t)(it & 1) * 3 * B + 3 * b + lane, __longlong_as_double(s_win[3 + lane]));
          st_ag(Q.node_tuv + (size_t)(it & 1) * 3 * B + 3 * b + lane, __longlong_as_double(s_win[7 + lane]));
        }
        if (lane == 0) st_ag(Q.node_rw + (size_t)(it & 1) * B + b, (int)s_win[6]);
        if (!RSH && lane == 1) st_ag(Q.node_g + (size_t)(it & 1) * B + b, __longlong_as_double(s_win[1]));
        if (!RSH && lane == 2) st_ag(Q.node_nn + (size_t)(it & 1) * B + b, nn0);
      }
      ha_stores_done();
      if (lane == 0) st_ag(Q.nx + b, 2 * it + 2 + (go ? 1 : 0));
    }
    if (lane == 0) {
      s_go = go;
      s_win[10] = wpos;
      if (SPEC) s_win[11] = hit;
    }
    PSTAMP(8);
  }
  if (SPEC) {
    // ---- the runner-up: the least of the same candidates without the winner -- each thread's least old entry
    // (its second when its least won) and, in wave 0, the lanes' changed / appended entries, reduced per wave
    // here, before FindNewNode's writes; wave 1 takes the least of the waves' beside wave 0's writes, off the
    // iteration's chain.  The candidate's owner stages its payload: a lane's own entry, the thread's least from
    // the registers the pop's scan filled, its second from the open list (read before this iteration's writes)
    __syncthreads();  // the pop's position and go
    const int wpos = (int)s_win[10];
    if (s_go) {  // block-uniform
      double cf = own_f;
      long long cs = own_s;
      int cp = own;
      if (own >= 0 && own == wpos) { cf = bf2; cs = bs2; cp = bp2; }
      bool cl = false;
      if (myp >= 0 && myp != wpos && (cp < 0 || key_before(tf, nseq, cf, cs))) { cf = tf; cs = nseq; cp = myp; cl = true; }
      const int cand = cp;
      key_min_dpp<0xB1>(cf, cs, cp);
      key_min_dpp<0x4E>(cf, cs, cp);
      key_min_dpp<0x141>(cf, cs, cp);
      key_min_dpp<0x140>(cf, cs, cp);
      double wf = __longlong_as_double(readlane_l(__double_as_longlong(cf), 0));
      long long ws = readlane_l(cs, 0);
      int wp_ = __builtin_amdgcn_readlane(cp, 0);
#pragma unroll
      for (int q = 1; q < 4; q++) {
        const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(cf), 16 * q));
        const long long os = readlane_l(cs, 16 * q);
        const int op = __builtin_amdgcn_readlane(cp, 16 * q);
        if (op >= 0 && (wp_ < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; wp_ = op; }
      }
      if (lane == 0) { u_f[wave] = wf; u_s[wave] = ws; u_p[wave] = wp_; }
      if (wp_ >= 0 && cand == wp_) {
        long long* u = u_pay[SPEC ? wave : 0];
        if (cl) {
          u[0] = id;
          u[1] = __double_as_longlong(tg);
          u[2] = nix;
          u[3] = __double_as_longlong(nst0);
          u[4] = __double_as_longlong(nst1);
          u[5] = __double_as_longlong(nst2);
          u[6] = nrw;
          u[7] = __double_as_longlong(nt0);
          u[8] = __double_as_longlong(nt1);
          u[9] = __double_as_longlong(nt2);
        } else if (cand == own) {
#pragma unroll
          for (int e = 0; e < 10; e++) u[e] = pay[e];
        } else {
          const size_t q = base + cand;
          u[0] = Q.oid[q];
          u[1] = __double_as_longlong(Q.og[q]);
          u[2] = Q.oix[q];
#pragma unroll
          for (int e = 0; e < 3; e++) u[3 + e] = __double_as_longlong(Q.ost[q * 3 + e]);
          u[6] = Q.orw[q];
#pragma unroll
          for (int e = 0; e < 3; e++) u[7 + e] = __double_as_longlong(Q.otuv[q * 3 + e]);
        }
      }
    }
    __syncthreads();
  }
  if (tid < 64) {
    const bool go = s_go;
    const int wpos = (int)s_win[10];
    // ---- FindNewNode's writes (as ha_book_spec)
    if (chg || app) {
      const size_t q = base + id;
      if (isnew) {
        Q.st[q * 3] = nst0;
        Q.st[q * 3 + 1] = nst1;
        Q.st[q * 3 + 2] = nst2;
        Q.index[q] = ix;
        Q.rw[q] = nrw;
        Q.tuv[q * 3] = nt0;
        Q.tuv[q * 3 + 1] = nt1;
        Q.tuv[q * 3 + 2] = nt2;
        if (ix > 0 && ix < Q.C) Q.nid[base + ix] = id;
      }
      Q.g[q] = tg;
      Q.h[q] = th;
      Q.f[q] = tf;
      Q.parent[q] = cidx;
      Q.seq[q] = nseq;
      const int p = myp;
      Q.of[base + p] = tf;
      Q.oseq[base + p] = nseq;
      Q.og[base + p] = tg;
      if (!chg) {
        Q.oid[base + p] = id;
        Q.oix[base + p] = nix;
        Q.orw[base + p] = nrw;
        Q.otuv[(base + p) * 3] = nt0;
        Q.otuv[(base + p) * 3 + 1] = nt1;
        Q.otuv[(base + p) * 3 + 2] = nt2;
        Q.ost[(base + p) * 3] = nst0;
        Q.ost[(base + p) * 3 + 1] = nst1;
        Q.ost[(base + p) * 3 + 2] = nst2;
        Q.pos[q] = p;
      }
    }
    if (lane == 0) Q.ctr[b] = ctr + __popcll(m_chg) + n_app;
    // ---- popfirst!'s removal: the last entry moves into the winner's place (ha_pop)
    if (go) {
      const int last = n_open - 1;
      const int wid = (int)s_win[0];
      if (wpos != last) {
        // the last entry: appended (the highest appending lane), changed in place, or the old one (lane 0)
        const unsigned long long mlast = __ballot(chg && po == last);
        const int hl = last >= n_open0 ? 63 - __builtin_clzll(m_app) : mlast ? __builtin_ctzll(mlast) : 0;
        if (lane == hl) {
          const bool own_vals = last >= n_open0 || mlast;
          // the old last entry (read only now: off the pop's publication path)
          double Lf = 0.0, Lg = 0.0, Ls0 = 0.0, Ls1 = 0.0, Ls2 = 0.0, Lt0 = 0.0, Lt1 = 0.0, Lt2 = 0.0;
          long long Lsq = 0, Lix = 0;
          int Lid = 0, Lrw = -1;
          if (!own_vals) {
            const size_t L = base + n_open0 - 1;
            Lf = Q.of[L]; Lsq = Q.oseq[L]; Lid = Q.oid[L]; Lg = Q.og[L]; Lix = Q.oix[L]; Lrw = Q.orw[L];
            Ls0 = Q.ost[L * 3]; Ls1 = Q.ost[L * 3 + 1]; Ls2 = Q.ost[L * 3 + 2];
            Lt0 = Q.otuv[L * 3]; Lt1 = Q.otuv[L * 3 + 1]; Lt2 = Q.otuv[L * 3 + 2];
          }
          const double f_ = own_vals ? tf : Lf, g_ = own_vals ? tg : Lg;
          const long long s_ = own_vals ? nseq : Lsq, x_ = own_vals ? nix : Lix;
          const int i_ = own_vals ? id : Lid, w_ = own_vals ? nrw : Lrw;
          const size_t d = base + wpos;
          Q.of[d] = f_;
          Q.oseq[d] = s_;
          Q.oid[d] = i_;
          Q.og[d] = g_;
          Q.oix[d] = x_;
          Q.orw[d] = w_;
          Q.ost[d * 3] = own_vals ? nst0 : Ls0;
          Q.ost[d * 3 + 1] = own_vals ? nst1 : Ls1;
          Q.ost[d * 3 + 2] = own_vals ? nst2 : Ls2;
          Q.otuv[d * 3] = own_vals ? nt0 : Lt0;
          Q.otuv[d * 3 + 1] = own_vals ? nt1 : Lt1;
          Q.otuv[d * 3 + 2] = own_vals ? nt2 : Lt2;
          Q.pos[base + i_] = wpos;
        }
      }
      if (lane == 0) {
        Q.pos[base + wid] = -1;
        Q.sc_i[SI_NOPEN * B + b] = last;
        Q.sc_i[SI_CUR * B + b] = wid;
        Q.cur_g[b] = __longlong_as_double(s_win[1]);
        Q.cur_ix[b] = s_win[2];
      }
    }
  } else if (SPEC && tid < 128 && s_go) {
    // ---- (wave 1) the runner-up: the least of the waves' candidates, its payload into sr, then its granules
    double cf = __builtin_inf();
    long long cs = 0x7fffffffffffffffLL;
    int cp = -1;
    if (lane < NT / 64 && u_p[lane] >= 0) { cf = u_f[lane]; cs = u_s[lane]; cp = u_p[lane]; }
    const int mine = cp;
    key_min_dpp<0xB1>(cf, cs, cp);
    key_min_dpp<0x4E>(cf, cs, cp);
    key_min_dpp<0x141>(cf, cs, cp);
    key_min_dpp<0x140>(cf, cs, cp);
    double wf = __longlong_as_double(readlane_l(__double_as_longlong(cf), 0));
    long long ws = readlane_l(cs, 0);
    int rpos = __builtin_amdgcn_readlane(cp, 0);
#pragma unroll
    for (int q = 1; q < 4; q++) {
      const double of_ = __longlong_as_double(readlane_l(__double_as_longlong(cf), 16 * q));
      const long long os = readlane_l(cs, 16 * q);
      const int op = __builtin_amdgcn_readlane(cp, 16 * q);
      if (op >= 0 && (rpos < 0 || key_before(of_, os, wf, ws))) { wf = of_; ws = os; rpos = op; }
    }
    if (rpos >= 0 && mine == rpos) {  // the owner lane (lane = the candidate's wave)
#pragma unroll
      for (int e = 0; e < 10; e++) sr[e] = u_pay[SPEC ? lane : 0][e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the owner's LDS writes before the wave reads them
    const bool valid = rpos >= 0;
    long long wv[10];
#pragma unroll
    for (int e = 0; e < 10; e++) wv[e] = valid ? sr[e] : 0;
    // skip (no runner-up): the speculative blocks count the round and wait for the next one
    ha_publish_node(Q.ngr2 + ((size_t)(it & (HA_NGR_SLOTS - 1)) * B + b) * HA_NGR, (unsigned)it + 1, lane, wv,
                    valid ? 1u : 3u);
    if (lane == 0) sr[10] = valid;
  }
  __syncthreads();
  if (SPEC) {
    if (hit_out) *hit_out = s_go ? (int)s_win[11] : 0;
    if (tid == 0 && s_go) {  // (diagnostics: MPGPU_HA_SPEC_STATS=1 prints the sums)
      Q.nhit[b] += (int)s_win[11];
      Q.nhit[B + b] += (int)sr[10];
    }
  }
  BookRec br;
  br.v[RC_GO] = s_go;
  br.v[RC_LOOP] = loop;
  br.v[RC_NN0] = nn0;
  br.v[RC_NNEW] = s_nnew;
  br.v[RC_NOPEN] = s_nopen;
  br.v[RC_CUR] = cur0;
  br.v[RC_IW] = s_go ? s_win[2] : 0;
  br.v[RC_N - 1] = 0;
#undef PSTAMP
  return br;
}

// Waves per SIMD each shape is compiled for.  The full-width shape (4-wave blocks, 1,280 of them at 256
// scenes) is occupancy-bound: 133 VGPRs would allow 3 waves per SIMD; 4 costs 20 B of spills and gains
// 0.3 ms per plan (r04zc: 29.7 vs 30.0 ms; round 4 had drifted to 169 VGPRs, 2 waves, 31.5 ms).  The
// tail shape's 12-wave blocks take one CU each either way (6 waves: 80 VGPRs + spills, 0.2 ms slower).
#ifndef HA_WPE_FULL
#define HA_WPE_FULL 4
#endif
#ifndef HA_WPE_TAIL
#define HA_WPE_TAIL 1
#endif
constexpr int HA_STAMP_EVERY = 25, HA_STAMP_N = 17;  // [6..11]: bookkeeping phases; [12..16]: block body phases
template <int HWt, int NBGt, bool RSH = false>
// (the 6-wave middle shape at 3 waves per SIMD -- 139 VGPRs, no spills, still two blocks per CU -- measured 1.4 ms
// slower per 256-plan than at 4 with 128 VGPRs and spills, r05zp; kept at 4)
#ifndef HA_WPE_MID
#define HA_WPE_MID 4
#endif
__global__ __launch_bounds__(64 * HWt) __attribute__((amdgpu_waves_per_eu(HWt == HW_TAIL ? HA_WPE_TAIL : HWt == 6 ? HA_WPE_MID : HA_WPE_FULL))) void ha_step_kernel(HaDev P, HaSearch Q, IterArgs A, int B, int it) {
  __shared__ int role;
  unsigned long long* stp = nullptr;
  if (HA_STAMP_CODE && A.stamps && it % HA_STAMP_EVERY == 0 && it / HA_STAMP_EVERY < 40 && (int)blockIdx.x < A.stamp_blocks &&
      threadIdx.x == 0)
    stp = A.stamps + ((size_t)(it / HA_STAMP_EVERY) * A.stamp_blocks + blockIdx.x) * HA_STAMP_N;
  if (stp) __hip_atomic_store(stp, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ha_mirror(A, it);
  const int per = 1 + (P.n_prim + NBGt - 1) / NBGt + (RSH ? 1 : 0);
  int slot = blockIdx.x / per, item = blockIdx.x % per;
  if (!RSH && A.rs_last) {  // the RS_connected blocks after every neighbour group in dispatch order
    const int n = gridDim.x / per, G = per - 1, bid = blockIdx.x;
    if (bid < n * G) { slot = bid / G; item = 1 + bid % G; }
    else { slot = bid - n * G; item = 0; }
  }
  if (RSH && item == per - 1) {  // the prescan block: counted among the bookkeeping's arrivals
    if (!ha_prescan<64 * HWt>(Q, A, B, it, slot, stp)) return;
  } else if (!ha_iter_body<HWt, NBGt, RSH>(P, A, stp, slot, item)) {
    return;  // block-uniform: no work for this block (not counted)
  }
  const int s = A.scene_of ? A.scene_of[slot] : slot;
  ha_stores_done();  // this thread's records acknowledged before the block's ticket
  __syncthreads();
  if (stp) __hip_atomic_store(stp + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) {
    int r = 2;  // RS_connected: straight to the final ticket
    if (item > 0) {
      const int t = __hip_atomic_fetch_add(Q.tk + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r = t == per - 2 ? 1 : 0;  // the last of the neighbour groups does the bookkeeping
      if (r) st_ag(Q.tk + s, 0);
    }
    role = r;
  }
  __syncthreads();
  const int r = role;
  if (stp) {
    __hip_atomic_store(stp + 2, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(stp + 5, (unsigned long long)r | ((unsigned long long)s << 4) | ((unsigned long long)item << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (r == 0) return;
  // The final ticket (two arrivals: this scene's RS_connected block and its bookkeeping block, so the launch
  // needs do_rs && do_exp -- mp_ha_plan checks it).  The bookkeeping block takes it before publishing anything: arriving second (the
  // usual case) it finishes with its own values; arriving first it publishes its record and then a
  // ready flag, which the RS_connected block, arriving second, waits for (a short wait: the bookkeeping
  // block is running and publishes without waiting on anything).
  long long* rc = Q.rec + (size_t)RC_N * s;
  if (r == 1) {
    const BookRec br = ha_book_spec<64 * HWt, RSH>(P, Q, A, B, it, s, stp);
    if (!HA_FIN_SHORTCUT) {  // (A/B) always publish the record first
      if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < RC_N - 1; i++) st_ag(rc + i, br.v[i]);
        ha_stores_done();
        st_ag(rc + RC_N - 1, 1LL);
        if (__hip_atomic_fetch_add(Q.tk + B + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
          asm volatile("" ::: "memory");
          st_ag(Q.tk + B + s, 0);
          st_ag(rc + RC_N - 1, 0LL);
          ha_finish(Q, A, B, it, s, br);
        }
      }
      return;
    }
    if (threadIdx.x == 0) {
      if (stp) __hip_atomic_store(stp + 3, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(Q.tk + B + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
        asm volatile("" ::: "memory");
        st_ag(Q.tk + B + s, 0);
        ha_finish(Q, A, B, it, s, br);
        if (stp) __hip_atomic_store(stp + 4, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
#pragma unroll
        for (int i = 0; i < RC_N - 1; i++) st_ag(rc + i, br.v[i]);
        ha_stores_done();
        st_ag(rc + RC_N - 1, 1LL);  // record ready
      }
    }
    return;
  }
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(Q.tk + B + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
    asm volatile("" ::: "memory");
    st_ag(Q.tk + B + s, 0);
    while (ld_ag(rc + RC_N - 1) == 0) __builtin_amdgcn_s_sleep(1);
    BookRec br;
#pragma unroll
    for (int i = 0; i < RC_N - 1; i++) br.v[i] = ld_ag(rc + i);
    st_ag(rc + RC_N - 1, 0LL);  // consumed: the next iteration's bookkeeping block sets it again
    ha_finish(Q, A, B, it, s, br);
    if (stp) __hip_atomic_store(stp + 4, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}



// ha_pipe_kernel: the pipelined tail's launch (see above).  Items per slot: 0 RS_connected(n_it), 1 the
// bookkeeping, 2 .. 1 + n_groups the expansion of n_{it+1}.  boot = 1: only the expansion, of n_it itself
// (node buffer (it - 1) & 1) into E[it & 1], for the first pipelined launch.
template <int HWt, int NBGt, bool RSH = true>
__global__ __launch_bounds__(64 * HWt) __attribute__((amdgpu_waves_per_eu(HWt == 4 ? HA_WPE_FULL : HA_WPE_TAIL))) void ha_pipe_kernel(
    HaDev P, HaSearch Q, IterArgs A, int B, int it, int boot) {
  __shared__ int role, sh_go;
  unsigned long long* stp = nullptr;
  if (HA_STAMP_CODE && A.stamps && !boot && it % HA_STAMP_EVERY == 0 && it / HA_STAMP_EVERY < 40 &&
      (int)blockIdx.x < A.stamp_blocks && threadIdx.x == 0)
    stp = A.stamps + ((size_t)(it / HA_STAMP_EVERY) * A.stamp_blocks + blockIdx.x) * HA_STAMP_N;
  if (stp) __hip_atomic_store(stp, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!boot) ha_mirror(A, it);
  const int ng = (P.n_prim + NBGt - 1) / NBGt, per = 2 + ng;
  const int slot = blockIdx.x / per, item = blockIdx.x % per;
  const int n_live = A.n_live ? *A.n_live : A.n_active;
  if (slot >= n_live) return;
  const int s = A.scene_of ? A.scene_of[slot] : slot;
  if (!A.n_live && A.active && !A.active[s]) return;
  const int np = P.n_prim;
  if (item >= 2) {  // the expansion of n_{it+1} (boot: of n_it) into E[(it + 1) & 1] (boot: E[it & 1])
    IterArgs X = e_par(A, B, np, boot ? (it & 1) : ((it + 1) & 1));
    if (!boot) {  // wait for the bookkeeping's pop (its block precedes this one in dispatch order)
      X.node = Q.node + (size_t)(it & 1) * 3 * B;
      X.node_ag = 1;
      X.node_flag = Q.nx;
      X.node_flag_min = 2 * it + 2;
      X.node_flag_err = Q.err;
      if (!RSH) {  // the Dict pre-check beside FindNewNode's writes (ha_iter_body)
        X.node_g = Q.node_g + (size_t)(it & 1) * B;
        X.node_nn = Q.node_nn + (size_t)(it & 1) * B;
      } else if (A.ngr_pub) {  // the node as tagged granules
        X.ngr = Q.ngr + (size_t)(it & (HA_NGR_SLOTS - 1)) * B * HA_NGR;
        X.ngr_tag = (unsigned)it + 1;
      }
    }
    X.do_rs = 0;
    ha_iter_body<HWt, NBGt, RSH>(P, X, stp, slot, item - 1);
    if (stp) {
      __hip_atomic_store(stp + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(stp + 5, ((unsigned long long)s << 4) | ((unsigned long long)(item - 1) << 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (boot) return;
  if (item == 0) {
    if (!ha_iter_body<HWt, NBGt, RSH>(P, A, stp, slot, 0)) return;
    ha_stores_done();
    __syncthreads();
  }
  if (stp) __hip_atomic_store(stp + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (stp) __hip_atomic_store(stp + 5, (unsigned long long)(item == 0 ? 2 : 1) | ((unsigned long long)s << 4) |
                                           ((unsigned long long)(item == 0 ? 0 : 17) << 32),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the final ticket: RS_connected (item 0) and the bookkeeping (item 1), as in ha_step_kernel
  long long* rc = Q.rec + (size_t)RC_N * s;
  if (item == 1) {
    const BookRec br = ha_book_pipe<64 * HWt, RSH>(P, Q, e_par(A, B, np, it & 1), B, it, s, stp);
    if (threadIdx.x == 0) {
      if (stp) __hip_atomic_store(stp + 3, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(Q.tk + B + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
        asm volatile("" ::: "memory");
        st_ag(Q.tk + B + s, 0);
        ha_finish(Q, A, B, it, s, br);
        if (stp) __hip_atomic_store(stp + 4, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
#pragma unroll
        for (int i = 0; i < RC_N - 1; i++) st_ag(rc + i, br.v[i]);
        ha_stores_done();
        st_ag(rc + RC_N - 1, 1LL);  // record ready
      }
    }
    return;
  }
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(Q.tk + B + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
    asm volatile("" ::: "memory");
    st_ag(Q.tk + B + s, 0);
    while (ld_ag(rc + RC_N - 1) == 0) __builtin_amdgcn_s_sleep(1);
    BookRec br;
#pragma unroll
    for (int i = 0; i < RC_N - 1; i++) br.v[i] = ld_ag(rc + i);
    st_ag(rc + RC_N - 1, 0LL);
    ha_finish(Q, A, B, it, s, br);
    if (stp) __hip_atomic_store(stp + 4, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


// ha_persist_kernel: the pipelined tail as ONE launch for the rest of the search, once every block of it can be
// resident at once (cooperative launch): per scene two RS_connected blocks (even / odd iterations), the
// bookkeeping block and the expansion groups each loop over the iterations, handing over through per-scene flags
// instead of launch boundaries -- the bookkeeping publishes n_{it+1} (tagged granules), the groups expand it into
// E[(it+1) & 1] and count themselves in (Q.ex), RS_connected(n_it) signals its verdict (Q.rsr by it & 1; verdict and
// path in the iteration's parity buffer); the bookkeeping of iteration it waits for E[it & 1] and RS_connected(n_it) and finishes the
// iteration as ha_step_kernel's finisher.  A finished scene publishes HA_DONE: every block of it leaves its loop.
// Same operations on the same values as ha_pipe_kernel: the same search, bit for bit.  Every wait is bounded.
// HA_SPEC (default 1): the speculative runner-up (ha_book_pipe<..., SPEC>).  The bookkeeping of iteration it also
// publishes r_{it+1}, the second-least of popfirst!'s candidates (Q.ngr2): the next pop is r_{it+1} or one of
// n_{it+1}'s children (the least of the two), and in configs[3] it is r_{it+1} for 87 % of the pops.  The
// expansion groups, after n_{it+1}, expand r_{it+1} into E slot 2 + ((it+1) & 3) (Q.exs, by the parity of it+1), the
// RS block of iteration it, after RS_connected(n_it), runs RS_connected(r_it) into RS slot 2 + (it & 3) (Q.rsrs).
// When the pop IS the runner-up (same node id, state and stored commands: the inputs of both), its granules carry
// skip, the groups and the RS block skip it and the bookkeeping reads the speculative records instead: the lone
// chain per hit iteration is then the bookkeeping (~14 us) instead of expansion + bookkeeping.  The same records, the same decisions:
// the search is bit for bit the same (the expansion and RS_connected are functions of the node alone).
#ifndef HA_SPEC
#define HA_SPEC 1
#endif
// blocks per scene of the persistent launch: two RS_connected blocks, the bookkeeping, ng expansion groups
#define HA_PERSIST_PER(ng) (3 + (ng))
template <int HWt, int NBGt, bool SPEC = HA_SPEC>
__global__ __launch_bounds__(64 * HWt) __attribute__((amdgpu_waves_per_eu(HWt == HW_TAIL ? HA_WPE_TAIL : 3))) void ha_persist_kernel(
    HaDev P, HaSearch Q, IterArgs A, int B, int it0, double* rs_path2, unsigned char* rs_ok2, int* rs_len2) {
  __shared__ int sh_f;
  __shared__ long long sh_run[12];  // (SPEC, the bookkeeping block) the last runner-up: payload + valid
  // per scene: item 0 / 2 RS_connected of the even / odd iterations, item 1 the bookkeeping, items 3.. the groups
  const int np = P.n_prim, ng = (np + NBGt - 1) / NBGt, per = HA_PERSIST_PER(ng);
  const int slot = blockIdx.x / per, item = blockIdx.x % per;
  const int n_live = A.n_live ? *A.n_live : A.n_active;
  if (slot >= n_live) return;
  const int s = A.scene_of ? A.scene_of[slot] : slot;
  if (!A.n_live && A.active && !A.active[s]) return;
  // RS_connected's outputs by slot: 0 / 1 the pop's (iteration parity), 2..5 the runner-up's (SPEC, it & 3) -- the
  // next iteration's may be written before the bookkeeping reads this one's
  auto rs_slot = [&](IterArgs& X, int k) {
    X.rs_ok = rs_ok2 + (size_t)k * B;
    X.rs_len = rs_len2 + (size_t)k * B;
    X.rs_path = rs_path2 + (size_t)k * B * MAXPATH * 3;
  };
  // (HA_STAMP_CODE builds, MPGPU_HA_STAMPS=1) this block's stamp record for iteration it, as ha_step_kernel's
  auto pst = [&](int it) -> unsigned long long* {
    if (!HA_STAMP_CODE || !A.stamps || it % HA_STAMP_EVERY || it / HA_STAMP_EVERY >= 40 ||
        (int)blockIdx.x >= A.stamp_blocks || threadIdx.x)
      return nullptr;
    return A.stamps + ((size_t)(it / HA_STAMP_EVERY) * A.stamp_blocks + blockIdx.x) * HA_STAMP_N;
  };
  auto now = [] { return __builtin_amdgcn_s_memrealtime(); };
  auto put = [](unsigned long long* p, int i, unsigned long long v) {
    if (p) __hip_atomic_store(p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (item >= 3) {  // the expansion of n_{it+1} (skipped when it is the runner-up), then (SPEC) of r_{it+1}
#ifndef HA_GROUP_PRIO
#define HA_GROUP_PRIO 2
#endif
    if (HA_GROUP_PRIO) __builtin_amdgcn_s_setprio(HA_GROUP_PRIO);
    for (int it = it0;; it++) {
      unsigned long long* stp0 = pst(it);  // (stamps: the r job's start / end in slots 6 / 7 of the n job's record)
      for (int job = 0; job < (SPEC ? 2 : 1); job++) {  // (one body for both: a loop, not two inlined copies)
        const bool r = SPEC && job == 1;
        if (r) put(stp0, 6, now());
        IterArgs X = e_par(A, B, np, r ? 2 + ((it + 1) & 3) : (it + 1) & 1);
        X.node = Q.node + (size_t)(it & 1) * 3 * B;
        X.node_ag = 1;
        X.node_flag = Q.nx;
        X.node_flag_min = 2 * it + 2;
        X.node_flag_err = Q.err;
        if (A.ngr_pub || r) {
          X.ngr = (r ? Q.ngr2 : Q.ngr) + (size_t)(it & (HA_NGR_SLOTS - 1)) * B * HA_NGR;
          X.ngr_tag = (unsigned)it + 1;
        }
        X.do_rs = 0;
        unsigned long long* stp = r ? nullptr : pst(it);
        put(stp, 0, now());
        if (!ha_iter_body<HWt, NBGt, true>(P, X, stp, slot, item - 2)) return;  // the search ended
        ha_stores_done();
        __syncthreads();
        // (the runner-up rounds count by the parity of the runner-up's iteration, see the bookkeeping's wait)
        if (threadIdx.x == 0)
          __hip_atomic_fetch_add(r ? Q.exs + (size_t)((it + 1) & 1) * B + s : Q.ex + s, 1, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        if (r) put(stp0, 7, now());
        put(stp, 1, now());
        put(stp, 5, ((unsigned long long)s << 4) | ((unsigned long long)(item - 2) << 32));
      }
    }
  }
  if (item == 0 || item == 2) {  // RS_connected(n_it) (skipped when it is the runner-up), then (SPEC) RS_connected(r_it)
    // two blocks, iterations of parity par each: RS_connected of the runner-up takes longer than the bookkeeping's
    // iteration (createActPath + the path sweep), so one block alone set the pace of a lone scene
    const int par = item == 0 ? 0 : 1;
    for (int it = it0 + ((par - it0) & 1);; it += 2) {
      unsigned long long* stp0 = pst(it);
      for (int job = 0; job < (SPEC && it > it0 ? 2 : 1); job++) {  // r_it: published by iteration it - 1 too
        const bool r = SPEC && job == 1;
        if (r) put(stp0, 6, now());
        IterArgs X = A;
        X.node = Q.node + (size_t)((it - 1) & 1) * 3 * B;
        X.node_rw = Q.node_rw + (size_t)((it - 1) & 1) * B;  // (with granules: non-null = use the stored winner)
        X.node_tuv = Q.node_tuv + (size_t)((it - 1) & 1) * 3 * B;
        if (it > it0) {  // n_it / r_it: published by iteration it - 1's bookkeeping in this launch
          X.node_ag = 1;
          X.node_flag = Q.nx;
          X.node_flag_min = 2 * (it - 1) + 2;
          X.node_flag_err = Q.err;
          if (A.ngr_pub || r) {
            X.ngr = (r ? Q.ngr2 : Q.ngr) + (size_t)((it - 1) & (HA_NGR_SLOTS - 1)) * B * HA_NGR;
            X.ngr_tag = (unsigned)it;
          }
        }
        rs_slot(X, r ? 2 + (it & 3) : it & 1);
        X.do_exp = 0;
        unsigned long long* stp = r ? nullptr : pst(it);
        put(stp, 0, now());
        if (!ha_iter_body<HWt, NBGt, true>(P, X, stp, slot, 0)) return;
        ha_stores_done();
        __syncthreads();
        if (threadIdx.x == 0) st_ag((r ? Q.rsrs : Q.rsr) + (size_t)par * B + s, 2 * it + 2);
        if (r) put(stp0, 7, now());
        put(stp, 1, now());
        put(stp, 5, 2ull | ((unsigned long long)s << 4));
      }
    }
  }
  // item 1: the bookkeeping of iteration it, it = it0, it0 + 1, ...
  // on HA_BOOK_WAVES waves of the block (the rest leave: a barrier counts only the waves still running), so its
  // block-wide steps (barriers, cross-wave reductions) span fewer waves
#ifndef HA_BOOK_WAVES
#define HA_BOOK_WAVES 4
#endif
  constexpr int NTB = 64 * (HWt < HA_BOOK_WAVES ? HWt : HA_BOOK_WAVES);
  if ((int)threadIdx.x >= NTB) return;
#ifndef HA_BOOK_PRIO
#define HA_BOOK_PRIO 3
#endif
  // the scene's chain: issued first where its CU is shared (other scenes' blocks, many scenes live)
  if (HA_BOOK_PRIO) __builtin_amdgcn_s_setprio(HA_BOOK_PRIO);
  if (SPEC && threadIdx.x < 12) sh_run[threadIdx.x] = 0;  // no runner-up yet: iteration it0's pop is no hit
  __syncthreads();
  int hit = 0;  // (SPEC) n_it is r_{it-1}: its records and RS_connected are the speculative ones
  for (int it = it0;; it++) {
    // E[it & 1]: every group of iteration it - 1 has expanded n_it (waited for inside, the open list's loads
    // in flight); on a hit the speculative E slot of r_{it-1} (its groups' round it - 2)
    unsigned long long* stp = pst(it);
    put(stp, 0, now());
    const int h = hit;
    const auto wait_exp = [&] {
      if (it > it0) {
        if (threadIdx.x == 0) {
          // r_{it-1}'s expansion: the groups' runner-up rounds of r_{it0+1}, r_{it0+3}, ... of r_{it-1}'s parity.
          // Counted by parity, not in one sum: r_it is published before this wait, so a fast group can already
          // have counted its round for r_it while a slow one still expands r_{it-1} (the groups' n rounds
          // cannot run ahead that way -- n_{it+1} is published after the wait)
          if (h) wait_ge(Q.exs + (size_t)((it - 1) & 1) * B + s, ng * ((it - 2 - it0) / 2 + 1), Q.err);
          else wait_ge(Q.ex + s, ng * (it - it0), Q.err);
        }
        __syncthreads();
      }
      put(stp, 2, now());  // (the book's wait for the expansion ends)
    };
    const IterArgs Ei = e_par(A, B, np, h ? 2 + ((it - 1) & 3) : it & 1);
    int hit_next = 0;
#ifndef HA_PREWAIT
#define HA_PREWAIT 1
#endif
    if (!HA_PREWAIT) wait_exp();  // (A/B build -DHA_PREWAIT=0: the wait before the bookkeeping's first load)
    const BookRec br = HA_PREWAIT ? ha_book_pipe<NTB, true, decltype(wait_exp), SPEC>(P, Q, Ei, B, it, s, stp,
                                                                                 wait_exp, sh_run, &hit_next)
                                  : ha_book_pipe<NTB, true, NoMid, SPEC>(P, Q, Ei, B, it, s, stp, NoMid(), sh_run,
                                                                   &hit_next);
    put(stp, 3, now());
    IterArgs F = A;
    rs_slot(F, h ? 2 + ((it - 1) & 3) : it & 1);
    if (threadIdx.x == 0) {
      // RS_connected(n_it) done; Q.rsr may already hold iteration it + 1's flag (that RS block starts once this
      // iteration's pop is published), the verdict itself stays in its slot until iteration it + 2 (+ 4: runner-up)
      const int f = h ? wait_ge(Q.rsrs + (size_t)((it - 1) & 1) * B + s, 2 * (it - 1) + 2, Q.err)
                      : wait_ge(Q.rsr + (size_t)(it & 1) * B + s, 2 * it + 2, Q.err);
      if (f == HA_DONE) {
        sh_f = 2;
      } else {
        ha_finish(Q, F, B, it, s, br, false);
        sh_f = ld_ag(F.rs_ok + s) ? 1 : !br.v[RC_GO] ? 2 : 0;
      }
      put(stp, 4, now());
      put(stp, 5, 1ull | ((unsigned long long)s << 4) | (17ull << 32));
    }
    __syncthreads();
    if (sh_f == 1) {  // RSpath_final into the canonical buffer the host reads
      const int n = ld_ag(F.rs_len + s);
      for (int i = threadIdx.x; i < 3 * n; i += NTB)
        A.rs_path[(size_t)s * MAXPATH * 3 + i] = ld_ag(F.rs_path + (size_t)s * MAXPATH * 3 + i);
    }
    if (sh_f) {
      if (A.ngr_pub && threadIdx.x < HA_NGR_SLOTS)  // the search ended: every slot's go word (whichever is waited on)
        __hip_atomic_store(Q.ngr + ((size_t)threadIdx.x * B + s) * HA_NGR + 13,
                           (unsigned long long)HA_NGR_DONE << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (SPEC && threadIdx.x >= HA_NGR_SLOTS && threadIdx.x < 2 * HA_NGR_SLOTS)  // and the runner-up's
        __hip_atomic_store(Q.ngr2 + ((size_t)(threadIdx.x - HA_NGR_SLOTS) * B + s) * HA_NGR + 13,
                           (unsigned long long)HA_NGR_DONE << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!A.ngr_pub && threadIdx.x == 0) st_ag(Q.nx + s, HA_DONE);
      return;
    }
    hit = hit_next;
    __syncthreads();
  }
}


// ------------------------------------------------------------- path finishing
// retrievePath + cubic_fit (hybrid_astar_utils.jl:100-177) for a planned scenario, one block each:
// the start state, a 100-point cubic between every pair of consecutive hybrid_astar_states (reversed
// to start -> goal order) and RSpath_final make actualpath; its cumulative arc length and the 50
// samples of the re-interpolated path at LinRange(0, tol_length, 50) (x_interp, y_interp, ψ_interp).
constexpr int RFIT = 100;  // num_path of cubic_fit (:101)
constexpr int RSAMP = 50;  // steps of retrievePath (:167)
constexpr int RT = 256;

// cubic_fit's coefficients (:101-111): [xg³ xg²; 3xg² 2xg] \ (pinv) [yg; tan ψg] in the frame of `cur`.
// pinv: Julia's LinearAlgebra.pinv through LAPACK dgesdd's 2x2 path (mp_jlmath.h mpj_pinv2).
__device__ __forceinline__ void cubic_params(const double* cur, const double* nxt, double* out) {
  double ns[3];
  change_basis(cur, nxt, 1.0, ns);
  const double xg = ns[0], yg = ns[1], pg = ns[2];
  const double M[4] = {xg * xg * xg, xg * xg, 3 * (xg * xg), 2 * xg};
  double Pm[4];
  mpj_pinv2(M, Pm);
  const double P0 = Pm[0], P1 = Pm[1], P2 = Pm[2], P3 = Pm[3];
  const double b0 = yg, b1 = mpj_tan(pg);
  out[0] = __builtin_fma(P1, b1, P0 * b0);  // pinv(A)*B: BLAS dgemv 'N' 2x2 (oracle/or_blas.h)
  out[1] = __builtin_fma(P3, b1, P2 * b0);
  out[2] = xg;
}

// Point k of cubic_fit(cur, ·) (:113-126): x = LinRange(0, xg, 100)[k], y = p1·x³ + p2·x², ψ = atan(3p1·x² +
// 2p2·x), rotated by ψ0 (Rmat·path .+ [x0; y0]) and ψ + ψ0.
__device__ __forceinline__ void cubic_point(const double* cur, const double* prm, int k, double* o) {
  const double t = (double)k / (RFIT - 1);
  const double x = (1 - t) * 0.0 + t * prm[2];
  const double y = prm[0] * (x * x * x) + prm[1] * (x * x);
  const double psi = mpj_atan((3 * prm[0]) * (x * x) + (2 * prm[1]) * x);
  double s0, c0;
  mpj_sincos(cur[2], &s0, &c0);
  o[0] = __builtin_fma(-s0, y, c0 * x) + cur[0];  // Rmat*path: BLAS dgemm, K = 2 (oracle/or_blas.h)
  o[1] = __builtin_fma(c0, y, s0 * x) + cur[1];
  o[2] = psi + cur[2];
}

// pts[off..][3] / plen[off..]: the dense actualpath and its arc length (the host sizes the ragged
// buffers from n_states and rs_len); seg[b][segstride][3]: cubic_params per segment.
__global__ __launch_bounds__(RT) void ha_retrieve_kernel(const double* start, const int* n_states,
                                                         const double* states, int sstride, const int* rs_len,
                                                         const double* rs_path, const long long* off, double* pts,
                                                         double* plen, double* seg, int segstride, int* npts,
                                                         double* tol, double* samples) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = n_states[b];
  double* smp = samples + (size_t)b * RSAMP * 3;
  if (n < 1) {  // not found: planHybridAstar! leaves no path to retrieve
    if (tid == 0) {
      npts[b] = 0;
      tol[b] = 0.0;
    }
    for (int i = tid; i < RSAMP * 3; i += RT) smp[i] = 0.0;
    return;
  }
  const int nseg = n - 1, nr = rs_len[b];
  const int L = 1 + RFIT * nseg + nr;
  double* P = pts + off[b] * 3;
  double* S = plen + off[b];
  const double* st = states + (size_t)b * sstride * 3;  // goal side first: start->goal state i = st[n-1-i]
  double* sg = seg + (size_t)b * segstride * 3;
  for (int t = tid; t < nseg; t += RT) cubic_params(st + 3 * (n - 1 - t), st + 3 * (n - 2 - t), sg + 3 * t);
  __syncthreads();
  for (int q = tid; q < L; q += RT) {
    double o[3];
    if (q == 0) {
      o[0] = start[3 * b];
      o[1] = start[3 * b + 1];
      o[2] = start[3 * b + 2];
    } else if (q <= RFIT * nseg) {
      const int t = (q - 1) / RFIT, k = (q - 1) - RFIT * t;
      cubic_point(st + 3 * (n - 1 - t), sg + 3 * t, k, o);
    } else {
      const double* r = rs_path + ((size_t)b * MAXPATH + (q - 1 - RFIT * nseg)) * 3;
      o[0] = r[0];
      o[1] = r[1];
      o[2] = r[2];
    }
    P[3 * q] = o[0];
    P[3 * q + 1] = o[1];
    P[3 * q + 2] = o[2];
  }
  __syncthreads();
  // ds = sqrt.(sum((p[:, 2:end] - p[:, 1:end-1]).^2, dims = 1)) (:153), then the running sum in order
  for (int q = tid + 1; q < L; q += RT) {
    const double dx = P[3 * q] - P[3 * (q - 1)], dy = P[3 * q + 1] - P[3 * (q - 1) + 1];
    S[q] = mpj_sqrt(dx * dx + dy * dy);
  }
  __syncthreads();
  __shared__ double sh_tot;
  if (tid == 0) {
    double acc = 0.0;
    S[0] = 0.0;
    for (int q = 1; q < L; q++) {
      acc = acc + S[q];
      S[q] = acc;
    }
    npts[b] = L;
    tol[b] = acc;
    sh_tot = acc;
  }
  __syncthreads();
  // x/y/ψ_interp_dense at traver_s_list = LinRange(0, tol_length, 50) (:167-170): Interpolations.jl
  // Gridded(Linear()): the last knot <= s (clamped to the last interval), weights (1-δ, δ)
  if (tid < RSAMP) {
    const double t = (double)tid / (RSAMP - 1);
    const double sv = (1 - t) * 0.0 + t * sh_tot;
    int lo = 0, hi = L - 1;  // largest i with S[i] <= sv
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (S[mid] <= sv) lo = mid;
      else hi = mid - 1;
    }
    const int i = lo < L - 1 ? lo : (L > 1 ? L - 2 : 0);
    if (L == 1) {
      smp[3 * tid] = P[0];
      smp[3 * tid + 1] = P[1];
      smp[3 * tid + 2] = P[2];
    } else {
      const double w = S[i + 1] - S[i];
      const double d = w > 0.0 ? (sv - S[i]) / w : 0.0;  // duplicate knots: the left value (as the oracle)
      for (int c = 0; c < 3; c++) smp[3 * tid + c] = (1 - d) * P[3 * i + c] + d * P[3 * (i + 1) + c];
    }
  }
}

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
  ctx->ha_prim_key.clear();  // a caller-given table: mp_ha_neighbor_origin recomputes next time
  if (ctx->ha_states_candi) { hipFree(ctx->ha_states_candi); ctx->ha_states_candi = nullptr; }
  if (ctx->ha_paths_candi) { hipFree(ctx->ha_paths_candi); ctx->ha_paths_candi = nullptr; }
  MP_HIP(ctx, hipMalloc(&ctx->ha_states_candi, sizeof(double) * 3 * p->n_prim));
  MP_HIP(ctx, hipMalloc(&ctx->ha_paths_candi, sizeof(double) * 3 * (size_t)p->n_prim * p->n_col));
  MP_HIP(ctx, hipMemcpy(ctx->ha_states_candi, states_candi, sizeof(double) * 3 * p->n_prim, hipMemcpyHostToDevice));
  MP_HIP(ctx, hipMemcpy(ctx->ha_paths_candi, paths_candi, sizeof(double) * 3 * (size_t)p->n_prim * p->n_col,
                        hipMemcpyHostToDevice));
  ctx->ha_n_prim = p->n_prim;
  ctx->ha_n_col = p->n_col;
  double ext = 0;
  for (size_t i = 0; i < 3 * (size_t)p->n_prim * p->n_col; i++)
    if (i % 3 != 2) ext = std::max(ext, std::fabs(paths_candi[i]));
  ctx->ha_prim_ext = ext;
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
  // the same settings as the installed table: hand back its host copies (each plan_batch call lands here)
  std::vector<double> key = {(double)n_steer, (double)n_gear, p->expand_time, (double)p->n_col, (double)p->n_prim};
  key.insert(key.end(), steer_set, steer_set + n_steer);
  key.insert(key.end(), gear_set, gear_set + n_gear);
  if (!ctx->ha_prim_key.empty() && ctx->ha_prim_key.size() == key.size() &&
      std::equal(key.begin(), key.end(), ctx->ha_prim_key.begin(),
                 [](double a, double b) { return __builtin_memcmp(&a, &b, sizeof a) == 0; }) &&
      ctx->ha_states_candi && ctx->ha_n_prim == p->n_prim && ctx->ha_n_col == p->n_col) {
    if (states_candi) std::copy(ctx->ha_sc_host.begin(), ctx->ha_sc_host.end(), states_candi);
    if (paths_candi) std::copy(ctx->ha_pc_host.begin(), ctx->ha_pc_host.end(), paths_candi);
    return MP_OK;
  }
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
  const int st = mp_ha_set_primitives(ctx, p, sc.data(), pc.data());  // (clears the key)
  if (st == MP_OK) {
    ctx->ha_prim_key = std::move(key);
    ctx->ha_sc_host = std::move(sc);
    ctx->ha_pc_host = std::move(pc);
  }
  return st;
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
  ha_cull_ok(ctx, p, &D, B, walls, node, goal);
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
  ha_cull_ok(ctx, p, &D, B, walls, node, goal);
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

int mp_ha_sat_cull_active(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* walls, const double* a,
                          const double* b, int32_t* active) {
  if (!ctx) return MP_ERR_INVALID;
  HaDev D;
  int st = make_ha(ctx, p, &D);
  if (st) return st;
  MP_CHECK(ctx, B >= 1 && (walls || p->n_walls == 0) && active, "bad arguments");
  ha_cull_ok(ctx, p, &D, B, walls, a, b);
  *active = D.cull;
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

int mp_ha_retrieve_path(mp_ctx* ctx, int32_t B, const double* start, const int32_t* n_states, const double* states,
                        int32_t state_stride, const int32_t* rs_len, const double* rs_path, int64_t* path_offset,
                        double* actualpath, double* path_length, int32_t* n_points, double* tol_length,
                        double* samples) {
  if (!ctx) return MP_ERR_INVALID;
  MP_CHECK(ctx, B >= 1 && start && n_states && states && rs_len && rs_path && n_points && tol_length && samples,
           "bad arguments to mp_ha_retrieve_path");
  MP_CHECK(ctx, state_stride >= 1, "state_stride (%d) must be >= 1", state_stride);
  MP_CHECK(ctx, (actualpath == nullptr) == (path_offset == nullptr) && (path_length == nullptr || path_offset),
           "actualpath / path_length need path_offset");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  // ragged layout: scenario b's points at [off[b], off[b+1])
  std::vector<long long> off(B + 1, 0);
  int max_seg = 1;
  for (int b = 0; b < B; b++) {
    const int n = n_states[b], nr = rs_len[b];
    MP_CHECK(ctx, n >= 0 && n <= state_stride, "n_states[%d] = %d outside [0, state_stride]", b, n);
    MP_CHECK(ctx, nr >= 0 && nr <= MAXPATH, "rs_len[%d] = %d outside [0, %d]", b, nr, MAXPATH);
    off[b + 1] = off[b] + (n >= 1 ? 1 + (long long)RFIT * (n - 1) + nr : 0);
    max_seg = std::max(max_seg, n - 1);
  }
  if (path_offset)
    for (int b = 0; b <= B; b++) path_offset[b] = off[b];
  const size_t tot = (size_t)std::max(off[B], 1LL);
  int st = MP_OK;
  const double* dstart = mp_upload(ctx, WS_IO0, start, 3 * (size_t)B, &st);
  const int* dns = mp_upload(ctx, WS_IO1, n_states, (size_t)B, &st);
  const double* dst = mp_upload(ctx, WS_IO2, states, 3 * (size_t)state_stride * B, &st);
  const int* drl = mp_upload(ctx, WS_IO3, rs_len, (size_t)B, &st);
  const double* drs = mp_upload(ctx, WS_IO4, rs_path, 3 * (size_t)MAXPATH * B, &st);
  const long long* doff = mp_upload(ctx, WS_IO5, off.data(), (size_t)B + 1, &st);
  double* dpts = (double*)mp_ws(ctx, WS_IO6, sizeof(double) * 3 * tot);
  double* dpl = (double*)mp_ws(ctx, WS_IO7, sizeof(double) * tot);
  double* dseg = (double*)mp_ws(ctx, WS_IO8, sizeof(double) * 3 * (size_t)max_seg * B);
  int* dnp = (int*)mp_ws(ctx, WS_IO9, sizeof(int) * (size_t)B);
  double* dtol = (double*)mp_ws(ctx, WS_IO10, sizeof(double) * (size_t)B);
  double* dsm = (double*)mp_ws(ctx, WS_IO11, sizeof(double) * RSAMP * 3 * (size_t)B);
  if (st || !dpts || !dpl || !dseg || !dnp || !dtol || !dsm) return st ? st : MP_ERR_NOMEM;
  hipLaunchKernelGGL(ha_retrieve_kernel, dim3(B), dim3(RT), 0, ctx->stream, dstart, dns, dst, state_stride, drl, drs,
                     doff, dpts, dpl, dseg, max_seg, dnp, dtol, dsm);
  MP_HIP(ctx, hipGetLastError());
  if ((st = mp_download(ctx, n_points, (const int32_t*)dnp, (size_t)B))) return st;
  if ((st = mp_download(ctx, tol_length, (const double*)dtol, (size_t)B))) return st;
  if ((st = mp_download(ctx, samples, (const double*)dsm, RSAMP * 3 * (size_t)B))) return st;
  if (off[B] > 0) {
    if ((st = mp_download(ctx, actualpath, (const double*)dpts, 3 * (size_t)off[B]))) return st;
    if ((st = mp_download(ctx, path_length, (const double*)dpl, (size_t)off[B]))) return st;
  }
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
  ha_cull_ok(ctx, p, &D, B, walls, start, goal);
  MP_CHECK(ctx, p->n_prim <= 64, "n_prim (%d) must be <= 64 (one neighbour per lane of the bookkeeping wave)",
           p->n_prim);
  MP_HIP(ctx, hipSetDevice(ctx->device));
  const int np = p->n_prim, mp = p->max_pops;
  // Encode range: 1 .. xnum*ynum*pnum (hybrid_astar_utils.jl:316-350)
  const long long ncell = (long long)(mpj_round((p->stbound[1] - p->stbound[0]) / p->res[0]) + 1) *
                          (long long)(mpj_round((p->stbound[3] - p->stbound[2]) / p->res[1]) + 1) *
                          (long long)(mpj_round((p->stbound[5] - p->stbound[4]) / p->res[2]) + 1);
  MP_CHECK(ctx, ncell > 0 && ncell < (1LL << 26), "state lattice too large (%lld cells)", ncell);
  const size_t C = (size_t)ncell + 1, nB = (size_t)B;
  // search state: node arrays and open list indexed [scene][node / cell]
  const size_t per_cell = 8 + 24 + 8 + 24 + 8 + 4 + 4 + 8 + 8 + 4 + 8 + 8 + 24 + 4 + 4 + 24 + 24;
  char* ws = (char*)mp_ws(ctx, WS_HA2, nB * C * per_cell + nB * (SI_N * 4 + 32) + nB * mp * 32 + nB * 48 +
                                           sizeof(int) * (mp + 2) + sizeof(int) * 4 * nB + nB * RC_N * 8 + nB * 8 + nB * 48 + nB * PRE_W * 8 + nB * 16 + 4 + nB * 24 + nB * HA_NGR_SLOTS * HA_NGR * 8 + 256 * 57 +
                                           nB * HA_NGR_SLOTS * HA_NGR * 8 + nB * 24 + 256 * 4);
  if (!ws) return MP_ERR_NOMEM;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* q = ws + off; off += (bytes + 255) & ~(size_t)255; return q; };
  HaSearch Q;
  Q.C = (int)C;
  Q.mp = mp;
  Q.parent = (long long*)take(nB * C * 8);
  Q.st = (double*)take(nB * C * 24);
  Q.index = (long long*)take(nB * C * 8);
  Q.g = (double*)take(nB * C * 8);
  Q.h = (double*)take(nB * C * 8);
  Q.f = (double*)take(nB * C * 8);
  Q.seq = (long long*)take(nB * C * 8);
  Q.pos = (int*)take(nB * C * 4);
  Q.nid = (int*)take(nB * C * 4);
  Q.of = (double*)take(nB * C * 8);
  Q.oseq = (long long*)take(nB * C * 8);
  Q.oid = (int*)take(nB * C * 4);
  Q.og = (double*)take(nB * C * 8);
  Q.oix = (long long*)take(nB * C * 8);
  Q.ost = (double*)take(nB * C * 24);
  Q.cur_g = (double*)take(nB * 8);
  Q.cur_ix = (long long*)take(nB * 8);
  Q.sc_i = (int*)take(nB * SI_N * 4);
  Q.ctr = (long long*)take(nB * 8);
  Q.start_index = (long long*)take(nB * 8);
  Q.pop_seq = (long long*)take(nB * mp * 8);
  Q.states = (double*)take(nB * mp * 24);
  Q.node = (double*)take(nB * 48);
  Q.live = (int*)take(sizeof(int) * (mp + 2));
  Q.lst = (int*)take(sizeof(int) * 2 * nB);
  Q.tk = (int*)take(sizeof(int) * 2 * nB);
  Q.rec = (long long*)take(nB * RC_N * 8);
  Q.rw = (int*)take(nB * C * 4);
  Q.orw = (int*)take(nB * C * 4);
  Q.node_rw = (int*)take(nB * 8);
  Q.tuv = (double*)take(nB * C * 24);
  Q.otuv = (double*)take(nB * C * 24);
  Q.node_tuv = (double*)take(nB * 48);
  Q.pre = (long long*)take(nB * PRE_W * 8);
  Q.nx = (int*)take(nB * 4);
  Q.ngr = (unsigned long long*)take(nB * HA_NGR_SLOTS * HA_NGR * 8);
  Q.ex = (int*)take(nB * 4);
  Q.rsr = (int*)take(nB * 8);
  Q.err = (int*)take(4);
  Q.node_g = (double*)take(nB * 16);
  Q.node_nn = (int*)take(nB * 8);
  Q.ngr2 = (unsigned long long*)take(nB * HA_NGR_SLOTS * HA_NGR * 8);
  Q.exs = (int*)take(nB * 8);
  Q.rsrs = (int*)take(nB * 8);
  Q.nhit = (int*)take(nB * 8);
  IterArgs A{};
  A.goal = mp_upload(ctx, WS_HA0, goal, 3 * nB, &st);
  A.walls = p->n_walls ? mp_upload(ctx, WS_HA1, walls, 5 * (size_t)p->n_walls * B, &st) : nullptr;
  const double* dstart = mp_upload(ctx, WS_IO0, start, 3 * nB, &st);
  // the expansion records: 2 parities (E[it & 1]) + (HA_SPEC) 4 runner-up slots
  constexpr size_t NPAR = HA_SPEC ? 6 : 2;
  A.h = (double*)mp_ws(ctx, WS_IO1, sizeof(double) * nB * np * NPAR);
  // the expansion records (nb, idx, fr, h, hw, hp_*) hold two parities: ha_pipe_kernel's launch it reads E[it & 1]
  // while its expansion blocks write E[(it + 1) & 1]; every other launch uses parity 0
  A.nb = (double*)mp_ws(ctx, WS_IO2, sizeof(double) * nB * np * 3 * NPAR);
  A.idx = (long long*)mp_ws(ctx, WS_IO3, sizeof(long long) * nB * np * NPAR);
  A.fr = (unsigned char*)mp_ws(ctx, WS_IO4, nB * np * NPAR);
  A.rs_ok = (unsigned char*)mp_ws(ctx, WS_IO5, nB);
  A.rs_len = (int*)mp_ws(ctx, WS_IO6, sizeof(int) * nB);
  A.rs_path = (double*)mp_ws(ctx, WS_IO7, sizeof(double) * nB * MAXPATH * 3);
  A.hw = (int*)mp_ws(ctx, WS_IO9, sizeof(int) * nB * np * NPAR);
  if (st || !A.h || !A.nb || !A.idx || !A.fr || !A.rs_ok || !A.rs_len || !A.rs_path || !A.hw)
    return st ? st : MP_ERR_NOMEM;
#ifndef HA_RS_WINNER
#define HA_RS_WINNER 1
#endif
  // (A/B build -DHA_RS_WINNER=0: RS_connected always runs the 48-candidate search)
  constexpr bool rs_full = !HA_RS_WINNER;
  // the pose table (A.ptab): the neighbour sweeps' heading terms for every lattice heading -- regulated
  // headings are round(modπ(ψ)/res)·res, so m spans round(±π/res) (one spare step each side); the few
  // microseconds of one launch per plan.
  {
    const double r = p->res[2];
    const int nsw = p->n_col > 5 ? (p->n_col - 1) / 5 + 1 : 1;
    const double lo = std::floor(-MPJ_PI / r) - 1, hi = std::ceil(MPJ_PI / r) + 1;
    const bool ok = r > 0 && hi - lo < 4096;
    const int mlo = ok ? (int)lo : 0, nm = ok ? (int)(hi - lo) + 1 : 0;
    const size_t n = (size_t)nm * np * nsw;
    double* tab = ok ? (double*)mp_ws(ctx, WS_IO10, sizeof(double) * 4 * n) : nullptr;
    if (ok && !tab) return MP_ERR_NOMEM;
    if (tab) {
      hipLaunchKernelGGL(ha_pose_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, D,
                         (const double*)ctx->ha_paths_candi, mlo, nm, nsw, tab);
      MP_HIP(ctx, hipGetLastError());
    }
    A.ptab = tab;
    A.pt_mlo = mlo;
    A.pt_nm = nm;
    A.pt_nsw = nsw;
    double* htn = ok ? (double*)mp_ws(ctx, WS_IO13, sizeof(double) * (2 * (size_t)nm + 4 * (size_t)nm * np)) : nullptr;
    if (ok && !htn) return MP_ERR_NOMEM;
    if (htn) {
      hipLaunchKernelGGL(ha_head_table_kernel, dim3((unsigned)((nm * np + 255) / 256)), dim3(256), 0, ctx->stream, D,
                         (const double*)ctx->ha_states_candi, mlo, nm, htn, htn + 2 * (size_t)nm);
      MP_HIP(ctx, hipGetLastError());
    }
    A.htn = htn;
    A.htk = htn ? htn + 2 * (size_t)nm : nullptr;
  }
  if (p->n_walls) {
    double* wt = (double*)mp_ws(ctx, WS_IO8, sizeof(double) * nB * p->n_walls * WT);
    if (!wt) return MP_ERR_NOMEM;
    hipLaunchKernelGGL(ha_wall_kernel, dim3((unsigned)((B * p->n_walls + 63) / 64)), dim3(64), 0, ctx->stream, D, B,
                       A.walls, wt);
    A.wtab = wt;
  }
  A.coherent = 1;
  A.dnid = Q.nid;  // the Dict pre-check: groups skip rs_heuristic when no neighbour of theirs can use it
  A.dg = Q.g;
  // (A/B build -DHA_DREC_CODE=1) the groups' Dict records
  A.drec = HA_DREC_CODE ? (long long*)mp_ws(ctx, WS_HA4, sizeof(long long) * nB * np * HA_DREC) : nullptr;
  A.dpos = Q.pos;
  A.df = Q.f;
  A.dseq = Q.seq;
  A.dindex = Q.index;
  A.drw = Q.rw;
  A.dst = Q.st;
  A.cur_g = Q.cur_g;
  A.C = (int)C;
  static const bool stamps_on = HA_STAMP_CODE && getenv("MPGPU_HA_STAMPS") && atoi(getenv("MPGPU_HA_STAMPS")) == 1;
  const int stamp_slots = std::min(mp / HA_STAMP_EVERY + 1, 40);  // iterations < 1,000
  A.stamps = nullptr;
  A.stamp_blocks = B * HA_PERSIST_PER((np + NBG_TAIL - 1) / NBG_TAIL);  // (the largest per-scene block count)
  if (stamps_on) {
    A.stamps = (unsigned long long*)mp_ws(ctx, WS_HA3, sizeof(unsigned long long) * HA_STAMP_N * (size_t)stamp_slots * A.stamp_blocks);
    if (!A.stamps) return MP_ERR_NOMEM;
    MP_HIP(ctx, hipMemsetAsync(A.stamps, 0, sizeof(unsigned long long) * HA_STAMP_N * (size_t)stamp_slots * A.stamp_blocks,
                               ctx->stream));
  }
  A.scene_of = nullptr;  // slot = scene
  A.active = Q.sc_i + SI_ACTIVE * B;
  A.sc = ctx->ha_states_candi;
  A.pc = ctx->ha_paths_candi;
  A.do_rs = 1;
  A.do_exp = 1;
  // ha_step_kernel's final ticket is taken by the RS_connected block and by the scene's bookkeeping block
  // (the last neighbour group): both roles must run, or no block finishes the iteration (and the RS block
  // would wait for a record that never comes)
  MP_CHECK(ctx, A.do_rs && A.do_exp, "ha_step_kernel needs both block roles");
  A.rs_path_free_only = 1;
  A.n_active = B;
  MP_HIP(ctx, hipMemsetAsync(Q.pop_seq, 0xff, nB * mp * 8, ctx->stream));  // -1 past each scene's pops
  MP_HIP(ctx, hipMemsetAsync(Q.live, 0, sizeof(int) * (mp + 2), ctx->stream));
  MP_HIP(ctx, hipMemsetAsync(Q.tk, 0, sizeof(int) * 2 * nB, ctx->stream));  // the finishers reset them
  MP_HIP(ctx, hipMemsetAsync(Q.rec, 0, sizeof(long long) * RC_N * nB, ctx->stream));  // record-ready flags
  MP_HIP(ctx, hipMemsetAsync(Q.nx, 0, sizeof(int) * nB, ctx->stream));  // ha_pipe_kernel's pop flags
  MP_HIP(ctx, hipMemsetAsync(Q.ngr, 0, sizeof(unsigned long long) * nB * HA_NGR_SLOTS * HA_NGR, ctx->stream));  // granule tags
  MP_HIP(ctx, hipMemsetAsync(Q.ex, 0, sizeof(int) * nB, ctx->stream));  // ha_persist_kernel's flags
  MP_HIP(ctx, hipMemsetAsync(Q.rsr, 0, sizeof(int) * 2 * nB, ctx->stream));
  MP_HIP(ctx, hipMemsetAsync(Q.ngr2, 0, sizeof(unsigned long long) * nB * HA_NGR_SLOTS * HA_NGR, ctx->stream));  // (HA_SPEC)
  MP_HIP(ctx, hipMemsetAsync(Q.exs, 0, sizeof(int) * 2 * nB, ctx->stream));
  MP_HIP(ctx, hipMemsetAsync(Q.rsrs, 0, sizeof(int) * 2 * nB, ctx->stream));
  MP_HIP(ctx, hipMemsetAsync(Q.nhit, 0, sizeof(int) * 2 * nB, ctx->stream));
  MP_HIP(ctx, hipMemsetAsync(Q.err, 0, sizeof(int), ctx->stream));
  hipLaunchKernelGGL(ha_init_kernel, dim3(B), dim3(256), 0, ctx->stream, D, Q, B, dstart);
  MP_HIP(ctx, hipGetLastError());
  // The whole search loop is enqueued without host round trips: iteration i = one ha_step_kernel
  // (RS_connected + 62 neighbours of every live scene, the bookkeeping + the next pop by the scene's
  // last neighbour-group block, beside RS_connected; the finisher publishes or undoes).  live[i] (scenes
  // still searching after iteration i) is copied back once per chunk of CH iterations; the host stays
  // at most two chunks ahead of the device and stops enqueueing when a copied count is 0 (at most
  // every scene's max_pops iterations).  (Round 1 fused the bookkeeping behind an agent-scope release
  // in every block -- an L2 write-back each -- and measured 67-90 ms vs 40 ms; ha_step_kernel hands
  // its records over with agent-coherent stores instead, so no block writes back its L2.)
  constexpr int CH = 16;  // iterations per live-count poll
  constexpr int NCK = 4;
  int* hl = (int*)mp_pinned(ctx, sizeof(int) * NCK);
  if (!hl) return mp_fail(ctx, MP_ERR_NOMEM, "pinned allocation failed");
  hipEvent_t ev[NCK];
  for (int i = 0; i < NCK; i++) MP_HIP(ctx, hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  auto cleanup = [&] { for (int i = 0; i < NCK; i++) hipEventDestroy(ev[i]); };
  const int per = 1 + (np + NBG - 1) / NBG, per_tail = 1 + (np + NBG_TAIL - 1) / NBG_TAIL;
  // the tail's rs_heuristic word units (ha_iter_body RSH): group g·4 + c holds neighbours 16g.. and word chunk
  // c, so there must be a group for every (16-neighbour set, chunk) -- n_prim mod 16 in {0, 13, 14, 15} with
  // 4 neighbours per group (62: yes); otherwise the groups' own word search.
  const bool tail_rsh = HA_TAIL_RSH && NBG_TAIL == 4 && per_tail - 1 >= 4 * ((np + 15) / 16);
  A.hp_c = (double*)mp_ws(ctx, WS_IO11, sizeof(double) * nB * np * 4 * NPAR);
  A.hp_i = (int*)mp_ws(ctx, WS_IO12, sizeof(int) * nB * np * 4 * NPAR);
  A.hp_t = (double*)mp_ws(ctx, WS_IO14, sizeof(double) * nB * np * 12 * NPAR);
  const bool tail_pipe = tail_rsh;
  // the persistent tail (ha_persist_kernel): one cooperative launch for the rest of the search once every block
  // of it fits the device at once.  Without cooperative launches (or when one is refused) the tail runs one
  // ha_pipe_kernel launch per iteration; MPGPU_HA_PERSIST=0 selects that fallback (a test hook: the same
  // results, tests/test_gpu_hastar.py runs it)
  const bool persist_env = !getenv("MPGPU_HA_PERSIST") || atoi(getenv("MPGPU_HA_PERSIST")) != 0;
  int persist_cap = 0;
  // the persistent kernel's block: 12 waves (one per CU: 14 scenes per launch), 6 (two per CU: 28 scenes; the
  // groups' sweep on 3 waves beside the 3 word waves) or 4 (three per CU: 42 scenes; the sweep on one wave).
  // Per call, the largest block that holds the whole batch in one launch from the start, and 6 when none does
  // (the tail then starts at 28 live scenes).  Measured: a lone scenario 18.7 / 18.9 / 20.4 us per iteration
  // with 12 / 6 / 4 (r05zg, r05zh); the 256-plan 24.0 ms with 6 or 4, 24.7 with 12; a 32-scene shard 16.4 ms with
  // 4 against 18.4-20.1 with 6, whose tail starts only at 28 live scenes, two blocks sharing each CU.
  const int per_ps = HA_PERSIST_PER((np + NBG_TAIL - 1) / NBG_TAIL);
  const void* pfn[3] = {reinterpret_cast<const void*>(ha_persist_kernel<HW_TAIL, NBG_TAIL>),
                        reinterpret_cast<const void*>(ha_persist_kernel<6, NBG_TAIL>),
                        reinterpret_cast<const void*>(ha_persist_kernel<4, NBG_TAIL>)};
  const int phws[3] = {HW_TAIL, 6, 4};
  int* pcap = ctx->ha_pcap;  // co-resident blocks of each on this context's device (0: no cooperative launch)
  int phw = 6;
  const void* persist_fn = pfn[1];
  double* rs_path2 = nullptr;
  int* rs_i2 = nullptr;
  if (tail_pipe && persist_env) {
    if (pcap[0] < 0) {
      int cus = 0, coop = 0;
      const bool ok = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess &&
                      hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device) == hipSuccess && coop;
      for (int v = 0; v < 3; v++) {
        int nbpc = 0;
        pcap[v] = ok && hipOccupancyMaxActiveBlocksPerMultiprocessor(&nbpc, pfn[v], 64 * phws[v], 0) == hipSuccess
                      ? nbpc * cus : 0;
      }
      (void)hipGetLastError();
    }
    int v = 1;
    for (int c = 0; c < 3; c++)
      if (B * per_ps <= pcap[c]) { v = c; break; }
    phw = phws[v];
    persist_fn = pfn[v];
    persist_cap = pcap[v];
    // RS_connected's outputs by slot (ha_persist_kernel rs_slot): NPAR slots of rs_path, rs_ok (bytes), rs_len
    rs_path2 = (double*)mp_ws(ctx, WS_IO15, sizeof(double) * NPAR * nB * MAXPATH * 3);
    rs_i2 = (int*)mp_ws(ctx, WS_IO16, sizeof(int) * 2 * NPAR * nB);
    if (!rs_path2 || !rs_i2) return MP_ERR_NOMEM;
  }
  bool persisted = false;
  bool piped_any = false;  // an ha_pipe_kernel launch ran: its bounded waits report through Q.err too
  // the pipelined launch's expansion blocks wait for their bookkeeping on a CU each: it pays only while the
  // whole launch is resident at once (one 12-wave block per CU).  (Measured and removed: the full-width shape
  // pipelined the same way, 0.4-0.9 ms slower per 256-plan, r05u/r05v: its bookkeeping publishes the pop ~10 us
  // after its start, so pop + expansion is no shorter than expansion + the whole bookkeeping.)
  constexpr int pipe_blocks = 256;
  int piped = 0;  // the format of the records the last launch left in E[it & 1]: 0 none, 2 tail
  // the prescan block only marks its record stale and takes its ticket (merging its PRE_K least entries into
  // popfirst! measured slower, r05j: 26.6 vs 25.7 us per lone iteration)
  A.no_pre = true;
  A.rs_last = true;  // RS_connected blocks dispatched after the groups (r05o: -0.2 ms)
  A.no_tuv = false;  // the tail stores the winners' (t, u, v): RS_connected rebuilds the commands from them
  A.ngr_pub = true;  // the popped node handed over as tagged granules (r05zl)
  // (A/B build -DHA_FULL_TUV_CODE=1) the full-width groups' winners' (t, u, v) too (neutral per plan, r05u)
  A.full_tuv = HA_FULL_TUV_CODE;
  if (!A.hp_c || !A.hp_i || !A.hp_t) return MP_ERR_NOMEM;
  // iteration it >= 2 works on the compact list of scenes still live (written by the previous
  // bookkeeping launch, count on the device); the host sizes the grids by the last live count it has
  // seen (an upper bound: it only decreases) and switches to the tail shape once that many scenes
  // fit in about two blocks per CU
#ifndef HA_TAIL_BLOCKS
#define HA_TAIL_BLOCKS 256
#endif
#ifndef HA_MID_BLOCKS
#define HA_MID_BLOCKS 512
#endif
  // the middle shape: HA_MID_HW-wave blocks, 16 neighbours each (5 blocks per scene), once known * 5 fits in
  // HA_MID_BLOCKS blocks.  r05x: the 6-wave middle shape for 16..102 live scenes and the tail from 15 (its
  // pipelined / persistent forms from 14) -- 256-plan 25.6 -> 24.9 ms, the largest strided / contiguous shard
  // 21.0 -> 19.2 / 17.9 -> 17.6 ms (the 12-wave tail step from 30 live scenes, round 4's threshold, and no middle)
  constexpr int tail_blocks = HA_TAIL_BLOCKS;
  constexpr int mid_blocks = HA_MID_BLOCKS;
  int known = B;
  int chunk = 0, checked = 0;
  bool finished = false;
  // (Measured and removed: a live-count mirror in host memory written by every launch, 1.1-1.4 ms slower per
  // 256-plan, r05u/r05v -- each launch's system-scope store delays its end.)
  A.mirror = nullptr;
  for (int it = 1; it <= mp && !finished; it++) {
    A.scene_of = it == 1 ? nullptr : Q.lst + ((it - 1) & 1) * B;
    A.n_live = it == 1 ? nullptr : Q.live + (it - 1);
    A.n_active = known;
    A.node = Q.node + (size_t)((it - 1) & 1) * 3 * B;  // the previous iteration's pops
    A.node_rw = rs_full ? nullptr : Q.node_rw + (size_t)((it - 1) & 1) * B;
    A.node_tuv = Q.node_tuv + (size_t)((it - 1) & 1) * 3 * B;
    const bool tail = known * per_tail <= tail_blocks;
    if (tail_pipe && known * per_ps <= persist_cap) {
      // the rest of the search in one cooperative launch, after the current nodes' expansion (bootstrap)
      const int per_pipe = 2 + (np + NBG_TAIL - 1) / NBG_TAIL;
      if (piped != 2) {
        hipLaunchKernelGGL((ha_pipe_kernel<HW_TAIL, NBG_TAIL>), dim3((unsigned)(known * per_pipe)), dim3(64 * HW_TAIL),
                           0, ctx->stream, D, Q, A, B, it, 1);
        piped = 2;
        piped_any = true;
      }
      unsigned char* rs_ok2 = reinterpret_cast<unsigned char*>(rs_i2);
      int* rs_len2 = rs_i2 + NPAR * nB;
      int it0 = it;
      void* args[] = {&D, &Q, &A, (void*)&B, &it0, &rs_path2, &rs_ok2, &rs_len2};
      // (MPGPU_HA_COOP=0: an ordinary launch of the same grid, co-resident by the occupancy check alone -- for
      // rocprofv3 runs: the profiler's exit handlers crash in a process that made a cooperative launch)
      static const bool coop_env = !getenv("MPGPU_HA_COOP") || atoi(getenv("MPGPU_HA_COOP")) != 0;
      const hipError_t le =
          coop_env ? hipLaunchCooperativeKernel(persist_fn, dim3((unsigned)(known * per_ps)), dim3(64 * phw), args, 0,
                                                ctx->stream)
                   : hipLaunchKernel(persist_fn, dim3((unsigned)(known * per_ps)), dim3(64 * phw), args, 0, ctx->stream);
      if (le != hipSuccess) {
        // refused (e.g. the device's co-residency changed under this context): the per-iteration pipelined
        // tail from this iteration on -- the bootstrap above already expanded the current nodes
        (void)hipGetLastError();
        persist_cap = 0;
        pcap[0] = pcap[1] = pcap[2] = 0;
        it--;
        continue;
      }
      persisted = true;
      break;
    } else if (tail && tail_pipe && known * (2 + (np + NBG_TAIL - 1) / NBG_TAIL) <= pipe_blocks) {
      const int per_pipe = 2 + (np + NBG_TAIL - 1) / NBG_TAIL;
      if (piped != 2) {  // the current nodes' expansion, for the first pipelined launch
        hipLaunchKernelGGL((ha_pipe_kernel<HW_TAIL, NBG_TAIL>), dim3((unsigned)(known * per_pipe)), dim3(64 * HW_TAIL),
                           0, ctx->stream, D, Q, A, B, it, 1);
        piped = 2;
      }
      hipLaunchKernelGGL((ha_pipe_kernel<HW_TAIL, NBG_TAIL>), dim3((unsigned)(known * per_pipe)), dim3(64 * HW_TAIL), 0,
                         ctx->stream, D, Q, A, B, it, 0);
      piped_any = true;
    } else if (tail) {
      piped = 0;
      if (tail_rsh)  // + the prescan block per scene
        hipLaunchKernelGGL((ha_step_kernel<HW_TAIL, NBG_TAIL, true>), dim3((unsigned)(known * (per_tail + 1))),
                           dim3(64 * HW_TAIL), 0, ctx->stream, D, Q, A, B, it);
      else
        hipLaunchKernelGGL((ha_step_kernel<HW_TAIL, NBG_TAIL>), dim3((unsigned)(known * per_tail)),
                           dim3(64 * HW_TAIL), 0, ctx->stream, D, Q, A, B, it);
    } else if (known * per <= mid_blocks) {
      piped = 0;
      hipLaunchKernelGGL((ha_step_kernel<HA_MID_HW, NBG>), dim3((unsigned)(known * per)),
                         dim3(64 * HA_MID_HW), 0, ctx->stream, D, Q, A, B, it);
    } else {
      piped = 0;
      hipLaunchKernelGGL((ha_step_kernel<HW, NBG>), dim3((unsigned)(known * per)), dim3(HT), 0,
                         ctx->stream, D, Q, A, B, it);
    }
    if (hipGetLastError() != hipSuccess) { cleanup(); return mp_fail(ctx, MP_ERR_HIP, "ha kernel launch failed"); }
    // (Measured and removed: polling the live count every 4 iterations near the persistent tail's threshold,
    // 1 ms slower per 256-plan, r05zn.)
    if (it % CH == 0 || it == mp) {
      const int slot = chunk % NCK;
      if (hipMemcpyAsync(hl + slot, Q.live + it, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
          hipEventRecord(ev[slot], ctx->stream) != hipSuccess) {
        cleanup();
        return mp_fail(ctx, MP_ERR_HIP, "live-count copy failed");
      }
      chunk++;
      // poll finished chunks without blocking; block only when two chunks ahead
      while (checked < chunk) {
        const int cs = checked % NCK;
        const bool must = chunk - checked > 2;
        const hipError_t q = must ? hipEventSynchronize(ev[cs]) : hipEventQuery(ev[cs]);
        if (q == hipErrorNotReady) break;
        if (q != hipSuccess) { cleanup(); return mp_fail(ctx, MP_ERR_HIP, "event wait failed"); }
        if (hl[cs] == 0) { finished = true; break; }
        known = std::min(known, std::max(hl[cs], 1));
        checked++;
      }
    }
  }
  // -1 past every scene's pops, filled while the search still runs on the device: the copy after it
  // overwrites columns [0, max_loop) (the device's memset padded those)
  std::fill(pop_seq, pop_seq + nB * mp, (int64_t)-1);
  if (A.stamps) {  // diagnostics: raw stamps to $MPGPU_HA_STAMPS_OUT (tools/ha_stamps.py reads them)
    std::vector<unsigned long long> h((size_t)HA_STAMP_N * stamp_slots * A.stamp_blocks);
    MP_HIP(ctx, hipMemcpyAsync(h.data(), A.stamps, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const char* fn = getenv("MPGPU_HA_STAMPS_OUT");
    if (FILE* f = fopen(fn ? fn : "ha_stamps.bin", "wb")) {
      const long long hdr[5] = {B, stamp_slots, A.stamp_blocks, HA_STAMP_EVERY, HA_STAMP_N};
      fwrite(hdr, sizeof hdr, 1, f);
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
  }
  if (persisted || piped_any) {  // a bounded wait (persistent or pipelined launch) that ran out: not trusted
    int err = 0;
    if (hipMemcpyAsync(&err, Q.err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      cleanup();
      return mp_fail(ctx, MP_ERR_HIP, "persistent search failed");
    }
    if (err) { cleanup(); return mp_fail(ctx, MP_ERR_HIP, "Hybrid A* search: a cross-block wait timed out"); }
  }
  if (getenv("MPGPU_HA_SPEC_STATS")) {  // diagnostics: how often the speculative runner-up was the next pop
    std::vector<int> nh(2 * nB);
    MP_HIP(ctx, hipMemcpyAsync(nh.data(), Q.nhit, sizeof(int) * 2 * nB, hipMemcpyDeviceToHost, ctx->stream));
    MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    long long hits = 0, pubs = 0;
    for (size_t i = 0; i < nB; i++) { hits += nh[i]; pubs += nh[nB + i]; }
    fprintf(stderr, "[ha spec] persisted %d: runner-ups published %lld, pops that were the runner-up %lld\n",
            (int)persisted, pubs, hits);
  }
  // outputs: per-scene counters, then the used prefix of pop_seq / states / RS paths
  std::vector<int> si(SI_N * nB);
  if ((st = mp_download(ctx, si.data(), (const int*)Q.sc_i, SI_N * nB))) { cleanup(); return st; }
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) { cleanup(); return mp_fail(ctx, MP_ERR_HIP, "search failed"); }
  cleanup();
  int max_loop = 0, max_ns = 0, max_rs = 0;
  for (int b = 0; b < B; b++) {
    found[b] = si[SI_FOUND * B + b];
    pops[b] = si[SI_LOOP * B + b];
    n_nodes[b] = si[SI_NNODES * B + b];
    n_states[b] = si[SI_NSTATES * B + b];
    rs_len[b] = found[b] ? si[SI_RSLEN * B + b] : 0;
    max_loop = std::max(max_loop, pops[b]);
    max_ns = std::max(max_ns, n_states[b]);
    max_rs = std::max(max_rs, rs_len[b]);
  }
  if (max_loop > 0)
    MP_HIP(ctx, hipMemcpy2DAsync(pop_seq, sizeof(int64_t) * mp, Q.pop_seq, sizeof(long long) * mp,
                                 sizeof(long long) * max_loop, nB, hipMemcpyDeviceToHost, ctx->stream));
  if (max_ns > 0)
    MP_HIP(ctx, hipMemcpy2DAsync(states_out, sizeof(double) * 3 * mp, Q.states, sizeof(double) * 3 * mp,
                                 sizeof(double) * 3 * max_ns, nB, hipMemcpyDeviceToHost, ctx->stream));
  std::vector<double> rsb;
  if (max_rs > 0) {
    rsb.resize(nB * max_rs * 3);
    MP_HIP(ctx, hipMemcpy2DAsync(rsb.data(), sizeof(double) * 3 * max_rs, A.rs_path, sizeof(double) * 3 * MAXPATH,
                                 sizeof(double) * 3 * max_rs, nB, hipMemcpyDeviceToHost, ctx->stream));
  }
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int b = 0; b < B; b++)
    if (found[b])
      std::copy(rsb.begin() + (size_t)b * max_rs * 3, rsb.begin() + ((size_t)b * max_rs + rs_len[b]) * 3,
                rs_path + (size_t)b * MAXPATH * 3);
  return MP_OK;
}

}  // extern "C"
