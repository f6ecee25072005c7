// tracker.hip — the Hybrid A* -> tracker hand-off and the path-tracker closed loop for gfx950
// (PathPlanning/HybridAstar/main_Tracker.jl:42-137, src/tracker_utils.jl:1-43) + C-ABI.
//
// track_kernel: one wavefront per planned scenario, B scenarios in lockstep.  The reference path
// x/y/ψ_ref = x/y/ψ_interp(LinRange(0, tol_length, n_ref)) and refined_length are built in LDS
// (structure of arrays, one point per lane per pass), then the simulation loop runs on the wave:
// every value of the tracker state is wave-uniform; the two findclosest windows of a step are
// scanned lane-parallel and reduced to the first minimum with DPP row operations + 4 readlanes (no
// LDS round trips on the serial chain), and the three time argmins of each step -- which depend
// only on the step number -- are computed 64 steps ahead, one step per lane, and read with
// v_readlane.
//
// The time argmins `argmin(abs.(refined_length .- c))` are evaluated on an 8-candidate window:
// refined_length .- c is LinRange(-c, tol - c, n) (Base's LinRange broadcast), whose elements w_j
// are within E <= 8·2^-52·(|c| + |tol - c| + tol) of the line L(j) = -c + j·(tol - c + c)/(n - 1).
// |L| grows by the slope s = tol/(n-1) per index away from its zero j* = c·(n-1)/tol, so when
// s > 4E every index more than 1.5 from j* (or from the clamped end) has |w| larger than the best
// one: the first minimum lies in [g-3, g+4] around g = rint(j*), clamped to [0, n-1].  When the
// guard fails (tol tiny against c) the lane scans all n elements instead.  Either way the result
// is the literal full scan's (oracle/or_track.c), bit for bit.
#include <cmath>
#include <cstdio>

#include "../../include/mp_jlmath.h"
#include "runtime.hpp"

namespace {

constexpr int TMAXREF = 2048;  // n_ref limit (LDS: 8 x 16 KB of reference data per block)

struct TrackDev {
  int n, max_steps, his_stride, his_cap, ns;
  double dt, la, pg, ig, L, msa;
};

// LinRange(a, b, n)[j+1]: Base lerpi, t = j/(n-1), (1-t)*a + t*b (t_j precomputed in LDS)
__device__ __forceinline__ double lerp_t(double t, double a, double b) { return (1 - t) * a + t * b; }

// one DPP step of the lexicographic (value, index) minimum (first minimum on ties)
template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ void red_dpp(double& v, int& i) {
  const long long bits = __double_as_longlong(v);
  const int lo = dpp<CTRL>((int)bits), hi = dpp<CTRL>((int)(bits >> 32));
  const double ov = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
  const int oi = dpp<CTRL>(i);
  if (ov < v || (ov == v && oi < i)) {
    v = ov;
    i = oi;
  }
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)bits, l), hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// wave-wide first minimum: quad xor 1 / xor 2, half-row and row mirrors (DPP, no LDS traffic), then the
// four row results combined in row order on uniform values
__device__ __forceinline__ int wave_min_index(double v, int i) {
  red_dpp<0xB1>(v, i);   // quad_perm [1,0,3,2]
  red_dpp<0x4E>(v, i);   // quad_perm [2,3,0,1]
  red_dpp<0x141>(v, i);  // row_half_mirror
  red_dpp<0x140>(v, i);  // row_mirror
  double bv = readlane_d(v, 0);
  int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
  for (int r = 1; r < 4; r++) {
    const double ov = readlane_d(v, 16 * r);
    const int oi = __builtin_amdgcn_readlane(i, 16 * r);
    if (ov < bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  return bi;
}

// argmin(abs.(LinRange(-c, tol - c, n))) on one lane: the 8-candidate window of the file header when
// its guard holds, else the full scan (both in increasing index order: the first minimum)
__device__ int argmin_time_lane(const double* tj, double tol, int n, double c, double jscale, bool fast) {
  const double a = 0.0 - c, b = tol - c;
  int lo = 0, cnt = n;
  if (fast) {
    double g = __builtin_rint(c * jscale);
    g = g < 0.0 ? 0.0 : (g > (double)(n - 1) ? (double)(n - 1) : g);
    lo = (int)g - 3;
    cnt = 8;
  }
  double bv = __builtin_inf();
  int bi = 0;
  for (int q = 0; q < cnt; q++) {
    int j = lo + q;
    j = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
    const double v = __builtin_fabs(lerp_t(tj[j], a, b));
    if (q == 0 || v < bv) {
      bv = v;
      bi = j;
    }
  }
  return bi;
}

// findclosest (tracker_utils.jl:38-43) over rows lo..hi of the LDS reference, first minimum of
// (x_ref - px)^2 + (y_ref - py)^2; -1 for an empty window (wave-uniform)
__device__ __forceinline__ int findclosest(const double* rx, const double* ry, double px, double py, int lo, int hi,
                                           int lane) {
  if (hi < lo) return -1;
  // the first 64 rows straight-line (windows are ~look_ahead / (tol / n_ref) rows: one pass), the rest
  // of a long window in a loop
  const int i0 = lo + lane;
  const bool in = i0 <= hi;
  const int ic = in ? i0 : lo;
  const double dx0 = rx[ic] - px, dy0 = ry[ic] - py;
  const double d0 = dx0 * dx0 + dy0 * dy0;
  double bv = in ? d0 : __builtin_inf();
  int bi = in ? i0 : 1 << 30;
  if (hi - lo >= 64) {
    for (int i = i0 + 64; i <= hi; i += 64) {
      const double dx = rx[i] - px, dy = ry[i] - py;
      const double d = dx * dx + dy * dy;
      if (d < bv) {
        bv = d;
        bi = i;
      }
    }
  }
  return wave_min_index(bv, bi);
}

__global__ __launch_bounds__(64) void track_kernel(TrackDev P, const double* __restrict__ start,
                                                   const double* __restrict__ tol_in,
                                                   const double* __restrict__ samples, int* __restrict__ n_steps,
                                                   int* __restrict__ status, double* __restrict__ fin,
                                                   double* __restrict__ eacc_out, double* __restrict__ ref_out,
                                                   double* __restrict__ his) {
  // reference data in LDS, structure of arrays: points, the inverse kinematics of every reference
  // point (functions of the closest index alone) and the headings' sin/cos
  __shared__ double rx[TMAXREF], ry[TMAXREF], rp[TMAXREF], rc[TMAXREF], rs[TMAXREF], tj[TMAXREF], iux[TMAXREF],
      isa[TMAXREF];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = P.n;
  const double tol = tol_in[b];
  double s0 = start[3 * b], s1 = start[3 * b + 1], s2 = start[3 * b + 2];
  double* hb = his ? his + (size_t)b * P.his_cap * 3 : nullptr;
  if (hb && P.his_cap > 0 && P.his_stride > 0 && lane == 0) {
    hb[0] = s0;
    hb[1] = s1;
    hb[2] = s2;
  }
  if (!(tol > 0.0)) {  // nothing planned for this scenario
    if (lane == 0) {
      n_steps[b] = 0;
      status[b] = MP_TRACK_NOPATH;
      fin[3 * b] = s0;
      fin[3 * b + 1] = s1;
      fin[3 * b + 2] = s2;
      eacc_out[b] = 0.0;
    }
    return;
  }
  // the hand-off (main_Tracker.jl:42-46): refined_length and x/y/ψ_interp at it, Interpolations.jl
  // linear interpolation on the knots LinRange(0, tol, ns): coordinate (ns-1)·(s-0)/(tol-0) + 1, floor
  // cell (the last knot and roundoff past it use the last interval), weights (1-δ, δ)
  const double* smp = samples + (size_t)b * P.ns * 3;
  for (int i = lane; i < n; i += 64) {
    const double t = (double)i / (double)(n - 1);
    const double s = lerp_t(t, 0.0, tol);
    tj[i] = t;
    const double c = ((double)(P.ns - 1) * (s - 0.0)) / (tol - 0.0) + 1.0;
    double f = __builtin_floor(c);
    if (c == (double)P.ns) f = f - 1.0;
    if (f > (double)(P.ns - 1)) f = (double)(P.ns - 1);
    if (f < 1.0) f = 1.0;
    const double d = c - f;
    const int k = (int)f - 1;
    double v[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      v[q] = (1 - d) * smp[3 * k + q] + d * smp[3 * (k + 1) + q];
      if (ref_out) ref_out[((size_t)b * n + i) * 3 + q] = v[q];
    }
    rx[i] = v[0];
    ry[i] = v[1];
    rp[i] = v[2];
  }
  __syncthreads();
  // per reference point i < n-1: dref (:91-93) and inverseKinematic (tracker_utils.jl:15-36) -- they
  // depend on the closest index alone, so the loop only looks them up -- and sin/cos(ψ_ref[i]) (:110)
  for (int i = lane; i < n; i += 64) {
    const double p0 = rp[i];
    double sp, cp;
    mpj_sincos(p0, &sp, &cp);
    double ux = 0.0, sa = 0.0;
    if (i + 1 < n) {
      const double r0 = lerp_t(tj[i], 0.0, tol), r1 = lerp_t(tj[i + 1], 0.0, tol);  // refined_length
      const double den = ((r1 - r0) + 1e-4) / 1;
      const double d0 = (rx[i + 1] - rx[i]) / den, d1 = (ry[i + 1] - ry[i]) / den;
      const double d2 = (rp[i + 1] - p0) / den;
      ux = __builtin_fabs(cp) >= mpj_sqrt(2.0) / 2 ? d0 / cp : d1 / sp;
      sa = __builtin_fabs(ux) >= 0.01 ? mpj_atan((d2 / ux) * P.L) : 0.0;
    }
    rc[i] = cp;
    rs[i] = sp;
    isa[i] = sa;
    iux[i] = ux;
  }
  __syncthreads();
  const double jscale = (double)(n - 1) / tol, slope = tol / (double)(n - 1);
  int least = 0, least_look = 0, sim = 0, stat = MP_TRACK_MAXSTEP;
  int mi1 = 0, mi0 = 0, mi2 = 0;  // time argmins of steps sim0 + lane (refilled every 64 steps)
  double eacc = 0.0;
  for (;;) {
    sim++;
    if (sim > P.max_steps) break;
    const int k = (sim - 1) & 63;
    if (k == 0) {
      // the three time argmins of every step only depend on the step number: lane l computes them for
      // step sim + l, the loop reads them with v_readlane
      const double t0 = (double)(sim + lane) * P.dt;
      const double c1 = t0 + P.la, c0 = t0, c2 = t0 + P.la * 2;
      const double E = 8 * 2.220446049250313e-16 *
                       (__builtin_fabs(c2) + __builtin_fabs(tol - c0) + __builtin_fabs(tol - c2) + tol);
      const bool fast = slope > 4 * E;
      mi1 = argmin_time_lane(tj, tol, n, c1, jscale, fast);
      mi0 = argmin_time_lane(tj, tol, n, c0, jscale, fast);
      mi2 = argmin_time_lane(tj, tol, n, c2, jscale, fast);
    }
    const int max_idx = __builtin_amdgcn_readlane(mi1, k);
    const int lt = __builtin_amdgcn_readlane(mi0, k);
    const int max_look = __builtin_amdgcn_readlane(mi2, k);
    double ss, cs;
    mpj_sincos(s2, &ss, &cs);  // the vehicle heading: look-ahead point and the Euler step
    const int idx = findclosest(rx, ry, s0, s1, least, max_idx, lane);
    if (idx < 0) {
      stat = MP_TRACK_EMPTY;
      break;
    }
    if (idx == n - 1) {
      stat = MP_TRACK_DONE;
      break;
    }
    least = idx > lt ? idx : lt;
    const double ux = iux[idx];
    double sa = isa[idx];
    // look-ahead point (:97-102) and its findclosest (:104-106)
    double lx = P.la * cs, ly = P.la * ss;
    if (ux > 0) {
      lx = s0 + lx;
      ly = s1 + ly;
    } else {
      lx = s0 - lx;
      ly = s1 - ly;
    }
    const int look_idx = findclosest(rx, ry, lx, ly, least_look, max_look, lane);
    if (look_idx < 0) {
      stat = MP_TRACK_EMPTY;
      break;
    }
    least_look = look_idx > max_idx ? look_idx : max_idx;
    // cross-track error and the PI correction with clamp (:108-119)
    const double v1x = rc[look_idx], v1y = rs[look_idx];
    const double v2x = lx - rx[look_idx], v2y = ly - ry[look_idx];
    const double err = v1x * v2y - v1y * v2x;
    eacc = eacc + err * P.dt;
    sa = (sa + P.pg * (-err)) + P.ig * (-eacc);
    sa = mpj_jmin(mpj_jmax(sa, -P.msa), P.msa);
    // kinematic Euler step (tracker_utils.jl:1-13, :121)
    const double k0 = ux * cs, k1 = ux * ss, k2 = ux / P.L * mpj_tan(sa);
    s0 = s0 + k0 * P.dt;
    s1 = s1 + k1 * P.dt;
    s2 = s2 + k2 * P.dt;
    if (hb && P.his_stride > 0 && lane == 0 && sim % P.his_stride == 0) {
      const int row = sim / P.his_stride;
      if (row < P.his_cap) {
        hb[3 * row] = s0;
        hb[3 * row + 1] = s1;
        hb[3 * row + 2] = s2;
      }
    }
  }
  if (lane == 0) {
    n_steps[b] = sim;
    status[b] = stat;
    fin[3 * b] = s0;
    fin[3 * b + 1] = s1;
    fin[3 * b + 2] = s2;
    eacc_out[b] = eacc;
  }
}

}  // namespace

extern "C" {

int mp_ha_track(mp_ctx* ctx, const mp_track_params* p, int32_t B, const double* start_real, const double* tol_length,
                const double* samples, int32_t n_samples, int32_t* n_steps, int32_t* status, double* final_state,
                double* err_acc, double* ref_out, double* his, int32_t his_cap) {
  if (!ctx) return MP_ERR_INVALID;
  MP_CHECK(ctx, p && B >= 1 && start_real && tol_length && samples && n_steps && status && final_state && err_acc,
           "bad arguments to mp_ha_track");
  MP_CHECK(ctx, p->n_ref >= 2 && p->n_ref <= TMAXREF, "n_ref (%d) must be in [2, %d]", p->n_ref, TMAXREF);
  MP_CHECK(ctx, n_samples >= 2, "n_samples (%d) must be >= 2", n_samples);
  MP_CHECK(ctx, p->max_steps >= 0, "max_steps (%d) must be >= 0", p->max_steps);
  MP_CHECK(ctx, p->dt_sim >= 0.0 && p->look_ahead >= 0.0, "dt_sim and look_ahead must be >= 0");
  MP_CHECK(ctx, p->his_stride >= 0 && (his == nullptr || (his_cap >= 1 && p->his_stride >= 1)),
           "his needs his_cap >= 1 and his_stride >= 1");
  MP_HIP(ctx, hipSetDevice(ctx->device));
  TrackDev D;
  D.n = p->n_ref;
  D.max_steps = p->max_steps;
  D.his_stride = his ? p->his_stride : 0;
  D.his_cap = his ? his_cap : 0;
  D.ns = n_samples;
  D.dt = p->dt_sim;
  D.la = p->look_ahead;
  D.pg = p->p_gain;
  D.ig = p->i_gain;
  D.L = p->veh_len;
  D.msa = p->max_sa;
  int st = MP_OK;
  const size_t nb = (size_t)B;
  const double* dstart = mp_upload(ctx, WS_IO0, start_real, 3 * nb, &st);
  const double* dtol = mp_upload(ctx, WS_IO1, tol_length, nb, &st);
  const double* dsmp = mp_upload(ctx, WS_IO2, samples, 3 * (size_t)n_samples * nb, &st);
  int* dns = mp_alloc_out(ctx, WS_IO3, n_steps, nb, &st);
  int* dstat = mp_alloc_out(ctx, WS_IO4, status, nb, &st);
  double* dfin = mp_alloc_out(ctx, WS_IO5, final_state, 3 * nb, &st);
  double* dea = mp_alloc_out(ctx, WS_IO6, err_acc, nb, &st);
  double* dref = mp_alloc_out(ctx, WS_IO7, ref_out, 3 * (size_t)p->n_ref * nb, &st);
  double* dhis = mp_alloc_out(ctx, WS_IO8, his, 3 * (size_t)(his ? his_cap : 0) * nb, &st);
  if (st) return st;
  mp_time_begin(ctx);
  hipLaunchKernelGGL(track_kernel, dim3((unsigned)B), dim3(64), 0, ctx->stream, D, dstart, dtol, dsmp, dns, dstat,
                     dfin, dea, dref, dhis);
  MP_HIP(ctx, hipGetLastError());
  mp_time_end(ctx);
  if ((st = mp_download(ctx, n_steps, (const int32_t*)dns, nb))) return st;
  if ((st = mp_download(ctx, status, (const int32_t*)dstat, nb))) return st;
  if ((st = mp_download(ctx, final_state, (const double*)dfin, 3 * nb))) return st;
  if ((st = mp_download(ctx, err_acc, (const double*)dea, nb))) return st;
  if ((st = mp_download(ctx, ref_out, (const double*)dref, 3 * (size_t)p->n_ref * nb))) return st;
  if ((st = mp_download(ctx, his, (const double*)dhis, 3 * (size_t)(his ? his_cap : 0) * nb))) return st;
  MP_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return MP_OK;
}

}  // extern "C"
