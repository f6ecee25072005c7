/*
 * ORACLE — test infrastructure only.  CPU restatement of the Hybrid A* -> tracker hand-off and the
 * tracker closed loop:
 *   PathPlanning/HybridAstar/main_Tracker.jl:42-137   (refined_length, x/y/ψ_ref, the simulation loop)
 *   PathPlanning/HybridAstar/src/tracker_utils.jl:1-43 (kinematic, inverseKinematic, findclosest)
 * Scalar C, fp64, the reference's evaluation order; libm = include/mp_jlmath.h (FDLIBM).  Every
 * argmin is the literal full scan the reference does (first minimum).
 *
 * Parity status: no reference artifact exists for this path (main_Tracker.jl writes no file), so the
 * loop is pinned GPU-vs-this-restatement bit-exactly.  Unpinned vs Julia (absent here):
 *  - Interpolations.jl (not vendored, version unpinned): linear_interpolation on a LinRange of knots is
 *    restated as coordlookup (len-1)*(x-start)/(stop-start) + 1, the floor cell (the last knot uses the
 *    last interval), weights (1-δ, δ) -- the same convention as or_ha_retrieve;
 *  - `refined_length .- c` is Base's LinRange broadcast specialisation, LinRange(start - c, stop - c, n),
 *    whose elements are lerps (1-t)(start-c) + t(stop-c), not element-wise differences.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mp_jlmath.h"
#include "../include/mpgpu.h"

/* LinRange(a, b, n)[j+1] (Base lerpi: t = j/(n-1), (1-t)*a + t*b) */
static double lin_el(double a, double b, int n, int j) {
  const double t = (double)j / (double)(n - 1);
  return (1 - t) * a + t * b;
}

/* argmin(abs.(refined_length .- c)) (main_Tracker.jl:82,90,104,106), 0-based; refined_length =
 * LinRange(0, tol, n), so the broadcast is LinRange(0 - c, tol - c, n). */
static int argmin_time(double tol, int n, double c) {
  const double a = 0.0 - c, b = tol - c;
  int best = 0;
  double bv = fabs(lin_el(a, b, n, 0));
  for (int j = 1; j < n; j++) {
    const double v = fabs(lin_el(a, b, n, j));
    if (v < bv) { bv = v; best = j; }
  }
  return best;
}

/* findclosest, tracker_utils.jl:38-43: argmin over rows lo..hi (0-based, inclusive) of
 * (x_ref - px)^2 + (y_ref - py)^2 (sum over dims = 2: x term + y term).  -1 for an empty window. */
static int findclosest(const double* ref, double px, double py, int lo, int hi) {
  if (hi < lo) return -1;
  int best = lo;
  double bv = 0.0;
  for (int i = lo; i <= hi; i++) {
    const double dx = ref[3 * i] - px, dy = ref[3 * i + 1] - py;
    const double d = dx * dx + dy * dy;
    if (i == lo || d < bv) { bv = d; best = i; }
  }
  return best;
}

/* x/y/ψ_interp(refined_length) (main_Tracker.jl:42-46): ref[n][3]. */
void or_track_reference(double tol, const double* samples, int ns, int n, double* ref) {
  for (int i = 0; i < n; i++) {
    const double s = lin_el(0.0, tol, n, i);
    const double c = ((double)(ns - 1) * (s - 0.0)) / (tol - 0.0) + 1.0; /* 1-based knot coordinate */
    double f = floor(c);
    if (c == (double)ns) f = f - 1.0;
    if (f > (double)(ns - 1)) f = (double)(ns - 1); /* roundoff past the last knot: the last interval */
    if (f < 1.0) f = 1.0;
    const double d = c - f;
    const int k = (int)f - 1;
    for (int q = 0; q < 3; q++) ref[3 * i + q] = (1 - d) * samples[3 * k + q] + d * samples[3 * (k + 1) + q];
  }
}

/* The tracker loop for one scenario, main_Tracker.jl:63-122.  Returns MP_TRACK_*; *n_steps =
 * simulation_idx at the end, st[3] = cur_states, *err_acc = err_accumulated; his (optional,
 * his_cap rows of 3) gets the state after every his_stride-th update, row 0 = start. */
int or_track(const mp_track_params* p, const double* start, double tol, const double* samples, int ns,
             double* ref /* [n_ref][3] scratch or output */, int32_t* n_steps, double* st, double* err_acc,
             double* his, int his_cap) {
  const int n = p->n_ref;
  const double dt = p->dt_sim, la = p->look_ahead, L = p->veh_len, msa = p->max_sa;
  memcpy(st, start, sizeof(double) * 3);
  *err_acc = 0.0;
  *n_steps = 0;
  if (his && his_cap > 0 && p->his_stride > 0) memcpy(his, start, sizeof(double) * 3);
  if (!(tol > 0.0)) return MP_TRACK_NOPATH;
  or_track_reference(tol, samples, ns, n, ref);
  int least = 0, least_look = 0, sim = 0;
  double eacc = 0.0;
  int status = MP_TRACK_MAXSTEP;
  for (;;) {
    sim++;
    if (sim > p->max_steps) break; /* every ending leaves the last entry without an update */
    const double t0 = (double)sim * dt;
    const int max_idx = argmin_time(tol, n, t0 + la);
    const int idx = findclosest(ref, st[0], st[1], least, max_idx);
    if (idx < 0) { status = MP_TRACK_EMPTY; break; }
    if (idx == n - 1) { status = MP_TRACK_DONE; break; }
    const int lt = argmin_time(tol, n, t0);
    least = idx > lt ? idx : lt;
    /* dref = (ref_next - ref_cur) / ((refined_length[idx+1] - refined_length[idx] + 1e-4) / 1) */
    const double den = ((lin_el(0.0, tol, n, idx + 1) - lin_el(0.0, tol, n, idx)) + 1e-4) / 1;
    const double* rc = ref + 3 * idx;
    const double d0 = (rc[3] - rc[0]) / den, d1 = (rc[4] - rc[1]) / den, d2 = (rc[5] - rc[2]) / den;
    /* inverseKinematic, tracker_utils.jl:15-36 */
    const double cp = mpj_cos(rc[2]), sp = mpj_sin(rc[2]);
    const double ux = fabs(cp) >= sqrt(2.0) / 2 ? d0 / cp : d1 / sp;
    double sa = fabs(ux) >= 0.01 ? mpj_atan((d2 / ux) * L) : 0.0;
    /* look-ahead point, :97-102 */
    const double cs = mpj_cos(st[2]), ss = mpj_sin(st[2]);
    double lx = la * cs, ly = la * ss;
    if (ux > 0) { lx = st[0] + lx; ly = st[1] + ly; }
    else { lx = st[0] - lx; ly = st[1] - ly; }
    const int max_look = argmin_time(tol, n, t0 + la * 2);
    const int look_idx = findclosest(ref, lx, ly, least_look, max_look);
    if (look_idx < 0) { status = MP_TRACK_EMPTY; break; }
    least_look = look_idx > max_idx ? look_idx : max_idx; /* argmin(|r - (t + look_ahead_dist)|) again */
    /* cross-track error, :108-115 */
    const double* rl = ref + 3 * look_idx;
    const double v1x = mpj_cos(rl[2]), v1y = mpj_sin(rl[2]);
    const double v2x = lx - rl[0], v2y = ly - rl[1];
    const double err = v1x * v2y - v1y * v2x; /* cross(vec1, vec2)[3] */
    eacc = eacc + err * dt;
    sa = (sa + p->p_gain * (-err)) + p->i_gain * (-eacc);
    sa = mpj_jmin(mpj_jmax(sa, -msa), msa);
    /* kinematic Euler step, tracker_utils.jl:1-13 and :121 */
    const double k0 = ux * cs, k1 = ux * ss, k2 = ux / L * mpj_tan(sa);
    st[0] = st[0] + k0 * dt;
    st[1] = st[1] + k1 * dt;
    st[2] = st[2] + k2 * dt;
    if (his && p->his_stride > 0 && sim % p->his_stride == 0) {
      const int row = sim / p->his_stride;
      if (row < his_cap) memcpy(his + 3 * row, st, sizeof(double) * 3);
    }
  }
  *n_steps = sim;
  *err_acc = eacc;
  return status;
}
