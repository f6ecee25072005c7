/* ORACLE under AddressSanitizer + UndefinedBehaviorSanitizer (test infrastructure only).
 *
 * tests/test_oracle_asan.py compiles this driver together with oracle/*.c using
 * -fsanitize=address,undefined, writes the inputs of one call per hot-path entry point into a
 * directory as raw little-endian arrays, runs the driver on it and compares every output file with
 * the regular liboracle.so results, bit for bit.  Each input file is read whole; sizes follow the
 * parameter structs, so a wrong size in the restatement shows up as a heap overflow here.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mpgpu.h"

int or_mppi_plan(const mp_mppi_params* p, int scene, const double* X0, const double* goal, const double* unom,
                 const double* obstacles, const uint8_t* grid, const double* noise, double* U, double* traj,
                 double* cost, int* feasible, int* rc, int* fc, double* ctraj, double* cctrl, double* ccost,
                 uint8_t* cfeas);
int or_mppi_closed_loop(const mp_mppi_params* p, int scene, int update_steps, int max_steps, double dt,
                        double goal_radius, const int32_t* hold, const double* X0, const double* goal,
                        const double* unom0, const double* obstacles, const uint8_t* grid, const double* noise,
                        double* his, int* n_rows, int* n_replans, double* U_log, double* traj_log, double* cost_log,
                        int32_t* feas_log, int32_t* rc_log);
int or_ilqr_solve(const mp_ilqr_params* p, double* X, double* U, double* J, int32_t* iters);
int or_ha_plan(const mp_ha_params* p, const double* start, const double* goal, const double* walls, const double* sc,
               const double* pc, int32_t* pops, int32_t* n_nodes, int64_t* seq, int32_t* n_states, double* states,
               int32_t* rs_len, double* rs);
int or_ha_retrieve(const double* start, int n, const double* states, int nr, const double* rs, double* pts,
                   double* plen, double* tol, double* smp);
int or_track(const mp_track_params* p, const double* start, double tol, const double* samples, int n_samples,
             double* ref, int32_t* n_steps, double* final_state, double* err_acc, double* his, int his_cap);

static const char* g_dir;

static void* rd(const char* name, size_t* nbytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", g_dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "missing %s\n", path); exit(2); }
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* b = malloc(n > 0 ? (size_t)n : 1);
  if (n > 0 && fread(b, 1, (size_t)n, f) != (size_t)n) exit(2);
  fclose(f);
  if (nbytes) *nbytes = (size_t)n;
  return b;
}

static void wr(const char* name, const void* p, size_t nbytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/out_%s", g_dir, name);
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(p, 1, nbytes, f) != nbytes) exit(3);
  fclose(f);
}

#define DBL(n) ((double*)calloc((size_t)(n), sizeof(double)))

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  g_dir = argv[1];
  { /* MPPIPlan with external noise, the TrajectoryCollection collected */
    mp_mppi_params* p = rd("mppi_p.bin", NULL);
    double *X0 = rd("mppi_x0.bin", NULL), *goal = rd("mppi_goal.bin", NULL), *un = rd("mppi_unom.bin", NULL);
    double *obs = rd("mppi_obs.bin", NULL), *z = rd("mppi_noise.bin", NULL);
    const int K = p->K, H = p->H;
    double *U = DBL(2 * H), *traj = DBL(7 * (H + 1)), cost = 0, *ct = DBL((size_t)K * 7 * (H + 1)),
           *cc = DBL((size_t)K * 2 * H), *co = DBL(K);
    uint8_t* cf = calloc(K, 1);
    int fe = 0, rc = 0, fc = 0;
    const int nan = or_mppi_plan(p, 0, X0, goal, un, obs, NULL, z, U, traj, &cost, &fe, &rc, &fc, ct, cc, co, cf);
    const int32_t ints[4] = {nan, fe, rc, fc};
    wr("mppi_U.bin", U, 16 * H);
    wr("mppi_traj.bin", traj, 56 * (H + 1));
    wr("mppi_cost.bin", &cost, 8);
    wr("mppi_ints.bin", ints, sizeof ints);
    wr("mppi_ccost.bin", co, 8 * (size_t)K);
    wr("mppi_ctraj.bin", ct, 56 * (size_t)K * (H + 1));
    free(p); free(X0); free(goal); free(un); free(obs); free(z); free(U); free(traj); free(ct); free(cc); free(co);
    free(cf);
  }
  { /* the closed loop of MPPI/main.jl:55-83, given noise */
    mp_mppi_params* p = rd("loop_p.bin", NULL);
    int32_t* cfg = rd("loop_cfg.bin", NULL); /* update_steps, max_steps */
    double* f = rd("loop_f.bin", NULL);      /* dt, radius */
    int32_t* hold = rd("loop_hold.bin", NULL);
    double *X0 = rd("loop_x0.bin", NULL), *goal = rd("loop_goal.bin", NULL), *un = rd("loop_unom.bin", NULL);
    double *obs = rd("loop_obs.bin", NULL), *z = rd("loop_noise.bin", NULL);
    const int H = p->H, M = cfg[1], R = (cfg[1] + cfg[0] - 1) / cfg[0];
    double *his = DBL((size_t)(M + 1) * 8), *Ul = DBL((size_t)R * 2 * H), *tl = DBL((size_t)R * 7 * (H + 1)),
           *cl = DBL(R);
    int32_t *fl = calloc(R, 4), *rl = calloc(R, 4);
    int nr = 0, np = 0;
    const int nan = or_mppi_closed_loop(p, 0, cfg[0], cfg[1], f[0], f[1], hold, X0, goal, un, obs, NULL, z, his, &nr,
                                        &np, Ul, tl, cl, fl, rl);
    const int32_t ints[3] = {nan, nr, np};
    wr("loop_ints.bin", ints, sizeof ints);
    wr("loop_his.bin", his, 64 * (size_t)(M + 1));
    wr("loop_U.bin", Ul, 16 * (size_t)R * H);
    free(p); free(cfg); free(f); free(hold); free(X0); free(goal); free(un); free(obs); free(z); free(his); free(Ul);
    free(tl); free(cl); free(fl); free(rl);
  }
  { /* the iLQR script loop (ILQR.jl:39-88), one instance */
    mp_ilqr_params* p = rd("ilqr_p.bin", NULL);
    double *X = rd("ilqr_X.bin", NULL), *U = rd("ilqr_U.bin", NULL), J = 0;
    int32_t it = 0;
    const int32_t fl = or_ilqr_solve(p, X, U, &J, &it);
    const int32_t ints[2] = {fl, it};
    wr("ilqr_X.bin", X, 32 * (size_t)p->N);
    wr("ilqr_U.bin", U, 16 * (size_t)p->N);
    wr("ilqr_J.bin", &J, 8);
    wr("ilqr_ints.bin", ints, sizeof ints);
    free(p); free(X); free(U);
  }
  { /* planHybridAstar! + retrievePath + the tracker loop, one parking scenario */
    mp_ha_params* p = rd("ha_p.bin", NULL);
    double *start = rd("ha_start.bin", NULL), *goal = rd("ha_goal.bin", NULL), *walls = rd("ha_walls.bin", NULL);
    double *sc = rd("ha_sc.bin", NULL), *pc = rd("ha_pc.bin", NULL), *real = rd("ha_real.bin", NULL);
    mp_track_params* tp = rd("track_p.bin", NULL);
    const int mp = p->max_pops;
    int32_t pops = 0, nn = 0, ns = 0, rl = 0;
    int64_t* seq = malloc(sizeof(int64_t) * mp);
    for (int i = 0; i < mp; i++) seq[i] = -1;
    double *states = DBL((size_t)mp * 3), *rs = DBL(501 * 3);
    const int32_t found = or_ha_plan(p, start, goal, walls, sc, pc, &pops, &nn, seq, &ns, states, &rl, rs);
    const int32_t ints[5] = {found, pops, nn, ns, rl};
    wr("ha_ints.bin", ints, sizeof ints);
    wr("ha_seq.bin", seq, 8 * (size_t)pops);
    wr("ha_states.bin", states, 24 * (size_t)ns);
    wr("ha_rs.bin", rs, 24 * (size_t)rl);
    const int L = ns ? 1 + 100 * (ns - 1) + rl : 1;
    double *pts = DBL((size_t)L * 3), *plen = DBL(L), tol = 0, *smp = DBL(150);
    const int32_t m = or_ha_retrieve(start, ns, states, rl, rs, pts, plen, &tol, smp);
    wr("ret_m.bin", &m, 4);
    wr("ret_pts.bin", pts, 24 * (size_t)m);
    wr("ret_smp.bin", smp, 150 * 8);
    const int cap = 4000;
    double *ref = DBL((size_t)tp->n_ref * 3), fin[3] = {0, 0, 0}, ea = 0, *th = DBL((size_t)cap * 3);
    int32_t nst = 0;
    const int32_t status = or_track(tp, real, tol, smp, 50, ref, &nst, fin, &ea, th, cap);
    const int32_t ti[2] = {status, nst};
    wr("track_ints.bin", ti, sizeof ti);
    wr("track_fin.bin", fin, 24);
    wr("track_ref.bin", ref, 24 * (size_t)tp->n_ref);
    free(p); free(start); free(goal); free(walls); free(sc); free(pc); free(real); free(tp); free(seq); free(states);
    free(rs); free(pts); free(plen); free(smp); free(ref); free(th);
  }
  puts("asan driver ok");
  return 0;
}
