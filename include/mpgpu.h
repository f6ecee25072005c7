/*
 * mpgpu.h — C ABI of libmpgpu.so, the MI355X (gfx950) hot path of
 * congkaishen/MotionPlanning.
 *
 * The reference is pure Julia; these entry points are what its planner calls
 * through `ccall` (binding shown in INTEGRATION.md, wrapper in julia/MPGPU.jl).
 * Every entry point cites the reference interface it replaces.
 *
 * Conventions
 *  - All functions return an int status: MP_OK (0) or an MP_ERR_* code; the
 *    message is available from mp_last_error(ctx).  This mirrors the
 *    reference's `error(...)` validation (OptimalControl/MPPI/src/setup.jl:19-38).
 *  - Arrays are dense, C row-major.  Shapes are written in C order; the
 *    equivalent Julia column-major shape is the reverse, e.g. noise
 *    [S][K][H][2] here == Array{Float64}(2, H, K, S) in Julia.
 *  - Functions without the _dev suffix take HOST pointers, are synchronous,
 *    and return after all results have been copied back (Julia arrays are
 *    rooted for the duration of the ccall).  _dev variants take DEVICE
 *    pointers, enqueue on the context's stream and do not synchronise.
 *  - A context owns one HIP device, one stream and cached device workspaces.
 *    It is not thread-safe; use one context per GPU / thread.
 *  - Precision: Float64 throughout, like the reference.
 */
#ifndef MPGPU_H
#define MPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPGPU_VERSION "0.1.0"

#define MP_OK 0
#define MP_ERR_INVALID 1   /* bad argument (shape, NULL, range)            */
#define MP_ERR_HIP 2       /* HIP runtime error                            */
#define MP_ERR_NOMEM 3     /* device allocation failed                     */
#define MP_ERR_NUMERIC 4   /* NaN / domain flag raised (outputs written)   */
#define MP_ERR_UNSUPPORTED 5

typedef struct mp_ctx mp_ctx;

/* ------------------------------------------------------------- context */
int mp_ctx_create(int device, mp_ctx** out);
int mp_ctx_destroy(mp_ctx* ctx);
const char* mp_last_error(mp_ctx* ctx);
const char* mp_version(void);
int mp_device_count(int* n);
/* Synchronise the context stream and its side stream (after _dev calls). */
int mp_ctx_synchronize(mp_ctx* ctx);
/* Order the context stream after all side-stream work enqueued so far (the deferred
 * MPPI final rollouts, mp_mppi_params.final_stream = 1): consumers of traj_out /
 * cost_out / feasible_out on the context stream call this first. */
int mp_ctx_join(mp_ctx* ctx);
/* The hipStream_t the context launches on (for HIP-event timing). */
void* mp_ctx_stream(mp_ctx* ctx);
/* Kernel timing: when enabled, every launch of the dominant kernel of a call
 * (mppi_plan_kernel, ...) is bracketed by HIP events on the context stream;
 * mp_ctx_kernel_ms synchronises, returns the summed milliseconds and launch
 * count since the last query, and resets them. */
int mp_ctx_kernel_timing(mp_ctx* ctx, int enable);
int mp_ctx_kernel_ms(mp_ctx* ctx, double* ms_sum, int32_t* count);
/* Device workspaces.  A context caches its scratch buffers across calls (they only grow, with
 * 25 % headroom).  mp_ctx_trim synchronises and frees every cached buffer larger than
 * keep_bytes (0: all of them); later calls re-allocate what they need.
 * mp_ctx_set_workspace_limit caps any single buffer (0: no cap).  Optional speed-up buffers
 * (mp_ilqr_solve's all-trials-at-once line-search slots, which are also skipped when they
 * would take more than half of the free device memory) fall back to a smaller layout with
 * identical results; a call that cannot run within the cap returns MP_ERR_NOMEM. */
int mp_ctx_trim(mp_ctx* ctx, size_t keep_bytes);
int mp_ctx_set_workspace_limit(mp_ctx* ctx, size_t bytes);

/* ---------------------------------------------------------------- MPPI */
#define MP_NX 7 /* [x, y, v, r, psi, ux, sa]  vehicledynamics.jl:20-26 */
#define MP_NU 2 /* [sr, ax]                    vehicledynamics.jl:27-28 */

#define MP_NOISE_EXTERNAL 0 /* z ~ N(0,I) supplied by the caller (parity mode) */
#define MP_NOISE_PHILOX 1   /* Philox4x32-10 + Box–Muller on device            */

/* Planner settings; fields mirror MPPISetting (OptimalControl/MPPI/src/types.jl:10-31). */
typedef struct mp_mppi_params {
  int32_t K;                 /* SamplingNumber                                  */
  int32_t H;                 /* N, horizon steps                                */
  int32_t feasibility_count; /* FeasibilityCount (default 1300); >= K disables  */
  int32_t n_obs;             /* circles per scene ([x, y, R] each)              */
  double dt;                 /* T / N                                           */
  double lambda;             /* λ                                               */
  double sigma[4];           /* Σ, row-major 2x2                                */
  double XL[MP_NX], XU[MP_NX];
  double CL[MP_NU], CU[MP_NU];
  double slack_penalty;      /* SlackPenalty (1e5)                              */
  double obs_penalty;        /* 100*712.5 (MPPIUtils.jl:127); DWA: 10000*712.5  */
  int32_t grid_nx, grid_ny;  /* occupancy grid (build extension), 0 = none      */
  double grid_x0, grid_y0, grid_dx, grid_dy;
  int32_t noise_mode;        /* MP_NOISE_*                                      */
  int32_t ctrl_cost;         /* 1: λ·u_nomᵀΣ⁻¹(u−u_nom) term (MPPIUtils.jl:45)  */
  uint64_t seed;             /* Philox key                                      */
  uint64_t offset;           /* Philox counter word (advance per solve)         */
  int32_t scene_base;        /* global index of this call's scene 0 (Philox     */
                             /*   counter word): a rank planning scenes [a,b)   */
                             /*   of a sharded batch passes a, so every scene   */
                             /*   draws the same stream at any world size       */
  int32_t final_stream;      /* 0: the final TrajectoryRollout(MPPICtrl) runs   */
                             /*   at the end of the plan kernel.  1: it runs on */
                             /*   the context's side stream from a snapshot of  */
                             /*   its inputs, overlapping the next call's       */
                             /*   rollouts (see mp_mppi_plan_dev)               */
  int32_t calls_in_flight;   /* 0 / 1: the call has the device to itself.  n > 1:*/
                             /*   the caller keeps n independent calls in       */
                             /*   flight on n contexts of this device (see      */
                             /*   INTEGRATION.md); the launch then takes the    */
                             /*   layout whose waves share the CUs with the     */
                             /*   other calls' (one rollout per lane).  Same    */
                             /*   rollouts bit for bit either way; MPPICtrl     */
                             /*   within the combine tolerance (the weighted    */
                             /*   sum's partition may differ)                   */
} mp_mppi_params;

/*
 * mp_mppi_plan — one MPPIPlan(mppi) per scene (OptimalControl/MPPI/src/MPPIUtils.jl:169-203),
 * S independent scenes per call.
 *
 * in : X0[S][7]       MPPI.s.X0 (ShiftInitialCondition, MPPIUtils.jl:24-27)
 *      goal[S][2]     MPPI.s.goal
 *      U_nom[S][H][2] MPPI.s.NominalControl (defineMPPINominalControl!, setup.jl:70-80)
 *      obstacles[S][n_obs][3]  MPPI.s.obstacle_list (defineMPPIobs!, setup.jl:61-64), may be NULL if n_obs == 0
 *      grid[S][ny][nx] uint8 occupancy (1 = occupied), NULL if grid_nx == 0
 *      noise[S][K][H][2]  standard normals z (MP_NOISE_EXTERNAL), else NULL;
 *                     control = clamp(U_nom + L z, CL, CU), L = chol(Σ).L (MPPIUtils.jl:5-20)
 * out: U_out[S][H][2]       MPPI.r.Control (= MPPICtrl)
 *      traj_out[S][H+1][7]  MPPI.r.Traj
 *      cost_out[S]          MPPI.r.cost
 *      feasible_out[S]      MPPI.r.Feasibility (1 = :Feasible)
 *      rollout_count_out[S] MPPI.r.RolloutCount (= m + 1, reference off-by-one)
 *      feasible_count_out[S] MPPI.r.FeasibleTrajCount
 * optional (NULL to skip) — MPPI.p.TrajectoryCollection[1:K] (types.jl:3-8):
 *      coll_traj[S][H+1][7][K], coll_ctrl[S][H][K][2], coll_cost[S][K], coll_feas[S][K]
 *      — structure of arrays, rollout index k fastest (Julia (K, 7, H+1, S) and
 *      (2, K, H, S)): holder k's Trajectory is coll_traj[s][:, :, k] transposed, and a
 *      wavefront's per-step stores for 32 consecutive rollouts are full 128-B lines.
 *      (all K rollouts are written; the planner uses the first m = rollout_count-1).
 * Returns MP_ERR_NUMERIC (after writing outputs) if any rollout cost was NaN.
 */
int mp_mppi_plan(mp_ctx* ctx, const mp_mppi_params* p, int32_t S, const double* X0,
                 const double* goal, const double* U_nom, const double* obstacles,
                 const uint8_t* grid, const double* noise, double* U_out, double* traj_out,
                 double* cost_out, int32_t* feasible_out, int32_t* rollout_count_out,
                 int32_t* feasible_count_out, double* coll_traj, double* coll_ctrl,
                 double* coll_cost, uint8_t* coll_feas);

/* Same contract, DEVICE pointers, asynchronous on the context stream.
 * With p->final_stream = 1, U_out, rollout/feasible counts and the TrajectoryCollection
 * are complete in context-stream order as usual, while traj_out, cost_out and
 * feasible_out (the final rollout, MPPIUtils.jl:192-198) are written by the side stream:
 * read them after mp_ctx_join() (stream order) or mp_ctx_synchronize().  The inputs may
 * be overwritten as soon as the context stream has passed the call (the side stream
 * works on a device snapshot).  The NaN check of the final cost is not reported. */
int mp_mppi_plan_dev(mp_ctx* ctx, const mp_mppi_params* p, int32_t S, const double* X0,
                     const double* goal, const double* U_nom, const double* obstacles,
                     const uint8_t* grid, const double* noise, double* U_out, double* traj_out,
                     double* cost_out, int32_t* feasible_out, int32_t* rollout_count_out,
                     int32_t* feasible_count_out, double* coll_traj, double* coll_ctrl,
                     double* coll_cost, uint8_t* coll_feas);

/*
 * mp_rollout — batched TrajectoryRollout with given controls
 * (MPPIUtils.jl:31-57; DynamicWindow/src/DWAUtils.jl:16-42).
 * ctrl[S][K][H][2] with the H stride given in elements (ctrl_stride_h = 2 for a
 * full control list, 0 for DWA's constant controls [S][K][2]); no clamping.
 * U_nom[S][H][2] is used only when p->ctrl_cost != 0.
 * out: traj[S][K][H+1][7] (optional), cost[S][K], feas[S][K],
 *      argmin[S] (optional; first minimum, Julia `minimum`/`argmin` on cost).
 * p->K is ignored; K is the argument.
 */
int mp_rollout(mp_ctx* ctx, const mp_mppi_params* p, int32_t S, int32_t K, const double* X0,
               const double* goal, const double* ctrl, int64_t ctrl_stride_h,
               const double* U_nom, const double* obstacles, const uint8_t* grid,
               double* traj, double* cost, uint8_t* feas, int32_t* argmin);

/*
 * mp_vehicle_euler — the closed-loop plant of MPPI/main.jl:259-261 and
 * DynamicWindow/main.jl:155-156: states .+= VehicleDynamics(states, u)*δt for
 * nsteps steps with control ctrl[n][2] held constant (zero-order hold).
 * states[n][7] updated in place; his[n][nsteps][7] (optional) gets every state.
 */
int mp_vehicle_euler(mp_ctx* ctx, int32_t n, double* states, const double* ctrl, double dt,
                     int32_t nsteps, double* his);

/* Closed-loop driver settings (OptimalControl/MPPI/main.jl:14-19,55-83). */
typedef struct mp_mppi_loop_params {
  int32_t update_steps; /* plant steps per replan: update_idx = Int32(floor(update_time/δt)) (main.jl:19) */
  int32_t max_steps;    /* plant steps of the run: Int32(floor(15/δt)) (main.jl:55)                     */
  double plant_dt;      /* δt (main.jl:18)                                                           */
  double goal_radius;   /* stop after the plant step that ends within this distance of goal (main.jl:80: 6) */
  int32_t poll_every;   /* replans enqueued between host checks of the live-scene flags (0: 8)        */
  int32_t reserved;
} mp_mppi_loop_params;

/*
 * mp_mppi_closed_loop — the MPPI closed loop of OptimalControl/MPPI/main.jl:55-83 for S independent
 * scenes (egos) in lockstep, entirely on the device.  Every update_steps plant steps (and at
 * step 1): ShiftInitialCondition(mppi, states); defineMPPINominalControl!(mppi, NominalControls);
 * MPPIPlan(mppi); NominalControls = mppi.r.Control.  Each plant step applies
 * controls[i] = NominalControls[hold_idx[i] + 1, :] (0-based row hold_idx[i] of U; the caller's
 * interpolate(time_serial, ·, Gridded(Constant{Previous}()))(fined_time_serial), main.jl:64-66),
 * i = (time_idx − 1) mod update_steps, and states .+= VehicleDynamics(states, u)·δt (main.jl:74-75).
 * A scene stops after the step whose (x, y) is within goal_radius of its goal (main.jl:77-79);
 * the others go on.  Replan r of every scene uses Philox counter word p->offset + r (MP_NOISE_PHILOX)
 * or the caller's z (MP_NOISE_EXTERNAL).  The final rollout of each plan runs on the side stream
 * (p->final_stream is ignored), beside the plant.
 *
 * in : X0[S][7], goal[S][2], U_nom0[S][H][2] (NominalControls before the first plan),
 *      obstacles[S][n_obs][3], grid[S][ny][nx] as mp_mppi_plan,
 *      hold_idx[update_steps] (0-based rows of U, each in [0, H)),
 *      noise[R][S][K][H][2] (MP_NOISE_EXTERNAL; R = ceil(max_steps / update_steps)) or NULL.
 * out: his[S][max_steps+1][8]  states_his' rows [time_idx·δt, states...]; row 0 = [0, X0]
 *      n_rows[S]               rows written (time steps run + 1)
 *      n_replans[S]            MPPIPlan calls made for the scene
 * optional (NULL to skip), per replan r < n_replans[s]:
 *      U_log[S][R][H][2] (mppi.r.Control), traj_log[S][R][H+1][7] (mppi.r.Traj),
 *      cost_log[S][R] (mppi.r.cost), feas_log[S][R] (mppi.r.Feasibility),
 *      rc_log[S][R] (mppi.r.RolloutCount).
 * Returns MP_ERR_NUMERIC (after writing outputs) if any rollout cost was NaN.
 */
int mp_mppi_closed_loop(mp_ctx* ctx, const mp_mppi_params* p, const mp_mppi_loop_params* lp, int32_t S,
                        const double* X0, const double* goal, const double* U_nom0, const double* obstacles,
                        const uint8_t* grid, const int32_t* hold_idx, const double* noise, double* his,
                        int32_t* n_rows, int32_t* n_replans, double* U_log, double* traj_log, double* cost_log,
                        int32_t* feas_log, int32_t* rc_log);

/* ----------------------------------------------------------- multi-GPU */
/*
 * One host process driving several GPUs (the Julia host of OptimalControl/MPPI/main.jl:59-61 keeps
 * its single process): one context per GPU, joined into one RCCL communicator
 * (ncclCommInitAll over the contexts' devices, xGMI between MI355X GPUs).  ctxs[i] is rank i; every
 * call below takes the same array in the same order.  Errors are reported on ctxs[0]
 * (mp_last_error(ctxs[0])).  RCCL is loaded on first use: MP_ERR_UNSUPPORTED without librccl.
 * Call mp_comm_destroy before destroying the contexts: mp_ctx_destroy refuses (MP_ERR_INVALID) a
 * context that still belongs to a communicator.
 */
int mp_comm_init(mp_ctx** ctxs, int32_t n);
int mp_comm_destroy(mp_ctx** ctxs, int32_t n);
/* ncclAllGather of `bytes` bytes per rank: DEVICE buffers send[i] (on ctxs[i]'s GPU) -> recv[i]
 * ([n][bytes], rank-major), enqueued on every context stream (asynchronous). */
int mp_comm_allgather_dev(mp_ctx** ctxs, int32_t n, void* const* send, void* const* recv, size_t bytes);

/*
 * mp_mppi_plan_sharded — multi-ego MPPIPlan (MPPIUtils.jl:169-203) of S independent scenes sharded over
 * the n GPUs of a communicator: ctxs[r] plans the balanced block [a_r, b_r) of scenes (the first
 * S mod n ranks take one extra) with Philox counter word p->scene_base + a_r — so every scene draws
 * the noise it draws in one mp_mppi_plan over all S — then one RCCL all-gather of the per-scene
 * results (MPPICtrl, final trajectory, cost, flags, counts: (2H + 7(H+1) + 4) doubles per scene) leaves
 * every GPU holding all S scenes' optimal controls; the host outputs are copied from ctxs[0]'s copy.
 * Inputs and outputs as mp_mppi_plan over all S scenes (HOST pointers, synchronous); the
 * TrajectoryCollection stays per GPU and is not returned here.
 */
int mp_mppi_plan_sharded(mp_ctx** ctxs, int32_t n, const mp_mppi_params* p, int32_t S, const double* X0,
                         const double* goal, const double* U_nom, const double* obstacles, const uint8_t* grid,
                         const double* noise, double* U_out, double* traj_out, double* cost_out,
                         int32_t* feasible_out, int32_t* rollout_count_out, int32_t* feasible_count_out);

/* ---------------------------------------------------------------- iLQR */
#define MP_ILQR_NX 4 /* [x, y, ux, ψ]  OptimalControl/ILQR/Dynamics.jl:4-7 */
#define MP_ILQR_NU 2 /* [ax, δ]                                          */
#define MP_ILQR_OPTIMALCONTROL 0 /* OptimalControl/ILQR/Cost.jl           */
#define MP_ILQR_PARKING 1        /* PathPlanning/Parking_ILQR/Cost.jl     */

typedef struct mp_ilqr_params {
  int32_t N;           /* knots per trajectory (ILQR.jl:15: 20; Parking: 30) */
  int32_t variant;     /* MP_ILQR_*: cost weights                            */
  double dT;           /* δT = 0.05                                          */
  double eps;          /* finite-difference step ϵ = 1e-3 (GetMatrix.jl:4)   */
  double alpha_floor;  /* 0: none (ILQR.jl:71-82); 1e-3 Parking_ILQR.jl:83-85 */
  double tol;          /* |ΔJ/J| stop (ILQR.jl:44): 1e-6                     */
  int32_t max_iter;    /* safety cap on outer iterations (reference: none)   */
  int32_t max_ls;      /* safety cap on line-search halvings (reference: none) */
} mp_ilqr_params;

/* Layouts (Julia column-major in parentheses):
 *   X[B][N][4]  (StatesList 4×N per instance)   U[B][N][2]  (CtrlsList 2×N)
 *   k[B][N-1][2]  (klist 2×1×(N-1))              Kg[B][N-1][4][2]  (Klist 2×4×(N-1))  */

/* Initial-guess roll out (ILQR.jl:31-37) + TotalCost (Cost.jl:1-8). */
int mp_ilqr_rollout(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* x0,
                    const double* U, double* X, double* J);
/* One backward Riccati sweep (ILQR.jl:46-67). */
int mp_ilqr_backward(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X,
                     const double* U, double* k, double* Kg);
/* One forward trial at step size alpha[B] (ILQR.jl:72-80): closed-loop RK4 roll out. */
int mp_ilqr_forward(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X,
                    const double* U, const double* k, const double* Kg, const double* alpha,
                    double* Xnew, double* Unew, double* Jnew);
/* Same contracts, DEVICE pointers, asynchronous on the context stream. */
int mp_ilqr_backward_dev(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X,
                         const double* U, double* k, double* Kg);
int mp_ilqr_forward_dev(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, const double* X,
                        const double* U, const double* k, const double* Kg, const double* alpha,
                        double* Xnew, double* Unew, double* Jnew);
/* The whole script loop (ILQR.jl:39-88) per instance: backward + halving line
 * search until |ΔJ/J| <= tol.  X/U in: initial guess; out: solution. */
int mp_ilqr_solve(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, double* X, double* U,
                  double* J, int32_t* iters);
/* Same, DEVICE pointers: X (B,N,4) / U (B,N,2) solved in place, J (B) and iters (B) written on the
 * device.  Synchronous like mp_ilqr_solve (its host loop polls the active count every iteration); it
 * only skips the host transfers -- the form the bench times, inputs resident in HBM. */
int mp_ilqr_solve_dev(mp_ctx* ctx, const mp_ilqr_params* p, int32_t B, double* X, double* U,
                      double* J, int32_t* iters);

/* ---------------------------------------------------------- Hybrid A* */
/* Settings mirror HybridAstarSettings (PathPlanning/HybridAstar/src/types.jl:20-43). */
typedef struct mp_ha_params {
  double vehicle_len, vehicle_wid; /* vehicle_size                               */
  double minR;                     /* minimum turning radius                     */
  double expand_time;              /* primitive length in time (2.5)             */
  double res[3];                   /* resolutions [x, y, ψ]                      */
  double stbound[6];               /* regulated [xmin, xmax, ymin, ymax, ψmin, ψmax] */
  int32_t n_walls;                 /* obstacle blocks per scene, [x,y,ψ,l/2,w/2] */
  int32_t n_prim;                  /* num_neighbors = num_gear*num_steer (62)    */
  int32_t n_col;                   /* primitive path columns (250)               */
  int32_t max_pops;                /* safety cap on search iterations            */
} mp_ha_params;

/* neighbor_origin (hybrid_astar_utils.jl:483-503) computed by the library (FDLIBM sin/cos,
 * Euler Δt = 1e-2, n_col = floor(expand_time/Δt)), returned and installed in the context:
 * states_candi[n_gear*n_steer][3], paths_candi[n_gear*n_steer][n_col][3] (either may be NULL: not
 * returned).  A repeat call with the same settings as the installed table returns its copies without
 * recomputing or re-uploading it (mp_ha_set_primitives clears that memo). */
int mp_ha_neighbor_origin(mp_ctx* ctx, const mp_ha_params* p, int32_t n_steer, const double* steer_set,
                          int32_t n_gear, const double* gear_set, double* states_candi, double* paths_candi);

/* Primitive table of neighbor_origin (hybrid_astar_utils.jl:483-503):
 * states_candi[n_prim][3], paths_candi[n_prim][n_col][3]  (Julia 3×n_prim, 3×n_col×n_prim). */
int mp_ha_set_primitives(mp_ctx* ctx, const mp_ha_params* p, const double* states_candi,
                         const double* paths_candi);

/* Batched FindNewNode device part (hybrid_astar_utils.jl:391-421) for B popped nodes:
 *   node[B][3], goal[B][3] (ending_states), walls[B][n_walls][5]
 * out: nb_states[B][n_prim][3] regulated neighbor states,
 *      idx[B][n_prim]  Encode (0 = out of bounds),
 *      free_[B][n_prim] 1 if in bounds and dg_cost finite (collision free),
 *      h[B][n_prim]     rs_heuristic (valid where free_ == 1). */
int mp_ha_expand(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* node,
                 const double* goal, const double* walls, double* nb_states, int64_t* idx,
                 uint8_t* free_, double* h);

/* Batched RS_connected (hybrid_astar_utils.jl:224-233): optimal Reeds–Shepp
 * path from node to goal, its 100-steps-per-segment Euler path and the
 * collision check.  path[B][501][3] (first path_len[B] columns valid). */
int mp_ha_rs_connect(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* node,
                     const double* goal, const double* walls, uint8_t* ok, double* path,
                     int32_t* path_len);

/* Whether the collision sweeps of mp_ha_expand / mp_ha_rs_connect / mp_ha_plan use their SAT culls
 * (certain-result SeparatingAxisTheorem calls skipped, CollisionDetection/src/utils.jl:37-74) for these
 * inputs: *active = 1 when every coordinate and length (walls[B][n_walls][5] centres + half extents,
 * stbound, a[B][3] and b[B][3] x/y -- start or node, goal -- minR, vehicle and primitive sizes) is
 * <= 1e6 m, the range the culls' rounding margin is proven for; 0 otherwise (every SAT call runs).
 * Either way the booleans are the reference's.  No device work. */
int mp_ha_sat_cull_active(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* walls, const double* a,
                          const double* b, int32_t* active);

/* allpath (ReedsSheppsCurves/src/ReedsSheppsUtils.jl:468-511) for B normalised
 * states; out: cost[B][48] (Inf where infeasible), cmds[B][48][5][3], best[B]. */
int mp_ha_allpath(mp_ctx* ctx, int32_t B, const double* norm_states, double* cost,
                  double* cmds, int32_t* best);

/* Whole planHybridAstar! search loop (hybrid_astar_utils.jl:235-296) for B
 * scenes in lockstep, entirely on the device: per iteration one fused
 * RS-connect + expansion launch and one bookkeeping launch (Dict, open list in
 * the reference's stable-sort order, popfirst!), enqueued without host round
 * trips.  n_prim <= 64.  start[B][3], goal[B][3] already regulated
 * (setup.jl:110-112).
 * out: found[B], pops[B] (loop_count), n_nodes[B] (length(nodes_collection)),
 *      pop_seq[B][max_pops] (Encode index of each popped node, -1 padded),
 *      n_states[B] and states_out[B][max_pops][3] (hybrid_astar_states, goal→start order),
 *      rs_len[B] and rs_path[B][501][3] (RSpath_final). */
int mp_ha_plan(mp_ctx* ctx, const mp_ha_params* p, int32_t B, const double* start,
               const double* goal, const double* walls, int32_t* found, int32_t* pops,
               int32_t* n_nodes, int64_t* pop_seq, int32_t* n_states, double* states_out,
               int32_t* rs_len, double* rs_path);

/* retrievePath + cubic_fit (PathPlanning/HybridAstar/src/hybrid_astar_utils.jl:100-177) for B planned
 * scenarios, one block each: actualpath = [starting_states, cubic_fit(states[:,i], states[:,i+1]) (100
 * points each, i over the hybrid_astar_states reversed to start -> goal order), RSpath_final], its
 * cumulative arc length path_length, tol_length = path_length[end], and the 50 samples of
 * x/y/ψ_interp_dense at LinRange(0, tol_length, 50) that x/y/ψ_interp are built on.
 * in : start[B][3] (starting_states), n_states[B] and states[B][state_stride][3] as mp_ha_plan returns
 *      them (goal side first; n_states = 0: nothing found, nothing retrieved), rs_len[B],
 *      rs_path[B][501][3] (RSpath_final).
 * out: n_points[B] = 1 + 100 (n_states - 1) + rs_len (0 if n_states = 0), tol_length[B],
 *      samples[B][50][3] (x, y, ψ at the 50 arc-length knots).
 * optional (all NULL or path_offset given): path_offset[B+1] (written: scenario b's points are
 *      [path_offset[b], path_offset[b+1])), actualpath[path_offset[B]][3], path_length[path_offset[B]]. */
int mp_ha_retrieve_path(mp_ctx* ctx, int32_t B, const double* start, const int32_t* n_states, const double* states,
                        int32_t state_stride, const int32_t* rs_len, const double* rs_path, int64_t* path_offset,
                        double* actualpath, double* path_length, int32_t* n_points, double* tol_length,
                        double* samples);

/* ------------------------------------------------------- path tracker */
/* Settings of the Hybrid A* path tracker (PathPlanning/HybridAstar/main_Tracker.jl:42-72). */
typedef struct mp_track_params {
  int32_t n_ref;      /* refined_length = LinRange(0, tol_length, n_ref): 1000 (:42); <= 2048           */
  int32_t max_steps;  /* safety cap on simulation steps (the reference loops until the closest point
                         is the last one, :84)                                                          */
  double dt_sim;      /* 1e-3 (:67)                                                                     */
  double look_ahead;  /* look_ahead_dist 1.0 (:57)                                                      */
  double p_gain;      /* 10 (:58)                                                                       */
  double i_gain;      /* 0.1 (:59)                                                                      */
  double veh_len;     /* veh_param[1] = vehicle_size[1] (:50)                                           */
  double max_sa;      /* veh_param[3] = max_δf + 0.1 (:52)                                              */
  int32_t his_stride; /* states_his: keep the state after every his_stride-th update (0: none)          */
  int32_t reserved;
} mp_track_params;

#define MP_TRACK_DONE 0    /* the closest reference point reached the last one (main_Tracker.jl:84-89) */
#define MP_TRACK_MAXSTEP 1 /* max_steps simulation steps ran without reaching it                         */
#define MP_TRACK_NOPATH 2  /* tol_length not > 0 (no planned path: "Can't find a path", :31-35)         */
#define MP_TRACK_EMPTY 3   /* an empty findclosest window (argmin of an empty range: a Julia error)      */

/*
 * mp_ha_track — the HA* -> tracker hand-off and the tracker closed loop of
 * PathPlanning/HybridAstar/main_Tracker.jl:42-137 for B planned scenarios in lockstep, one wavefront
 * each.  x_ref/y_ref/ψ_ref = x/y/ψ_interp(refined_length) (:42-46, Interpolations.jl linear
 * interpolation on the n_samples knots LinRange(0, tol_length, n_samples)); then per step
 * (simulation_idx = 1, 2, ...): findclosest (tracker_utils.jl:38-43) inside the time windows of
 * :82-90, inverseKinematic (tracker_utils.jl:15-36), the look-ahead point and its findclosest
 * (:97-108), the cross-track PI correction with clamp (:110-119) and the kinematic Euler step
 * (tracker_utils.jl:1-13, :121).
 * in : start_real[B][3] (cur_states = starting_real, :64), tol_length[B] and samples[B][n_samples][3]
 *      as mp_ha_retrieve_path returns them (x/y/ψ_interp values at their knots).
 * out: n_steps[B] (simulation_idx when the loop ended), status[B] (MP_TRACK_*),
 *      final_state[B][3] (cur_states), err_acc[B] (err_accumulated),
 * optional (NULL to skip): ref_out[B][n_ref][3] (x_ref, y_ref, ψ_ref: the hand-off),
 *      his[B][his_cap][3]: states_his (:122) every his_stride-th update, row 0 = starting_real;
 *      rows written = min(his_cap, (n_steps - 1) / his_stride + 1).
 */
int mp_ha_track(mp_ctx* ctx, const mp_track_params* p, int32_t B, const double* start_real,
                const double* tol_length, const double* samples, int32_t n_samples, int32_t* n_steps,
                int32_t* status, double* final_state, double* err_acc, double* ref_out, double* his,
                int32_t his_cap);

/* ---------------------------------------------------------- diagnostics */
/* Evaluate one include/mp_jlmath.h function on the device for n inputs
 * (bit-exactness check against the CPU build).  fn: 0 sin, 1 cos, 2 tan, 3 atan,
 * 4 atan2(x, y), 5 asin, 6 acos, 7 exp, 8 log, 9 modpi, 10 sqrt; the branch-free
 * variants of the hot kernels: 11 modpi_bl, 12 atan_bl, 13 atan_tab, 14 sin (sincos_bl),
 * 15 cos (sincos_bl), 16 exp_fdlibm, 17 tan_bl, 18 atan2_sel(x, y), 19 sin / 20 cos (sincos_wide),
 * 21 tan_wide, 22 sin_34 (tyre sin, |x| <= 3π/4 fast path), 23 log_bl — each must equal its exact
 * routine bit for bit. */
int mp_math_eval(mp_ctx* ctx, int32_t fn, int64_t n, const double* x, const double* y, double* out);

#ifdef __cplusplus
}
#endif
#endif /* MPGPU_H */
