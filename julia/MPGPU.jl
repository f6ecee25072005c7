"""
    MPGPU

Julia binding of libmpgpu.so (include/mpgpu.h) for the reference's planner scripts.
`include("MPGPU.jl")` after the reference's own `include("src/...")` lines and the
hot-path functions below take over the reference's names on the same searcher objects:

  * `MPPIPlan(mppi::MPPISearcher)`      OptimalControl/MPPI/src/MPPIUtils.jl:169-203
  * `TrajectoryRollout(mppi, ctrl)`     MPPIUtils.jl:31-57 (batched form: `rollout_batch`)
  * `MPPIClosedLoop(mppi)`              the replan / plant loop of OptimalControl/MPPI/main.jl:49-83
  * `mppi_plan_sharded` (+ `comm_init`) multi-ego MPPIPlan over all GPUs of the node from one process
                                        (RCCL all-gather of the optimal controls)
  * `planHybridAstar!(ha)`              PathPlanning/HybridAstar/src/hybrid_astar_utils.jl:235-296
  * `RS_connected`, `FindNewNode` device parts (`ha_rs_connect`, `ha_expand`)
  * iLQR passes (`ilqr_backward!`, `ilqr_forward!`, `ilqr_solve!`)  OptimalControl/ILQR/ILQR.jl:44-88
  * `retrieve_batch!` (retrievePath + cubic_fit, hybrid_astar_utils.jl:100-177) and `track_batch!`
    (the HA* -> tracker hand-off and tracker loop of PathPlanning/HybridAstar/main_Tracker.jl:42-137)

Errors: every non-zero status is re-raised as `error(mp_last_error(ctx))`, the style of
the reference's own validation (MPPI/src/setup.jl:19-38).  Arrays are passed in Julia's
native column-major layout; each call documents the Julia shape (the C header writes the
same buffer in reversed, row-major order).

This file cannot be executed in the build container (no Julia toolchain); the same entry
points are exercised from Python ctypes by tests/ with identical layouts.
"""
module MPGPU

using Interpolations: interpolate, Gridded, Constant, Previous, linear_interpolation   # as the reference drivers

export MPPIPlan, MPPIClosedLoop, planHybridAstar!, mppi_plan_batch, mppi_plan_sharded, comm_init, mppi_closed_loop_batch,
       rollout_batch, ha_expand, ha_rs_connect,
       ha_allpath, ha_neighbor_origin, retrieve_batch!, track_batch!, ilqr_rollout, ilqr_backward!, ilqr_forward!,
       ilqr_solve!, vehicle_euler!, ctx_join

const libmpgpu = get(ENV, "MPGPU_LIB", joinpath(@__DIR__, "..", "motionplanning_amd", "lib", "libmpgpu.so"))

const MP_OK = Cint(0)
const MP_ERR_NUMERIC = Cint(4)
const MP_NOISE_EXTERNAL = Int32(0)
const MP_NOISE_PHILOX = Int32(1)

# ------------------------------------------------------------------ context
const CTX = Ref{Ptr{Cvoid}}(C_NULL)

last_error(c::Ptr{Cvoid}) = unsafe_string(ccall((:mp_last_error, libmpgpu), Cstring, (Ptr{Cvoid},), c))

function check(st::Cint, c::Ptr{Cvoid} = CTX[])
    st == MP_OK || error("libmpgpu: ", last_error(c))
    return nothing
end

"""One context (device + HIP stream + cached workspaces) per process; device = LOCAL_RANK."""
function ctx(device::Integer = parse(Int, get(ENV, "LOCAL_RANK", "0")))
    if CTX[] == C_NULL
        r = Ref{Ptr{Cvoid}}(C_NULL)
        st = ccall((:mp_ctx_create, libmpgpu), Cint, (Cint, Ref{Ptr{Cvoid}}), device, r)
        st == MP_OK || error("libmpgpu: ", last_error(Ptr{Cvoid}(C_NULL)))
        CTX[] = r[]
        atexit(() -> (ccall((:mp_ctx_destroy, libmpgpu), Cint, (Ptr{Cvoid},), CTX[]); CTX[] = C_NULL))
    end
    return CTX[]
end

# --------------------------------------------------------------------- MPPI
"""mp_mppi_params, field for field (isbits => C layout)."""
struct MppiParams
    K::Int32
    H::Int32
    feasibility_count::Int32
    n_obs::Int32
    dt::Float64
    lambda::Float64
    sigma::NTuple{4,Float64}      # Σ row-major
    XL::NTuple{7,Float64}
    XU::NTuple{7,Float64}
    CL::NTuple{2,Float64}
    CU::NTuple{2,Float64}
    slack_penalty::Float64
    obs_penalty::Float64
    grid_nx::Int32
    grid_ny::Int32
    grid_x0::Float64
    grid_y0::Float64
    grid_dx::Float64
    grid_dy::Float64
    noise_mode::Int32
    ctrl_cost::Int32
    seed::UInt64
    offset::UInt64
    scene_base::Int32
    final_stream::Int32
    calls_in_flight::Int32
end

"""MppiParams from an MPPISearcher's settings (MPPI/src/types.jl:10-31, setup.jl:3-59)."""
function params(mppi; noise_mode = MP_NOISE_PHILOX, seed = 0, offset = 0, grid = nothing)
    s = mppi.s
    Σ = Matrix{Float64}(s.Σ)
    nx, ny, x0, y0, dx, dy = 0, 0, 0.0, 0.0, 0.0, 0.0
    if grid !== nothing            # (occupancy::Matrix{UInt8} (nx, ny), x0, y0, dx, dy) — build extension
        occ, x0, y0, dx, dy = grid
        nx, ny = size(occ)
    end
    MppiParams(s.SamplingNumber, s.N, s.FeasibilityCount, length(s.obstacle_list), s.dt, s.lambda,
               (Σ[1, 1], Σ[1, 2], Σ[2, 1], Σ[2, 2]), Tuple(s.XL), Tuple(s.XU), Tuple(s.CL), Tuple(s.CU),
               s.SlackPenalty, 100 * 712.5, nx, ny, x0, y0, dx, dy, noise_mode, 1, seed, offset, 0, 0, 0)
end

"""
    mppi_plan_batch(p, X0, goal, Unom; obstacles, grid, noise, collect) -> NamedTuple

S scenes in one launch.  Julia shapes: X0 (7, S), goal (2, S), Unom (2, H, S),
obstacles (3, n_obs, S), grid occupancy (nx, ny, S) UInt8, noise z (2, H, K, S) or
`nothing` (device Philox).  Returns U (2, H, S), traj (7, H+1, S), cost, feasible,
rollout_count, feasible_count (S,) and, with `collect`, the TrajectoryCollection arrays
(structure of arrays, rollout index first) coll_traj (K, 7, H+1, S), coll_ctrl (2, K, H, S),
coll_cost (K, S), coll_feas (K, S).
"""
function mppi_plan_batch(p::MppiParams, X0::Matrix{Float64}, goal::Matrix{Float64}, Unom::Array{Float64,3};
                         obstacles = nothing, grid = nothing, noise = nothing, collect::Bool = false)
    S = size(X0, 2); H = Int(p.H); K = Int(p.K)
    p = noise === nothing ? p : MppiParams(ntuple(i -> i == 20 ? MP_NOISE_EXTERNAL : getfield(p, i), 26)...)
    U = zeros(2, H, S); traj = zeros(7, H + 1, S); cost = zeros(S)
    feas = zeros(Int32, S); rc = zeros(Int32, S); fc = zeros(Int32, S)
    ct = collect ? zeros(K, 7, H + 1, S) : nothing
    cc = collect ? zeros(2, K, H, S) : nothing
    ck = collect ? zeros(K, S) : nothing
    cf = collect ? zeros(UInt8, K, S) : nothing
    nz(a) = a === nothing ? C_NULL : pointer(a)
    c = ctx()
    st = GC.@preserve X0 goal Unom obstacles grid noise U traj cost feas rc fc ct cc ck cf begin
        ccall((:mp_mppi_plan, libmpgpu), Cint,
              (Ptr{Cvoid}, Ref{MppiParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
               Ptr{UInt8}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32},
               Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}),
              c, p, S, X0, goal, Unom, nz(obstacles), nz(grid), nz(noise), U, traj, cost, feas, rc, fc,
              nz(ct), nz(cc), nz(ck), nz(cf))
    end
    st == MP_ERR_NUMERIC && @warn "MPPIPlan: NaN rollout cost (outputs written)"
    st == MP_ERR_NUMERIC || check(st, c)
    return (; U, traj, cost, feasible = feas, rollout_count = rc, feasible_count = fc,
            coll_traj = ct, coll_ctrl = cc, coll_cost = ck, coll_feas = cf)
end

const SOLVES = Ref{UInt64}(0)   # per-process solve counter = Philox counter word

"""
    MPPIPlan(mppi; noise = nothing, seed = 0, collect = true)

Drop-in for MPPIUtils.jl:169-203: mutates `mppi.r.{Traj, Control, Feasibility, cost, time,
FeasibleTrajCount, RolloutCount}` and `mppi.p.TrajectoryCollection[1:m]`.  `noise` is the
caller's z (2, N, SamplingNumber) (the draws the reference takes from `MvNormal`); by
default the device Philox stream keyed by `seed` and a per-call counter is used.
"""
function MPPIPlan(mppi; noise = nothing, seed = 0, collect::Bool = true)
    t1 = time()
    s = mppi.s
    p = params(mppi; seed = seed, offset = SOLVES[])
    SOLVES[] += 1
    obs = isempty(s.obstacle_list) ? nothing : reshape(reduce(hcat, s.obstacle_list), 3, :, 1)
    Unom = reshape(permutedims(Matrix{Float64}(s.NominalControl)), 2, s.N, 1)   # N×2 -> (2, N, 1)
    z = noise === nothing ? nothing : reshape(noise, 2, s.N, s.SamplingNumber, 1)
    r = mppi_plan_batch(p, reshape(s.X0, 7, 1), reshape(s.goal, 2, 1), Unom; obstacles = obs, noise = z,
                        collect = collect)
    mppi.r.Control = permutedims(r.U[:, :, 1])          # N×2
    mppi.r.Traj = permutedims(r.traj[:, :, 1])          # (N+1)×7
    mppi.r.Feasibility = r.feasible[1] == 1 ? :Feasible : :InFeasible
    mppi.r.cost = r.cost[1]
    mppi.r.RolloutCount = r.rollout_count[1]
    mppi.r.FeasibleTrajCount = r.feasible_count[1]
    if collect
        m = r.rollout_count[1] - 1
        hold = eltype(mppi.p.TrajectoryCollection)
        mppi.p.TrajectoryCollection = [hold(permutedims(r.coll_traj[k, :, :, 1]), permutedims(r.coll_ctrl[:, k, :, 1]),
                                            r.coll_feas[k, 1] == 1, r.coll_cost[k, 1]) for k in 1:m]
    end
    mppi.r.time = time() - t1
    return nothing
end

struct MppiLoopParams
    update_steps::Int32
    max_steps::Int32
    plant_dt::Float64
    goal_radius::Float64
    poll_every::Int32
    reserved::Int32
end

"""
    mppi_closed_loop_batch(p, X0 (7,S), goal (2,S), Unom0 (2,H,S), hold::Vector{Int32}, update_idx, max_steps,
                           δt, goal_radius; obstacles, noise (2,H,K,S,R)) -> NamedTuple

S closed loops of OptimalControl/MPPI/main.jl:55-83 in lockstep on the device (mp_mppi_closed_loop).
`grid` is the occupancy grid (grid_nx, grid_ny, S) UInt8 of the MppiParams, or `nothing`.
`hold[i]` is the 1-based row of NominalControls the interpolation picks at plant step i of a
period.  Returns his (8, max_steps+1, S) with n_rows[s] valid columns (the states_his matrix of
main.jl per scene), n_replans, and per-replan logs U (2, H, R, S), traj (7, H+1, R, S),
cost / feasible / rollout_count (R, S).
"""
function mppi_closed_loop_batch(p::MppiParams, X0::Matrix{Float64}, goal::Matrix{Float64},
                                Unom0::Array{Float64,3}, hold::Vector{Int32}, update_idx::Integer,
                                max_steps::Integer, δt::Float64, goal_radius::Float64;
                                obstacles = nothing, grid = nothing, noise = nothing, poll_every::Integer = 0)
    S = size(X0, 2); H = Int(p.H)
    R = cld(max_steps, update_idx)
    p = noise === nothing ? p : MppiParams(ntuple(i -> i == 20 ? MP_NOISE_EXTERNAL : getfield(p, i), 26)...)
    lp = MppiLoopParams(update_idx, max_steps, δt, goal_radius, poll_every, 0)
    h0 = Int32.(hold .- 1)
    his = zeros(8, max_steps + 1, S); nr = zeros(Int32, S); np_ = zeros(Int32, S)
    U = zeros(2, H, max(R, 1), S); traj = zeros(7, H + 1, max(R, 1), S)
    cost = zeros(max(R, 1), S); feas = zeros(Int32, max(R, 1), S); rc = zeros(Int32, max(R, 1), S)
    nz(a) = a === nothing ? C_NULL : pointer(a)
    c = ctx()
    grid === nothing || size(grid) == (Int(p.grid_nx), Int(p.grid_ny), S) ||
        error("grid must be UInt8 (grid_nx, grid_ny, S) = ", (p.grid_nx, p.grid_ny, S))
    st = GC.@preserve X0 goal Unom0 obstacles grid h0 noise his nr np_ U traj cost feas rc begin
        ccall((:mp_mppi_closed_loop, libmpgpu), Cint,
              (Ptr{Cvoid}, Ref{MppiParams}, Ref{MppiLoopParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
               Ptr{Float64}, Ptr{UInt8}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32},
               Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}),
              c, p, lp, S, X0, goal, Unom0, nz(obstacles), nz(grid), h0, nz(noise), his, nr, np_, U, traj, cost,
              feas, rc)
    end
    st == MP_ERR_NUMERIC && @warn "MPPI closed loop: NaN rollout cost (outputs written)"
    st == MP_ERR_NUMERIC || check(st, c)
    return (; his, n_rows = nr, n_replans = np_, U, traj, cost, feasible = feas, rollout_count = rc)
end

"""
    MPPIClosedLoop(mppi; update_time = 0.1, δt = 1e-3, sim_time = 15, goal_radius = 6, seed = 0)

The driver loop of OptimalControl/MPPI/main.jl:49-83 (without plotting) on the device: returns
`states_his` (8 × n, rows [t; states], as main.jl builds it and MPPITrajectory.csv stores
transposed) and leaves the last plan in `mppi.r`.  The zero-order hold is the reference's own
`interpolate((time_serial,), ·, Gridded(Constant{Previous}()))` evaluated on the row indices.
"""
function MPPIClosedLoop(mppi; update_time = 0.1, δt = 1e-3, sim_time = 15, goal_radius = 6.0, seed = 0)
    s = mppi.s
    update_idx = Int32(floor(update_time / δt))
    max_steps = Int32(floor(sim_time / δt))
    time_serial = collect(range(0.0, s.T, length = s.N))
    fined_time_serial = collect(range(0.0, update_time, length = update_idx))
    rows = interpolate((time_serial,), Float64.(1:s.N), Gridded(Constant{Previous}()))
    hold = Int32.(rows(fined_time_serial))
    p = params(mppi; seed = seed, offset = SOLVES[])
    obs = isempty(s.obstacle_list) ? nothing : reshape(reduce(hcat, s.obstacle_list), 3, :, 1)
    Unom = reshape(permutedims(Matrix{Float64}(s.NominalControl)), 2, s.N, 1)
    r = mppi_closed_loop_batch(p, reshape(Float64.(s.X0), 7, 1), reshape(Float64.(s.goal), 2, 1), Unom, hold,
                               update_idx, max_steps, δt, Float64(goal_radius); obstacles = obs)
    R = r.n_replans[1]
    SOLVES[] += R
    if R > 0
        mppi.r.Control = permutedims(r.U[:, :, R, 1])
        mppi.r.Traj = permutedims(r.traj[:, :, R, 1])
        mppi.r.Feasibility = r.feasible[R, 1] == 1 ? :Feasible : :InFeasible
        mppi.r.cost = r.cost[R, 1]
        mppi.r.RolloutCount = r.rollout_count[R, 1]
    end
    return r.his[:, 1:r.n_rows[1], 1]
end

"""Order the context stream after the side stream's deferred final rollouts (MppiParams.final_stream = 1)."""
ctx_join() = (c = ctx(); check(ccall((:mp_ctx_join, libmpgpu), Cint, (Ptr{Cvoid},), c), c))

"""
    vehicle_euler!(states (7, n), ctrl (2, n), δt, nsteps; his = false) -> (states, his (7, nsteps, n) or nothing)

The closed-loop plant of MPPI/main.jl and DynamicWindow/main.jl:155-156 (`states .+= VehicleDynamics(states,
u)*δt`, u held) for n vehicles, in place.
"""
function vehicle_euler!(states::Matrix{Float64}, ctrl::Matrix{Float64}, δt::Float64, nsteps::Integer; his = false)
    n = size(states, 2); h = his ? zeros(7, nsteps, n) : nothing
    c = ctx()
    check(GC.@preserve states ctrl h ccall((:mp_vehicle_euler, libmpgpu), Cint,
        (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Float64, Int32, Ptr{Float64}),
        c, n, states, ctrl, δt, nsteps, h === nothing ? C_NULL : pointer(h)), c)
    return states, h
end

# ------------------------------------------------------ multi-GPU, one process
const GROUP = Ref{Vector{Ptr{Cvoid}}}(Ptr{Cvoid}[])

"""
    comm_init(devices = all) -> Vector{Ptr{Cvoid}}

One context per GPU of this node joined into one RCCL communicator (mp_comm_init: ncclCommInitAll,
xGMI between the MI355X GPUs), created once per process.  The Julia host stays a single process
(north_star); `mppi_plan_sharded` spreads the scenes over these contexts.
"""
function comm_init(devices = nothing)
    if isempty(GROUP[])
        nd = Ref{Cint}(0)
        st = ccall((:mp_device_count, libmpgpu), Cint, (Ref{Cint},), nd)
        st == MP_OK || error("libmpgpu: ", last_error(Ptr{Cvoid}(C_NULL)))
        devs = devices === nothing ? collect(0:nd[]-1) : collect(devices)
        cs = Ptr{Cvoid}[]
        for d in devs
            r = Ref{Ptr{Cvoid}}(C_NULL)
            st = ccall((:mp_ctx_create, libmpgpu), Cint, (Cint, Ref{Ptr{Cvoid}}), d, r)
            st == MP_OK || error("libmpgpu: ", last_error(Ptr{Cvoid}(C_NULL)))
            push!(cs, r[])
        end
        st = ccall((:mp_comm_init, libmpgpu), Cint, (Ptr{Ptr{Cvoid}}, Int32), cs, length(cs))
        st == MP_OK || error("libmpgpu: ", last_error(cs[1]))
        GROUP[] = cs
        atexit() do
            g = GROUP[]
            ccall((:mp_comm_destroy, libmpgpu), Cint, (Ptr{Ptr{Cvoid}}, Int32), g, length(g))
            foreach(c -> ccall((:mp_ctx_destroy, libmpgpu), Cint, (Ptr{Cvoid},), c), g)
            GROUP[] = Ptr{Cvoid}[]
        end
    end
    return GROUP[]
end

"""
    mppi_plan_sharded(p, X0 (7,S), goal (2,S), Unom (2,H,S); obstacles, grid, noise) -> NamedTuple

Multi-ego MPPIPlan over every GPU of `comm_init()` (mp_mppi_plan_sharded): scenes in balanced blocks per
GPU, then one RCCL all-gather of the optimal controls, final trajectories, costs and counts.  Same
results as `mppi_plan_batch` over all S scenes (the noise stream of a scene does not depend on the GPU
count).  Shapes as `mppi_plan_batch`; no TrajectoryCollection.
"""
function mppi_plan_sharded(p::MppiParams, X0::Matrix{Float64}, goal::Matrix{Float64}, Unom::Array{Float64,3};
                           obstacles = nothing, grid = nothing, noise = nothing)
    cs = comm_init()
    S = size(X0, 2); H = Int(p.H)
    p = noise === nothing ? p : MppiParams(ntuple(i -> i == 20 ? MP_NOISE_EXTERNAL : getfield(p, i), 26)...)
    U = zeros(2, H, S); traj = zeros(7, H + 1, S); cost = zeros(S)
    feas = zeros(Int32, S); rc = zeros(Int32, S); fc = zeros(Int32, S)
    nz(a) = a === nothing ? C_NULL : pointer(a)
    st = GC.@preserve cs X0 goal Unom obstacles grid noise U traj cost feas rc fc begin
        ccall((:mp_mppi_plan_sharded, libmpgpu), Cint,
              (Ptr{Ptr{Cvoid}}, Int32, Ref{MppiParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
               Ptr{Float64}, Ptr{UInt8}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32},
               Ptr{Int32}, Ptr{Int32}),
              cs, length(cs), p, S, X0, goal, Unom, nz(obstacles), nz(grid), nz(noise), U, traj, cost, feas, rc, fc)
    end
    st == MP_ERR_NUMERIC && @warn "MPPIPlan (sharded): NaN rollout cost (outputs written)"
    st == MP_ERR_NUMERIC || check(st, cs[1])
    return (; U, traj, cost, feasible = feas, rollout_count = rc, feasible_count = fc)
end

"""
    rollout_batch(p, X0 (7,S), goal (2,S), ctrl (2,H,K,S); Unom, obstacles) -> (traj, cost, feas, argmin)

Batched TrajectoryRollout (MPPIUtils.jl:31-57, DWAUtils.jl:16-42) with given controls.
"""
function rollout_batch(p::MppiParams, X0::Matrix{Float64}, goal::Matrix{Float64}, ctrl::Array{Float64,4};
                       Unom = nothing, obstacles = nothing)
    _, H, K, S = size(ctrl)
    traj = zeros(7, H + 1, K, S); cost = zeros(K, S); feas = zeros(UInt8, K, S); am = zeros(Int32, S)
    nz(a) = a === nothing ? C_NULL : pointer(a)
    c = ctx()
    st = GC.@preserve X0 goal ctrl Unom obstacles traj cost feas am ccall((:mp_rollout, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{MppiParams}, Int32, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64},
         Ptr{Float64}, Ptr{UInt8}, Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Ptr{Int32}),
        c, p, S, K, X0, goal, ctrl, 2, nz(Unom), nz(obstacles), C_NULL, traj, cost, feas, am)
    check(st, c)
    return traj, cost, feas, am .+ 1     # 1-based argmin
end

# ---------------------------------------------------------------- Hybrid A*
struct HaParams
    vehicle_len::Float64
    vehicle_wid::Float64
    minR::Float64
    expand_time::Float64
    res::NTuple{3,Float64}
    stbound::NTuple{6,Float64}
    n_walls::Int32
    n_prim::Int32
    n_col::Int32
    max_pops::Int32
end

function ha_params(ha; max_pops = 5000)
    s = ha.s
    sb = s.stbound                       # 3×2 [min max] per state (setup.jl:27-33)
    HaParams(s.vehicle_size[1], s.vehicle_size[2], s.minR, s.expand_time, Tuple(s.resolutions),
             (sb[1, 1], sb[1, 2], sb[2, 1], sb[2, 2], sb[3, 1], sb[3, 2]), length(s.obstacle_list),
             s.num_neighbors, size(s.paths_candi, 2), max_pops)
end

"""neighbor_origin (hybrid_astar_utils.jl:483-503) computed on the device and installed in the context:
(states_candi 3×n, paths_candi 3×n_col×n), n = length(gear_set)·length(steer_set)."""
function ha_neighbor_origin(p::HaParams, steer_set::Vector{Float64}, gear_set::Vector{Float64})
    n = length(steer_set) * length(gear_set)
    sc = zeros(3, n); pc = zeros(3, Int(p.n_col), n)
    c = ctx()
    check(GC.@preserve steer_set gear_set sc pc ccall((:mp_ha_neighbor_origin, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{HaParams}, Int32, Ptr{Float64}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        c, p, length(steer_set), steer_set, length(gear_set), gear_set, sc, pc), c)
    return sc, pc
end

"""Install the searcher's own neighbor_origin table (states_candi 3×n, paths_candi 3×n_col×n):
the device transforms Julia-computed bits (SURVEY §8c)."""
function ha_install!(ha, p::HaParams)
    sc = Matrix{Float64}(ha.s.states_candi); pc = Array{Float64,3}(ha.s.paths_candi)
    c = ctx()
    check(GC.@preserve sc pc ccall((:mp_ha_set_primitives, libmpgpu), Cint,
                                   (Ptr{Cvoid}, Ref{HaParams}, Ptr{Float64}, Ptr{Float64}), c, p, sc, pc), c)
end

walls_of(ha) = reshape(reduce(hcat, ha.s.obstacle_list), 5, :)

"""
    planHybridAstar!(ha)

Drop-in for hybrid_astar_utils.jl:235-296 (one scenario; `plan_batch!` for many).  Fills
`ha.r.hybrid_astar_states` (3×n, goal-side first, as the reference's hcat loop),
`ha.r.RSpath_final` (3×len), `ha.p.loop_count` and `ha.r.planning_time`, then calls the
reference's own `retrievePath(ha)` when a path was found.
"""
planHybridAstar!(ha; retrieve = nothing) = (plan_batch!([ha]; retrieve = retrieve); nothing)

function plan_batch!(has::AbstractVector; retrieve = nothing, max_pops = 5000)
    t1 = time()
    h0 = has[1]
    p = ha_params(h0; max_pops = max_pops)
    ha_install!(h0, p)
    B = length(has)
    start = reduce(hcat, [h.s.starting_states for h in has]); goal = reduce(hcat, [h.s.ending_states for h in has])
    walls = reshape(reduce(hcat, [walls_of(h) for h in has]), 5, Int(p.n_walls), B)
    found = zeros(Int32, B); pops = zeros(Int32, B); nn = zeros(Int32, B)
    seq = fill(Int64(-1), max_pops, B); ns = zeros(Int32, B); states = zeros(3, max_pops, B)
    rl = zeros(Int32, B); rs = zeros(3, 501, B)
    c = ctx()
    st = GC.@preserve start goal walls found pops nn seq ns states rl rs ccall((:mp_ha_plan, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{HaParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32},
         Ptr{Int32}, Ptr{Int64}, Ptr{Int32}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}),
        c, p, B, start, goal, walls, found, pops, nn, seq, ns, states, rl, rs)
    check(st, c)
    dt = time() - t1
    for (b, h) in enumerate(has)
        h.p.loop_count = pops[b]
        h.r.planning_time = dt
        if found[b] == 1
            h.r.hybrid_astar_states = states[:, 1:ns[b], b]
            h.r.RSpath_final = rs[:, 1:rl[b], b]
            retrieve === nothing || retrieve(h)     # e.g. Main.retrievePath
        end
    end
    return (; found, pops, n_nodes = nn, pop_sequence = seq)
end

"""Batched FindNewNode device part for B popped nodes (3, B): neighbour states (3, n, B),
Encode indices (n, B) (0 = out of bounds), collision-free flags (n, B), rs heuristics (n, B)."""
"""
    retrieve_batch!(has)

retrievePath (hybrid_astar_utils.jl:129-177, with cubic_fit :100-127) for planned searchers in one launch
(mp_ha_retrieve_path): sets `r.actualpath` (3 × L), `r.tol_length` and `r.x_interp`, `r.y_interp`,
`r.ψ_interp` = `linear_interpolation(LinRange(0, tol_length, 50), samples)` as the reference builds them.
Pass it as `plan_batch!(has; retrieve = nothing)` then call this once for the whole batch (the
reference's own `retrievePath` per searcher stays available through `retrieve = retrievePath`).
"""
const SAMPLES = WeakKeyDict{Any,Matrix{Float64}}()

function retrieve_batch!(has::AbstractVector)
    B = length(has)
    ok(h) = h.r.hybrid_astar_states !== nothing && size(h.r.hybrid_astar_states, 2) > 0
    ns = Int32[ok(h) ? size(h.r.hybrid_astar_states, 2) : 0 for h in has]
    stride = max(1, maximum(ns))
    start = reduce(hcat, [Float64.(h.s.starting_states) for h in has])
    states = zeros(3, stride, B); rl = zeros(Int32, B); rs = zeros(3, 501, B)
    for (b, h) in enumerate(has)
        ns[b] == 0 && continue
        states[:, 1:ns[b], b] = h.r.hybrid_astar_states
        rl[b] = size(h.r.RSpath_final, 2)
        rs[:, 1:rl[b], b] = h.r.RSpath_final
    end
    tot = sum(n == 0 ? 0 : 1 + 100 * (n - 1) + r for (n, r) in zip(ns, rl))
    off = zeros(Int64, B + 1); pts = zeros(3, max(tot, 1)); plen = zeros(max(tot, 1))
    np_ = zeros(Int32, B); tol = zeros(B); smp = zeros(3, 50, B)
    c = ctx()
    check(GC.@preserve start ns states rl rs off pts plen np_ tol smp ccall((:mp_ha_retrieve_path, libmpgpu), Cint,
        (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Int32, Ptr{Int32}, Ptr{Float64}, Ptr{Int64},
         Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}),
        c, B, start, ns, states, stride, rl, rs, off, pts, plen, np_, tol, smp), c)
    for (b, h) in enumerate(has)
        ns[b] == 0 && continue
        SAMPLES[h] = smp[:, :, b]     # the knot values, for track_batch!
        h.r.actualpath = pts[:, off[b]+1:off[b+1]]
        h.r.tol_length = tol[b]
        knots = LinRange(0, tol[b], 50)
        h.r.x_interp = linear_interpolation(knots, smp[1, :, b])
        h.r.y_interp = linear_interpolation(knots, smp[2, :, b])
        h.r.ψ_interp = linear_interpolation(knots, smp[3, :, b])
    end
    return has
end

struct TrackParams     # mp_track_params (main_Tracker.jl:42-72)
    n_ref::Int32
    max_steps::Int32
    dt_sim::Float64
    look_ahead::Float64
    p_gain::Float64
    i_gain::Float64
    veh_len::Float64
    max_sa::Float64
    his_stride::Int32
    reserved::Int32
end

"""
    track_batch!(has; look_ahead_dist = 1.0, p_gain = 10, i_gain = 0.1, dt_sim = 1e-3, max_sa = max_δf + 0.1, ...)

The tracker of PathPlanning/HybridAstar/main_Tracker.jl:42-137 for every planned + retrieved searcher
(`retrieve_batch!` first) in one launch (mp_ha_track, one wavefront per searcher): the hand-off
x/y/ψ_ref = x/y/ψ_interp(LinRange(0, tol_length, 1000)), then findclosest / inverseKinematic /
look-ahead PI / kinematic Euler steps of 1 ms from `starting_real` until the closest reference point
is the last one.  Returns, per searcher, `(; status, n_steps, states_his (3 × rows, every his_stride-th
update), cur_states, err_accumulated, x_ref, y_ref, ψ_ref)`; `status` is :done, :max_steps, :no_path or
:empty_window.  (The reference's plotting/gif of the loop is not reproduced.)
"""
function track_batch!(has::AbstractVector; look_ahead_dist = 1.0, p_gain = 10, i_gain = 0.1, dt_sim = 1e-3,
                      max_sa = pi / 6 + 0.1, n_ref = 1000, max_steps = 200_000, his_stride = 1, his_cap = 30_000)
    B = length(has)
    start = reduce(hcat, [Float64.(h.s.starting_real) for h in has])
    tol = [haskey(SAMPLES, h) ? Float64(h.r.tol_length) : 0.0 for h in has]
    smp = zeros(3, 50, B)
    for (b, h) in enumerate(has)
        haskey(SAMPLES, h) && (smp[:, :, b] = SAMPLES[h])
    end
    vl = unique(Float64(h.s.vehicle_size[1]) for h in has)   # veh_param[1] per searcher (main_Tracker.jl:50)
    if length(vl) > 1        # one launch per vehicle length, results in the caller's order
        out = Vector{Any}(undef, B)
        for L in vl
            ix = findall(h -> Float64(h.s.vehicle_size[1]) == L, has)
            out[ix] = track_batch!(has[ix]; look_ahead_dist, p_gain, i_gain, dt_sim, max_sa, n_ref, max_steps,
                                   his_stride, his_cap)
        end
        return out
    end
    p = TrackParams(n_ref, max_steps, dt_sim, look_ahead_dist, p_gain, i_gain, vl[1], max_sa, his_stride, 0)
    n = zeros(Int32, B); st = zeros(Int32, B); fin = zeros(3, B); ea = zeros(B)
    ref = zeros(3, n_ref, B); his = zeros(3, his_cap, B)
    c = ctx()
    check(GC.@preserve start tol smp n st fin ea ref his ccall((:mp_ha_track, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{TrackParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int32, Ptr{Int32}, Ptr{Int32},
         Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int32),
        c, p, B, start, tol, smp, 50, n, st, fin, ea, ref, his, his_cap), c)
    names = (:done, :max_steps, :no_path, :empty_window)
    return [(; status = names[st[b] + 1], n_steps = Int(n[b]),
              states_his = his[:, 1:(n[b] == 0 ? 1 : min(his_cap, (n[b] - 1) ÷ his_stride + 1)), b],
              cur_states = fin[:, b], err_accumulated = ea[b],
              x_ref = ref[1, :, b], y_ref = ref[2, :, b], ψ_ref = ref[3, :, b]) for b in 1:B]
end

function ha_expand(p::HaParams, node::Matrix{Float64}, goal::Matrix{Float64}, walls::Array{Float64,3})
    B = size(node, 2); n = Int(p.n_prim)
    nb = zeros(3, n, B); idx = zeros(Int64, n, B); fr = zeros(UInt8, n, B); h = zeros(n, B)
    c = ctx()
    check(GC.@preserve node goal walls nb idx fr h ccall((:mp_ha_expand, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{HaParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int64},
         Ptr{UInt8}, Ptr{Float64}), c, p, B, node, goal, walls, nb, idx, fr, h), c)
    return nb, idx, fr, h
end

"""Batched RS_connected: (ok (B,), paths (3, 501, B), lengths (B,))."""
function ha_rs_connect(p::HaParams, node::Matrix{Float64}, goal::Matrix{Float64}, walls::Array{Float64,3})
    B = size(node, 2)
    ok = zeros(UInt8, B); path = zeros(3, 501, B); len = zeros(Int32, B)
    c = ctx()
    check(GC.@preserve node goal walls ok path len ccall((:mp_ha_rs_connect, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{HaParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Ptr{Float64},
         Ptr{Int32}), c, p, B, node, goal, walls, ok, path, len), c)
    return ok, path, len
end

"""Whether the library's collision sweeps use their SAT culls for these inputs (coordinates <= 1e6 m)."""
function ha_sat_cull_active(p::HaParams, walls::Array{Float64,3}, a::Matrix{Float64}, b::Matrix{Float64})
    B = size(a, 2); on = Ref{Int32}(0)
    c = ctx()
    check(GC.@preserve walls a b ccall((:mp_ha_sat_cull_active, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{HaParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{Int32}),
        c, p, B, walls, a, b, on), c)
    return on[] == 1
end

"""allpath (ReedsSheppsUtils.jl:468-511) for normalised states (3, B): best (1-based), cost (48, B),
cmds (3, 5, 48, B) (rows [distance, gear, steer] of each command)."""
function ha_allpath(ns::Matrix{Float64})
    B = size(ns, 2)
    cost = zeros(48, B); cmds = zeros(3, 5, 48, B); best = zeros(Int32, B)
    c = ctx()
    check(GC.@preserve ns cost cmds best ccall((:mp_ha_allpath, libmpgpu), Cint,
        (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}), c, B, ns, cost, cmds, best), c)
    return best .+ 1, cost, cmds
end

# --------------------------------------------------------------------- iLQR
struct IlqrParams
    N::Int32
    variant::Int32        # 0 OptimalControl/ILQR/Cost.jl, 1 PathPlanning/Parking_ILQR/Cost.jl
    dT::Float64
    eps::Float64
    alpha_floor::Float64
    tol::Float64
    max_iter::Int32
    max_ls::Int32
end
IlqrParams(N; variant = 0, dT = 0.05, eps = 1e-3, tol = 1e-6, max_iter = 1000, max_ls = 200) =
    IlqrParams(N, variant, dT, eps, variant == 1 ? 1e-3 : 0.0, tol, max_iter, max_ls)

"""Initial-guess roll out (ILQR.jl:31-37) + TotalCost (Cost.jl:1-8): x0 (4, B), U (2, N, B) -> (X (4, N, B), J (B,))."""
function ilqr_rollout(p::IlqrParams, x0::Matrix{Float64}, U::Array{Float64,3})
    B = size(x0, 2); X = zeros(4, Int(p.N), B); J = zeros(B); c = ctx()
    check(GC.@preserve x0 U X J ccall((:mp_ilqr_rollout, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{IlqrParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        c, p, B, x0, U, X, J), c)
    return X, J
end

"""One backward Riccati sweep (ILQR.jl:46-67) for B instances: X (4, N, B), U (2, N, B)
-> k (2, N-1, B), K (2, 4, N-1, B) (the reference's klist / Klist per instance)."""
function ilqr_backward!(k, K, p::IlqrParams, X, U)
    B = size(X, 3); c = ctx()
    check(GC.@preserve X U k K ccall((:mp_ilqr_backward, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{IlqrParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        c, p, B, X, U, k, K), c)
    return k, K
end

"""One forward trial at step sizes α (B,) (ILQR.jl:72-80) -> (Xnew, Unew, Jnew)."""
function ilqr_forward!(Xn, Un, Jn, p::IlqrParams, X, U, k, K, α)
    B = size(X, 3); c = ctx()
    check(GC.@preserve X U k K α Xn Un Jn ccall((:mp_ilqr_forward, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{IlqrParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
         Ptr{Float64}, Ptr{Float64}, Ptr{Float64}), c, p, B, X, U, k, K, α, Xn, Un, Jn), c)
    return Xn, Un, Jn
end

"""The whole ILQR.jl:39-88 loop per instance, in place on X (4, N, B), U (2, N, B)."""
function ilqr_solve!(X, U, p::IlqrParams)
    B = size(X, 3); J = zeros(B); it = zeros(Int32, B); c = ctx()
    st = GC.@preserve X U J it ccall((:mp_ilqr_solve, libmpgpu), Cint,
        (Ptr{Cvoid}, Ref{IlqrParams}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
        c, p, B, X, U, J, it)
    st == MP_ERR_NUMERIC && @warn "iLQR: some instances hit max_iter / max_ls (results written)"
    st == MP_ERR_NUMERIC || check(st, c)
    return J, it
end

end # module
