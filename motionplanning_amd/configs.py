"""Reference settings and the BASELINE.json workload configurations.

Every constant cites where the reference sets it.  These are plain data used by
the host-side planner mirror (mppi.py / dwa.py / ilqr.py / hybrid_astar.py),
the tests and bench.py.
"""
import math
import os

import numpy as np

from .abi import MP_NOISE_EXTERNAL, MPPIParams

# OptimalControl/MPPI/main.jl:7-11 (identical bounds in DynamicWindow/main.jl:7-9)
X0_REF = [0.0, 0.0, 0.0, 0.0, 0.0, 5.0, 0.0]
XL_REF = [-10.0, -20.0, -2.0, -math.pi / 2, -math.pi / 2, 1.0, -math.pi / 9]
XU_REF = [130.0, 20.0, 2.0, math.pi / 2, math.pi / 2, 10.0, math.pi / 9]
CL_MPPI = [-0.5, -2.5]
CU_MPPI = [0.5, 2.5]
GOAL_REF = [110.0, 0.0]  # MPPI/main.jl:23
SIGMA_REF = [0.05, 0.0, 0.0, 0.1]  # MPPI/main.jl:27
LAMBDA_REF = 25.0  # MPPI/main.jl:24
OBSTACLES_REF = [[50.0, 1.0, 2.5], [70.0, -1.0, 2.5], [90.0, 1.0, 2.5]]  # MPPI/main.jl:30
# the reference's three circles plus two
OBSTACLES_CFG1 = [[30.0, -1.0, 2.5], [50.0, 1.0, 2.5], [70.0, -1.0, 2.5], [90.0, 1.0, 2.5], [100.0, -1.0, 2.5]]
MPPI_OBS_PENALTY = 100.0 * 712.5  # MPPIUtils.jl:127
DWA_OBS_PENALTY = 10000.0 * 712.5  # DWAUtils.jl:112
SLACK_PENALTY = 1e5  # MPPI/src/types.jl:30
FEASIBILITY_COUNT_REF = 1300  # MPPI/src/types.jl:24

# DynamicWindow/main.jl:10-11, 26; setup.jl:59-85
CL_DWA = [-0.3, -2.5]
CU_DWA = [0.3, 2.5]
DWA_SAMPLES = [31, 41]
DWA_N = 20  # DWASetting default N (DynamicWindow/src/types.jl:20)


def julia_linrange(a, b, n):
    """Julia `LinRange(a, b, n)` elements: (1-t)*a + t*b, t = (i-1)/(n-1) (base/range.jl lerpi)."""
    out = np.empty(n)
    for i in range(n):
        t = i / (n - 1)
        out[i] = (1 - t) * a + t * b
    return out


# MPPI closed loop, OptimalControl/MPPI/main.jl:17-19,55,77
UPDATE_TIME_REF = 0.1
PLANT_DT_REF = 1e-3
SIM_TIME_REF = 15.0
GOAL_RADIUS_MPPI = 6.0


def julia_range(a, b, n):
    """collect(range(a, b, length=n)) for Float64 endpoints: Julia's StepRangeLen evaluates each
    element in TwicePrecision, i.e. the correctly rounded a + (i-1)(b-a)/(n-1) (exact rationals here)."""
    from fractions import Fraction

    if n == 1:
        return np.array([float(a)])
    fa, fb = Fraction(float(a)), Fraction(float(b))
    return np.array([float(fa + (fb - fa) * i / (n - 1)) for i in range(n)])


def mppi_hold_index(T, N, update_time=UPDATE_TIME_REF, plant_dt=PLANT_DT_REF):
    """The zero-order hold of MPPI/main.jl:51-52,64-66: update_idx = Int32(floor(update_time/δt)) plant
    steps per replan, and step i of a period applies row j of NominalControls where
    interpolate((time_serial,), ·, Gridded(Constant{Previous}())) picks the last knot
    time_serial[j] <= fined_time_serial[i].  Returns (update_idx, 0-based rows [update_idx])."""
    update_idx = int(math.floor(update_time / plant_dt))
    ts = julia_range(0.0, T, N)
    fs = julia_range(0.0, update_time, update_idx)
    hold = np.array([int(np.searchsorted(ts, t, side="right")) - 1 for t in fs], np.int32)
    if hold.min() < 0:
        raise ValueError("fined_time_serial starts before time_serial")
    return update_idx, hold


def dwa_control_samples(CL=CL_DWA, CU=CU_DWA, counts=DWA_SAMPLES):
    """defineDWAcontrols! (DynamicWindow/src/setup.jl:59-94): sr-major, ax-minor grid."""
    v1 = julia_linrange(CL[0], CU[0], counts[0])
    v2 = julia_linrange(CL[1], CU[1], counts[1])
    out = np.empty((counts[0] * counts[1], 2))
    for i in range(counts[0] * counts[1]):
        out[i, 0] = v1[i // counts[1]]
        out[i, 1] = v2[i % counts[1]]
    return out


def mppi_params(K=1500, H=20, T=3.0, lam=LAMBDA_REF, sigma=SIGMA_REF, XL=XL_REF, XU=XU_REF, CL=CL_MPPI,
                CU=CU_MPPI, n_obs=3, feasibility_count=FEASIBILITY_COUNT_REF, obs_penalty=MPPI_OBS_PENALTY,
                grid=None, noise_mode=MP_NOISE_EXTERNAL, ctrl_cost=1, seed=0, offset=0, dt=None):
    """mp_mppi_params from defineMPPI arguments (MPPI/src/setup.jl:3-59); defaults = MPPI/main.jl."""
    p = MPPIParams()
    p.K, p.H = K, H
    p.feasibility_count = feasibility_count
    p.n_obs = n_obs
    p.dt = (T / H) if dt is None else dt
    p.lambda_ = lam
    for i in range(4):
        p.sigma[i] = sigma[i]
    for i in range(7):
        p.XL[i], p.XU[i] = XL[i], XU[i]
    for i in range(2):
        p.CL[i], p.CU[i] = CL[i], CU[i]
    p.slack_penalty = SLACK_PENALTY
    p.obs_penalty = obs_penalty
    if grid is not None:
        p.grid_nx, p.grid_ny = grid["nx"], grid["ny"]
        p.grid_x0, p.grid_y0, p.grid_dx, p.grid_dy = grid["x0"], grid["y0"], grid["dx"], grid["dy"]
    p.noise_mode = noise_mode
    p.ctrl_cost = ctrl_cost
    p.seed = seed
    p.offset = offset
    return p


def dwa_params():
    """DWA settings (DynamicWindow/main.jl:7-26): N=20, dt=T/N=0.15, obstacle penalty 7.125e6, no control cost."""
    return mppi_params(K=DWA_SAMPLES[0] * DWA_SAMPLES[1], H=DWA_N, T=3.0, CL=CL_DWA, CU=CU_DWA, n_obs=3,
                       obs_penalty=DWA_OBS_PENALTY, ctrl_cost=0)


# ------------------------------------------------------------- occupancy grid
GRID_NX, GRID_NY = 100, 100  # GridNum (MPPI/main.jl:25; unused by the reference)


def grid_spec(XL=XL_REF, XU=XU_REF, nx=GRID_NX, ny=GRID_NY):
    """Cells over x in [XL1, XU1], y in [XL2, XU2]: 1.4 m x 0.4 m."""
    return dict(nx=nx, ny=ny, x0=XL[0], y0=XL[1], dx=(XU[0] - XL[0]) / nx, dy=(XU[1] - XL[1]) / ny)


def rasterize_circles(circles, spec):
    """uint8 [ny][nx] grid; a cell is occupied when its centre lies in a circle (build extension)."""
    g = np.zeros((spec["ny"], spec["nx"]), np.uint8)
    xc = spec["x0"] + (np.arange(spec["nx"]) + 0.5) * spec["dx"]
    yc = spec["y0"] + (np.arange(spec["ny"]) + 0.5) * spec["dy"]
    X, Y = np.meshgrid(xc, yc)
    for cx, cy, r in circles:
        g |= ((X - cx) ** 2 + (Y - cy) ** 2 <= r * r).astype(np.uint8)
    return g


def cfg1():
    """BASELINE.json configs[0]: K=128, H=30, 5 circles, CPU plumbing."""
    p = mppi_params(K=128, H=30, T=4.5, n_obs=5)
    return dict(params=p, X0=np.array(X0_REF), goal=np.array(GOAL_REF), obstacles=np.array(OBSTACLES_CFG1),
                grid=None, unom=np.zeros((30, 2)))


def cfg2(feasibility_count=None, noise_mode=MP_NOISE_EXTERNAL, seed=20260415, with_circles=False):
    """BASELINE.json configs[1]: K=8192, H=50, 2-D occupancy grid."""
    spec = grid_spec()
    grid = rasterize_circles(OBSTACLES_CFG1, spec)
    K, H = 8192, 50
    p = mppi_params(K=K, H=H, T=H * 0.15, n_obs=5 if with_circles else 0,
                    feasibility_count=K if feasibility_count is None else feasibility_count, grid=spec,
                    noise_mode=noise_mode, seed=seed)
    return dict(params=p, X0=np.array(X0_REF), goal=np.array(GOAL_REF),
                obstacles=np.array(OBSTACLES_CFG1) if with_circles else None, grid=grid, unom=np.zeros((H, 2)))


def standard_noise(K, H, seed=20260415):
    """z ~ N(0,1), numpy PCG64(seed), shape (K, H, 2)."""
    return np.random.Generator(np.random.PCG64(seed)).standard_normal((K, H, 2))


# ------------------------------------------------- configs[4]: 64 multi-ego scenes
FIELDS_NPZ = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                          "obstacle_fields_64.npz")
N_SCENES_CFG5 = 64


def obstacle_field(g):
    """Circles [n][3] of scene g (0-based): PathPlanning/Scenarios/obstacle_field.mat field g+1 (Julia
    index), rescaled into the corridor by tests/golden/make_obstacle_fields.py."""
    d = np.load(FIELDS_NPZ)
    f = g % N_SCENES_CFG5
    return d["circles"][f, :int(d["count"][f])]


def cfg5_x0(g):
    """X0 of scene g: the reference start (MPPI/main.jl:7) with the lateral offset y = -0.5 + (g mod 8)/7."""
    x = np.array(X0_REF)
    x[1] = -0.5 + (g % 8) / 7.0
    return x


def cfg5_shard(scene_base, S, noise_mode=MP_NOISE_EXTERNAL, seed=20260415):
    """BASELINE.json configs[4] ("64 independent scenes x K=8192 x H=50"): scenes [scene_base, scene_base+S),
    each configs[1] (K=8192, H=50, 100x100 occupancy grid) with its own X0 (cfg5_x0) and its own grid,
    rasterised from obstacle_field.mat field g+1.  params.scene_base = scene_base (Philox counter word)."""
    c = cfg2(noise_mode=noise_mode, seed=seed)
    p = c["params"]
    p.scene_base = scene_base
    spec = grid_spec()
    gs = list(range(scene_base, scene_base + S))
    X0 = np.stack([cfg5_x0(g) for g in gs])
    grids = np.stack([rasterize_circles(obstacle_field(g), spec) for g in gs])
    return dict(params=p, X0=X0, goal=np.tile(GOAL_REF, (S, 1)), grid=grids, unom=np.zeros((S, p.H, 2)),
                fields=[g % N_SCENES_CFG5 + 1 for g in gs])
