"""Generate tests/golden/obstacle_fields_64.npz: the obstacle sets of BASELINE.json configs[4]
("Multi-ego MPPI: 64 independent scenes", BASELINE.md cfg5: "scenes vary X0 and the obstacle set
(PathPlanning/Scenarios/obstacle_field.mat fields 1-64, rescaled)").

Run in the build container (needs /root/reference, read-only; data only, no reference code runs):

    python tests/golden/make_obstacle_fields.py

Input: PathPlanning/Scenarios/obstacle_field.mat, variable `obstacle_field` (100×1 cell of n×3 [x, y, R]
circles over the 120 m × 120 m field of PathPlanning/Astar/main.jl:14-17, read there with
`obsinfo[Trial_num]`; read here with scipy.io.loadmat, which executes nothing from the file).

Rescaling into the MPPI corridor (x ∈ [-10, 130], y ∈ [-20, 20] of OptimalControl/MPPI/main.jl:8-9,
start x = 0, goal x = 110): centres x' = 10 + x·(100/120) (the field spans the stretch between start
and goal), y' = (y − 60)·(40/120), radius R' = R·(40/120) (the tighter axis factor, so a circle stays a
circle inside the corridor).  Output arrays:
  circles[64][max_n][3] (rows past count[f] are zero), count[64] — field f+1 of the .mat (1-based as Julia)
  sha256 — of the source .mat
"""
import hashlib
import os

import numpy as np

REF = "/root/reference/PathPlanning/Scenarios/obstacle_field.mat"
HERE = os.path.dirname(os.path.abspath(__file__))
N_FIELDS = 64


def rescale(c):
    c = np.asarray(c, np.float64).reshape(-1, 3)
    out = np.empty_like(c)
    out[:, 0] = 10.0 + c[:, 0] * (100.0 / 120.0)
    out[:, 1] = (c[:, 1] - 60.0) * (40.0 / 120.0)
    out[:, 2] = c[:, 2] * (40.0 / 120.0)
    return out


def main():
    import scipy.io

    raw = open(REF, "rb").read()
    cells = scipy.io.loadmat(REF)["obstacle_field"]
    fields = [rescale(cells.flat[f]) for f in range(N_FIELDS)]
    n = max(len(f) for f in fields)
    circles = np.zeros((N_FIELDS, n, 3))
    count = np.zeros(N_FIELDS, np.int32)
    for i, f in enumerate(fields):
        circles[i, :len(f)] = f
        count[i] = len(f)
    np.savez_compressed(os.path.join(HERE, "obstacle_fields_64.npz"), circles=circles, count=count,
                        sha256=np.array(hashlib.sha256(raw).hexdigest()))
    print(f"wrote {N_FIELDS} fields, {count.min()}..{count.max()} circles each")


if __name__ == "__main__":
    main()
