"""Generate the committed golden fixtures from the reference's own artifacts.

Run in the build container (needs /root/reference, read-only):

    python tests/golden/make_golden.py

Inputs (reference-produced outputs, data only — no reference code is run):
  - OptimalControl/DynamicWindow/DWATrajectory.csv  12,633 rows [t, x, y, v, r, ψ, ux, sa]
    written by the DWA closed loop (DynamicWindow/main.jl:139-167; deterministic).
  - OptimalControl/MPPI/MPPITrajectory.csv          11,929 rows, same columns
    (MPPI/main.jl:238-270; the MPPI noise was unseeded, so only the plant is pinned).

Outputs (tests/golden/*.npz):
  dwa_closed_loop.npz  rows every 10th step + every replan row + last row, their
                       step indices, the 127 replan states, the grid index (1-based
                       i_sr, i_ax) chosen at each replan recovered by differencing,
                       and the sha256 of the source CSV.
  mppi_plant.npz       the same subsampling of MPPITrajectory.csv plus the per-block
                       controls (sr, ax) recovered by differencing.
"""
import hashlib
import os

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
DT = 1e-3
UPDATE = 100


def _load(rel):
    path = os.path.join(REF, rel)
    raw = open(path, "rb").read()
    arr = np.loadtxt(path, delimiter=",")
    return arr, hashlib.sha256(raw).hexdigest()


def _subsample(arr):
    n = arr.shape[0]
    keep = set(range(0, n, 10)) | set(range(0, n, UPDATE)) | {n - 1}
    idx = np.array(sorted(keep), dtype=np.int64)
    return idx, arr[idx]


def _block_controls(arr):
    """(sr, ax) applied during each 100-step block: dsa = sr, dux = ax (vehicledynamics.jl:48-49)."""
    nblk = (arr.shape[0] - 1 + UPDATE - 1) // UPDATE
    out = np.zeros((nblk, 2))
    for b in range(nblk):
        r0 = b * UPDATE
        out[b, 0] = (arr[r0 + 1, 7] - arr[r0, 7]) / DT
        out[b, 1] = (arr[r0 + 1, 6] - arr[r0, 6]) / DT
    return out


def dwa():
    arr, sha = _load("OptimalControl/DynamicWindow/DWATrajectory.csv")
    ctrl = _block_controls(arr)
    # DWA grid: LinRange(CL, CU, n) with Julia's lerpi formula (DynamicWindow/main.jl:10-11, setup.jl:66)
    def linrange(a, b, n):
        t = np.arange(n) / (n - 1)
        return (1 - t) * a + t * b
    sr_grid = linrange(-0.3, 0.3, 31)
    ax_grid = linrange(-2.5, 2.5, 41)
    i_sr = np.array([int(np.argmin(np.abs(sr_grid - c))) + 1 for c in ctrl[:, 0]])
    i_ax = np.array([int(np.argmin(np.abs(ax_grid - c))) + 1 for c in ctrl[:, 1]])
    err = max(np.abs(sr_grid[i_sr - 1] - ctrl[:, 0]).max(), np.abs(ax_grid[i_ax - 1] - ctrl[:, 1]).max())
    assert err < 1e-9, err
    idx, rows = _subsample(arr)
    replan_rows = arr[0 : arr.shape[0] : UPDATE][: len(ctrl)]
    np.savez_compressed(
        os.path.join(HERE, "dwa_closed_loop.npz"),
        step_index=idx, rows=rows, replan_states=replan_rows[:, 1:],
        i_sr=i_sr, i_ax=i_ax, n_rows=np.int64(arr.shape[0]), sha256=np.bytes_(sha),
        final_row=arr[-1],
    )
    print("dwa:", arr.shape, "replans", len(ctrl), "first choice", i_sr[0], i_ax[0])


def mppi():
    arr, sha = _load("OptimalControl/MPPI/MPPITrajectory.csv")
    ctrl = _block_controls(arr)
    idx, rows = _subsample(arr)
    replan_rows = arr[0 : arr.shape[0] : UPDATE][: len(ctrl)]
    np.savez_compressed(
        os.path.join(HERE, "mppi_plant.npz"),
        step_index=idx, rows=rows, replan_states=replan_rows[:, 1:], block_ctrl=ctrl,
        n_rows=np.int64(arr.shape[0]), sha256=np.bytes_(sha), final_row=arr[-1],
    )
    print("mppi:", arr.shape, "replans", len(ctrl))


if __name__ == "__main__":
    dwa()
    mppi()
