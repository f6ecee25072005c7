"""Diagnostic: phase timings of mp_mppi_plan at cfg2 (run with MPGPU_STAMPS=1)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from motionplanning_amd import configs
from motionplanning_amd.abi import MP_NOISE_PHILOX
from motionplanning_amd.mppi import mppi_plan_batch
for S in (1, 8):
    c = configs.cfg2(noise_mode=MP_NOISE_PHILOX)
    p = c["params"]
    for i in range(3):
        mppi_plan_batch(p, np.tile(c["X0"], (S, 1)), np.tile(c["goal"], (S, 1)), np.zeros((S, p.H, 2)), None,
                        np.tile(c["grid"], (S, 1, 1)), None, collect=(i == 2))
