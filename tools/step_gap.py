"""Per-step wall time of the bench headline loop (bench.run: 8 configs[4] scenes per step) with the
kernel-timing events on and off, to size the per-step overhead outside mppi_plan_kernel."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from motionplanning_amd.context import Context  # noqa: E402

ctx = Context(0)
dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.ExternalStream(ctx.stream, device=dev))
a = argparse.Namespace(final_inline=False)
for steps in (50, 200):
    for timing in (1, 0, 1):
        ctx.lib.mp_ctx_kernel_timing(ctx.handle, timing)
        el, kms, ok, K, H, fc, _ = bench.run(a, 8, ctx, dev, 1, 0, steps, 5, 3)
        print(f"steps {steps} timing {timing}: {el / steps * 1e3:.4f} ms/step, kernel {kms:.4f} ms, ok {ok}", flush=True)
