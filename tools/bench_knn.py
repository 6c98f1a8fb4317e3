"""Times the float-descriptor k-NN matcher (SIFT/SURF modes) through the C-ABI
at SIFT-sized workloads; run under rocprofv3 --kernel-trace --stats for the
per-kernel durations (DESIGN.md row f, rank 4)."""
import sys
import time

import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from droplet_visual_odometry_amd import ops
from droplet_visual_odometry_amd._native import Context

ctx = Context.default(0)
rng = np.random.default_rng(0)
for n, dim, norm in [(2000, 128, 0), (5000, 128, 0), (5000, 64, 0), (5000, 128, 1)]:
    dq = rng.integers(0, 256, (n, dim)).astype(np.float32)
    dt = rng.integers(0, 256, (n, dim)).astype(np.float32)
    ops.bf_knn_float(dq, dt, 2, norm, ctx=ctx)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        ops.bf_knn_float(dq, dt, 2, norm, ctx=ctx)
    dt_ms = (time.perf_counter() - t0) / reps * 1e3
    print(f"n={n} dim={dim} norm={norm}: {dt_ms:.3f} ms/call incl. H2D/D2H, "
          f"{n * n / dt_ms / 1e6:.2f} G distance pairs/s", flush=True)
sys.exit(0)
