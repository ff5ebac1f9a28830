"""Per-call cost of one small FM3D host-entry solve (ctx.tmap3d on a 60 x 60 x 41 volume, the
end-effector size): wall time per call and the device solve time from the context's stats.
Run under rocprofv3 --kernel-trace and read the timeline with tools/trace_gaps.py.
  python tools/fm3d_single_probe.py [calls]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "planning-motion_planning_amd"))
import eikonal  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rng = np.random.default_rng(1)
c = rng.uniform(1, 3, (60, 60, 41))
c[rng.random(c.shape) < 0.1] = np.inf
c[:, :, 0] = c[:, :, -1] = np.inf
goal = [40, 30, 20]
c[goal[1], goal[0], goal[2]] = 1.0
ctx = eikonal.Context(0)
T = ctx.tmap3d(c, goal)
walls, solves = [], []
for _ in range(n):
    t0 = time.perf_counter()
    T = ctx.tmap3d(c, goal)
    walls.append((time.perf_counter() - t0) * 1e3)
    solves.append(ctx.stats()["solve_ms"])
print(f"tmap3d 60x60x41 f64: wall median {np.median(walls):.3f} ms, device solve median {np.median(solves):.3f} ms, "
      f"finite {np.isfinite(T).mean():.3f}")
ctx.close()
