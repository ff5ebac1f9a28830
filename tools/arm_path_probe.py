"""Timeline of the planner's arm call (host DEM area -> end-effector volume -> FM3D early-exit
field -> 3D path, eik_arm_path_f64) on bench.py's end-effector case: wall time per call; run
under rocprofv3 --kernel-trace and read the gaps with tools/trace_gaps.py.
  python tools/arm_path_probe.py [calls]"""
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal  # noqa: E402
import planner  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
half, m, res = 30, 40, 0.05  # bench.py bench_arm's case
rng = np.random.default_rng(5)
n = 2 * half
yy, xx = np.mgrid[0:n, 0:n] * res
Z = 0.1 * np.sin(2.1 * xx) * np.cos(0.9 * yy + 0.3) + 0.03 * rng.standard_normal((n, n))
Z -= Z.min()
resX = res * (2 * n - 1) / (2 * n)
sZ = int(round((Z.max() + 0.5) / 0.02))
obst = (rng.random((n, n)) < 0.1).astype(np.float64)
p0, p1 = np.array([0.2, 0.35]) * n * resX, np.array([0.6, 0.5]) * n * resX
t = np.linspace(0, 1, m)[:, None]
base = np.zeros((m, 3))
base[:, :2] = p0 + t * (p1 - p0)
base[:, 2] = 0.25
heading = np.stack([np.zeros(m), np.zeros(m), np.full(m, math.atan2(*(p1 - p0)[::-1]))], 1)
fw = np.uint32(np.round([(p1[0] + 0.2) / resX, (p1[1] + 0.15) / resX, (Z.max() * 0.6 + 0.1) / 0.02]))
iw = np.uint32(np.round([(p0[0] + 0.15) / resX, (p0[1] + 0.1) / resX, 0.45 / 0.02]))
vol = planner.volume(n, n, sZ, resX, resX, 0.02, 1.0, 2.0, 0.527, 0.2673, 0.1105, fw, iw)
ctx = eikonal.Context(0)
path, st = ctx.arm_path(Z, obst, base, heading, vol, 0.5)[:2]
walls = []
for _ in range(calls):
    t0 = time.perf_counter()
    ctx.arm_path(Z, obst, base, heading, vol, 0.5)
    walls.append((time.perf_counter() - t0) * 1e3)
print(f"arm_path {n}x{n}x{sZ}: wall median {np.median(walls):.3f} ms, {len(path)} points, status {st}")
ctx.close()
