"""ms-to-path through the drop-in's host calls, call by call (bench.py ms_to_path's route):
eik_tmap2d_f64 (host cost -> host field) and eik_path2d_f64 (host field -> path), each timed alone."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import numpy as np
import eikonal

N = 4096
rng = np.random.default_rng(0)
cost = rng.uniform(1, 4, (N, N))
cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
ctx = eikonal.Context(0)
goal, start = (2048, 2048), (256, 256)
for rep in range(4):
    t0 = time.perf_counter()
    T = ctx.tmap2d(cost, goal)
    t1 = time.perf_counter()
    p, st = ctx.path2d(T, start, goal)
    t2 = time.perf_counter()
    Tc = np.array(T)  # a pageable copy of the field
    t3 = time.perf_counter()
    p2, _ = ctx.path2d(Tc, start, goal)
    t4 = time.perf_counter()
    s = ctx.stats()
    print(f"tmap2d {1e3 * (t1 - t0):7.2f} ms (solve {s['solve_ms']:.2f})  path2d(pinned field) {1e3 * (t2 - t1):6.2f} ms  "
          f"path2d(pageable field) {1e3 * (t4 - t3):6.2f} ms  points {len(p)}", flush=True)
