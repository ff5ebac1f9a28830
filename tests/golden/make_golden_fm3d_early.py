"""Golden fixtures for FastMarching3D as the planner CALLS it: early exit at ``start``.

The planner solves the end-effector volume with ``FM3D.computeTmap(Cmap, finalWayPointArm,
initialWayPointArm)`` (Coupled_motion_planner.py:1636) and descends the returned field with
``FM3D.getPathGDM(Tmap3D, initialWayPointArm, finalWayPointArm, 0.5)`` (:1639).  computeTmap
stops as soon as ``start`` is popped (FastMarching3D.py:141), so the field is PARTIAL: cells
popped before ``start`` hold their final values, the narrow band its tentative values and the
rest +inf -- and np.gradient (:200) sees all of it.  This script records that partial field and
the path descended on it, on

  * cubes  -- random / uniform / obstacle volumes with +inf faces (trilinear walks),
  * arm    -- the end-effector volumes of tests/golden/make_golden_arm.py (Cmap = GetObstMap's
              final map x TunnelCost, :1576-1627), goal = finalWayPointArm, start =
              initialWayPointArm, exactly the planner's call.

Run ONCE in the build container (reference sources readable):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fm3d_early.py

Output: fm3d_early.npz next to this script (inputs + the reference's outputs only).  Nothing under
tests/ reads /root/reference at test time.
"""
import os
import sys
import time
import warnings

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF_SRC)
sys.path.insert(0, OUT)
warnings.simplefilter("ignore")

import FastMarching.FastMarching3D as FM3D  # noqa: E402  (reference, read-only)
import make_golden_arm as ARM  # noqa: E402  (compiles GetObstMap / TunnelCost from the reference)


def run(fn, *a):
    try:
        return fn(*a), None
    except Exception as e:  # the reference's own failure modes are recorded, not hidden
        return None, f"{type(e).__name__}: {e}"


def faces_inf(c):
    c = c.copy()
    c[0, :, :] = c[-1, :, :] = np.inf
    c[:, 0, :] = c[:, -1, :] = np.inf
    c[:, :, 0] = c[:, :, -1] = np.inf
    return c


def cube(kind, h, w, L, seed):
    r = np.random.default_rng(5000 + seed)
    if kind == "uniform":
        c = np.ones((h, w, L))
    elif kind == "random":
        c = r.uniform(1.0, 4.0, (h, w, L))
    elif kind == "obst":
        c = r.uniform(1.0, 4.0, (h, w, L))
        c[r.random((h, w, L)) < 0.12] = np.inf
    elif kind == "levels":  # few distinct costs: many exact ties in the band
        c = r.integers(1, 4, (h, w, L)).astype(np.float64)
    c = faces_inf(c.astype(np.float32).astype(np.float64))
    while True:
        goal = np.array([r.integers(1, w - 1), r.integers(1, h - 1), r.integers(1, L - 1)], np.uint32)
        start = np.array([r.integers(1, w - 1), r.integers(1, h - 1), r.integers(1, L - 1)], np.uint32)
        if np.isfinite(c[goal[1], goal[0], goal[2]]) and np.isfinite(c[start[1], start[0], start[2]]) \
                and np.abs(goal.astype(int) - start.astype(int)).sum() > (h + w + L) // 4:
            break
    return c, goal, start


def main():
    t0 = time.time()
    out = {}
    cases = [("uniform", 18, 20, 16, 0), ("random", 24, 22, 18, 1), ("obst", 26, 30, 14, 2),
             ("levels", 20, 20, 20, 3), ("random", 12, 40, 10, 4), ("obst", 30, 26, 22, 5)]
    n = 0
    for kind, h, w, L, seed in cases:
        c, goal, start = cube(kind, h, w, L, seed)
        out[f"c{n}_kind"] = np.array("cube:" + kind)
        out[f"c{n}_cost"] = c.astype(np.float32)
        out[f"c{n}_goal"] = goal.astype(np.int64)
        out[f"c{n}_start"] = start.astype(np.int64)
        n += 1
    for i, (seed, half, grid) in enumerate([(1, 16, False), (2, 20, True), (3, 24, False), (4, 30, False)]):
        a = ARM.case(seed, half, sample_on_grid=grid)
        cm = a["finalMap"] * a["tunnel"]  # :1627
        out[f"c{n}_kind"] = np.array(f"arm:seed{seed}:half{half}")
        out[f"c{n}_cost"] = cm  # f64 as the planner builds it (not float32-exact)
        out[f"c{n}_goal"] = a["finalWP"].astype(np.int64)
        out[f"c{n}_start"] = a["initWP"].astype(np.int64)
        n += 1
    for i in range(n):
        p = f"c{i}_"
        c = out[p + "cost"].astype(np.float64)
        goal = out[p + "goal"].astype(np.uint32)
        start = out[p + "start"].astype(np.uint32)
        T, e1 = run(FM3D.computeTmap, c, goal, start)  # :1636
        out[p + "T_early"] = T if T is not None else np.zeros((0, 0, 0))
        out[p + "err"] = np.array(e1 or "")
        path, e2 = (None, "no field") if T is None else run(FM3D.getPathGDM, T, start, goal, 0.5)  # :1639
        out[p + "path"] = path if path is not None else np.zeros((0, 3))
        out[p + "path_err"] = np.array(e2 or "")
        print(f"{p} {out[p + 'kind']} {c.shape} err={e1} path={None if path is None else path.shape} "
              f"perr={e2} t={time.time() - t0:.1f}s", flush=True)
    out["n_cases"] = np.array(n)
    np.savez_compressed(os.path.join(OUT, "fm3d_early.npz"), **out)


if __name__ == "__main__":
    main()
