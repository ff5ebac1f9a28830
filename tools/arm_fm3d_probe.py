"""FM3D (general 3D solver, fim3d.hip) on the bench's end-effector volume: wall time, device solve
time, launches and visits, for several host-sync cadences (EIK_OPT_SYNC_EVERY)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal
from eikonal import _lib as L
import bench

ctx = eikonal.Context(0)
_orig = bench.timed_loop
cap = {}


def grab(fn, steps, warmup=1):  # capture the arm volume bench_arm builds, skip its timing loops
    return _orig(fn, 1, 0)


bench.timed_loop = grab
import planner  # noqa: E402
orig_arm_path = ctx.arm_path


def arm_path(*a, **k):
    want = k.pop("want_fields", False)
    r = orig_arm_path(*a, want_fields=True, **k)
    cap["cost"], cap["args"] = r[2], a
    return r if want else r[:2]


ctx.arm_path = arm_path
bench.bench_arm(ctx, 1)
cost = cap["cost"]
H, W, Lz = cost.shape
fin = np.argwhere(np.isfinite(cost))
goal = fin[len(fin) // 2][[1, 0, 2]]
print("volume", cost.shape, "goal", goal, flush=True)
# the whole volume -> FM3D (early exit) -> path call, and its solve's share
a = cap["args"]
ref = None
for mode in (L.MODE_PERSISTENT, L.MODE_LIST, L.MODE_PERSISTENT, L.MODE_LIST):
    ctx.set_option(L.OPT_MODE, mode)
    for _ in range(3):
        t0 = time.perf_counter()
        path, st = orig_arm_path(*a)
        el = (time.perf_counter() - t0) * 1e3
        s = ctx.stats()
        same = ref is None or (path.shape == ref.shape and np.abs(path - ref).max() <= 1e-9)
        ref = path if ref is None else ref
        print(f"mode {mode}: arm_path wall {el:.3f} ms; its FM3D solve: device {s['solve_ms']:.3f} ms, launches "
              f"{s['iterations']}, visits {s['tile_visits']}; path {len(path)} points, same as the first: {same}",
              flush=True)
ctx.set_option(L.OPT_MODE, L.MODE_LIST)
for se, grid in ((32, 0), (32, 256)):
    ctx.set_option(L.OPT_SYNC_EVERY, se)
    ctx.set_option(L.OPT_GRID, grid)
    ctx.tmap3d(cost, goal)
    t0 = time.perf_counter()
    for _ in range(10):
        ctx.tmap3d(cost, goal)
    el = (time.perf_counter() - t0) / 10 * 1e3
    s = ctx.stats()
    print(f"sync_every={se} grid={grid or 'default'}: wall {el:.3f} ms, device {s['solve_ms']:.3f} ms, launches {s['iterations']}, "
          f"visits {s['tile_visits']}", flush=True)
Tl = ctx.tmap3d(cost, goal)
ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
ctx.set_option(L.OPT_GRID, 0)
for _ in range(2):
    t0 = time.perf_counter()
    for _ in range(10):
        Tp = ctx.tmap3d(cost, goal)
    el = (time.perf_counter() - t0) / 10 * 1e3
    s = ctx.stats()
    print(f"persistent: wall {el:.3f} ms, device {s['solve_ms']:.3f} ms, visits {s['tile_visits']}", flush=True)
fin = np.isfinite(Tl)
print("persistent vs list field: masks equal", np.array_equal(fin, np.isfinite(Tp)), "max abs",
      float(np.abs(Tl[fin] - Tp[fin]).max()), flush=True)
# in-tile relaxation passes per visit (EIK_OPT_PASSES), persistent driver
for passes in (24, 48, 24, 48):
    ctx.set_option(L.OPT_PASSES, passes)
    ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
    ctx.tmap3d(cost, goal)
    t0 = time.perf_counter()
    for _ in range(10):
        ctx.tmap3d(cost, goal)
    el = (time.perf_counter() - t0) / 10 * 1e3
    s = ctx.stats()
    t1 = time.perf_counter()
    orig_arm_path(*a)
    el2 = (time.perf_counter() - t1) * 1e3
    s2 = ctx.stats()
    print(f"passes {passes}: full field wall {el:.3f} ms, device {s['solve_ms']:.3f} ms, visits {s['tile_visits']} passes {s['inplace_passes']}; "
          f"arm_path wall {el2:.3f} ms, early-exit solve {s2['solve_ms']:.3f} ms, visits {s2['tile_visits']}", flush=True)
