"""Generate the golden fixtures that pin the oracle (and, through it, the HIP path).

Run ONCE in the build container, where the reference Python sources are readable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own ``FastMarching.FastMarching`` / ``FastMarching3D`` modules from
``/root/reference/src`` (read-only, never copied) and records inputs + outputs as ``.npz``
fixtures next to this script.  Nothing under ``tests/`` reads ``/root/reference`` at test time;
the GPU box only sees the committed ``.npz`` files.

Drivers (reference file:line they follow):
  * full 2D field  -- the loop of ``FastMarching.py:92-112`` driven with the reference's own
    ``updateNode``/``getMinNB`` and a 3-value unpack (``computeTmap`` itself raises at :107,
    SURVEY.md §3.2); optional early exit when ``start`` is popped (:108-109).
  * bidirectional  -- ``biComputeTmap`` ``FastMarching.py:114-162`` as is.
  * 2D paths       -- ``getPathGDM`` ``FastMarching.py:164-236`` as is.
  * 3D field/path  -- ``FastMarching3D.computeTmap`` :126-145 / ``getPathGDM`` :198-271 as is.
  * helpers        -- ``getEikonal`` :17-29, ``computeGradient`` :242-300, ``interpolatePoint``
    :305-338 (2D) and ``FastMarching3D.interpolatePoint`` :275-314.

Costs are drawn so every value is exactly representable in float32 (stored as float32,
used as float64 exactly like the reference would see them).
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
warnings.simplefilter("ignore")

import FastMarching.FastMarching as FM  # noqa: E402  (reference, read-only)
import FastMarching.FastMarching3D as FM3D  # noqa: E402


# ----------------------------------------------------------------------------- cost generators
def _border(c):
    c = c.copy()
    c[0, :] = np.inf
    c[-1, :] = np.inf
    c[:, 0] = np.inf
    c[:, -1] = np.inf
    return c


def cost_uniform(h, w, seed=0):
    return _border(np.ones((h, w)))


def cost_random(h, w, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(1.0, 10.0, (h, w)).astype(np.float32).astype(np.float64)
    return _border(c)


def cost_obstacles(h, w, seed, frac=0.12):
    rng = np.random.default_rng(seed)
    c = rng.uniform(1.0, 10.0, (h, w)).astype(np.float32).astype(np.float64)
    c[rng.random((h, w)) < frac] = np.inf
    return _border(c)


def cost_blobs(h, w, seed, jitter=True):
    """Planner-like raster: disk obstacles at cost 300, distance ramp, box blur
    (the shape of Coupled_motion_planner.py:1183-1216, in miniature)."""
    from scipy import ndimage

    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    obst = np.zeros((h, w))
    for _ in range(max(3, (h * w) // 900)):
        cy, cx, r = rng.integers(0, h), rng.integers(0, w), rng.integers(2, max(3, h // 10))
        obst[(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1.0
    dist = ndimage.distance_transform_edt(obst == 0)
    ramp = np.clip(1.0 - dist / 6.0, 0.0, 1.0)
    c = 1.0 + 300.0 * obst + 10.0 * ramp
    c = ndimage.uniform_filter(c, size=5, mode="constant", cval=300.0)
    if jitter:  # break the exact ties of blurred plateaus (see "blobs_ties" for why)
        c = c + rng.uniform(0.0, 1e-3, c.shape)
    c = c.astype(np.float32).astype(np.float64)
    return _border(c)


def cost_blobs_ties(h, w, seed):
    """Un-jittered blobs: exact ties on plateaus make the reference's decrease-key raise
    StopIteration (FastMarching.py:72-73 with nIndex == 0) -- recorded as data."""
    return cost_blobs(h, w, seed, jitter=False)


GENS = {"uniform": cost_uniform, "random": cost_random, "obst": cost_obstacles, "blobs": cost_blobs,
        "blobs_ties": cost_blobs_ties}


def free_cell(c, rng, avoid=None):
    h, w = c.shape
    while True:
        x, y = int(rng.integers(2, w - 2)), int(rng.integers(2, h - 2))
        if np.isfinite(c[y, x]) and (avoid is None or abs(x - avoid[0]) + abs(y - avoid[1]) > (h + w) // 4):
            return [x, y]


def connect(c, a, b):
    """Make sure a and b are in one 4-connected finite component (carve a straight L if not)."""
    from scipy import ndimage

    lab, _ = ndimage.label(np.isfinite(c))
    if lab[a[1], a[0]] == lab[b[1], b[0]] and lab[a[1], a[0]] != 0:
        return c
    c = c.copy()
    x0, y0 = a
    x1, y1 = b
    for x in range(min(x0, x1), max(x0, x1) + 1):
        if not np.isfinite(c[y0, x]):
            c[y0, x] = 5.0
    for y in range(min(y0, y1), max(y0, y1) + 1):
        if not np.isfinite(c[y, x1]):
            c[y, x1] = 5.0
    return c


# ----------------------------------------------------------------------------- reference drivers
def ref_full_field(cost, goal, start=None):
    """FastMarching.py:92-112 with the 3-value unpack; start=None -> full field."""
    closed = np.zeros_like(cost)
    closed[np.where(cost == np.inf)] = 1
    T = np.ones_like(cost) * np.inf
    nbT, nbNodes = [], []
    T[goal[1], goal[0]] = 0
    closed[goal[1], goal[0]] = 1
    node = [goal[0], goal[1]]
    T, nbT, nbNodes = FM.updateNode(node, cost, T, nbT, nbNodes, closed)
    pops = 0
    while nbT:
        node, nbT, nbNodes = FM.getMinNB(nbT, nbNodes)
        closed[node[1], node[0]] = 1
        T, nbT, nbNodes = FM.updateNode(node, cost, T, nbT, nbNodes, closed)
        pops += 1
        if start is not None and np.array_equal(node, start):
            break
    return T, pops


def run(fn, *a):
    try:
        return fn(*a), None
    except Exception as e:  # the reference's own failure modes are recorded as data
        return None, type(e).__name__


def main():
    t0 = time.time()
    rng = np.random.default_rng(2024)

    # ---------------------------------------------------------------- 1. full 2D fields (+paths)
    f2 = {}
    cases = []
    for size in (64, 96, 128):
        for kind in ("uniform", "random", "obst", "blobs"):
            cases.append((size, kind))
    cases.append((64, "blobs_ties"))
    for ci, (size, kind) in enumerate(cases):
        h = size
        w = size + (8 if kind == "random" else 0)  # one non-square family
        if kind == "blobs_ties":  # a seed/goal on which the reference's decrease-key raises
            c = GENS[kind](h, w, 103)
            goal, start = [54, 6], [11, 12]
        else:
            c = GENS[kind](h, w, 100 + ci)
            goal = free_cell(c, rng)
            start = free_cell(c, rng, avoid=goal)
        c = connect(c, goal, start)
        res, ferr = run(ref_full_field, c, goal)
        T, pops = res if res is not None else (np.zeros((0, 0)), -1)
        p = f"c{ci}_"
        f2[p + "err"] = np.array(ferr or "")
        f2[p + "cost"] = c.astype(np.float32)
        f2[p + "goal"] = np.array(goal, np.int64)
        f2[p + "start"] = np.array(start, np.int64)
        f2[p + "T"] = T
        f2[p + "kind"] = np.array(kind)
        # early-exit variant (stops when start is popped) -- only for the smallest size
        if size == 64:
            res, eerr = run(ref_full_field, c, goal, start)
            f2[p + "T_early"] = res[0] if res is not None else np.zeros((0, 0))
            f2[p + "early_err"] = np.array(eerr or "")
        # GDM path on the full field, start -> goal (planner convention: init is an ndarray)
        path, err = run(FM.getPathGDM, T, np.array(start, np.uint32), list(goal), 0.5) if ferr is None \
            else (None, "no-field")
        f2[p + "path"] = path if path is not None else np.zeros((0, 2))
        f2[p + "path_err"] = np.array(err or "")
        print(f"[2d] {p} {kind} {h}x{w} ferr={ferr} pops={pops} path={None if path is None else path.shape} err={err} "
              f"t={time.time()-t0:.1f}s", flush=True)
    f2["n_cases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(OUT, "fmm2d_fields.npz"), **f2)

    # ---------------------------------------------------------------- 2. bidirectional + paths
    bi = {}
    kinds = ["uniform", "uniform", "random", "random", "obst", "blobs"]
    for bi_i, kind in enumerate(kinds):
        c = GENS[kind](80, 80, 500 + bi_i)
        goal = free_cell(c, rng)
        start = free_cell(c, rng, avoid=goal)
        c = connect(c, goal, start)
        res, err = run(FM.biComputeTmap, c, goal, start)
        p = f"b{bi_i}_"
        bi[p + "cost"] = c.astype(np.float32)
        bi[p + "goal"] = np.array(goal, np.int64)
        bi[p + "start"] = np.array(start, np.int64)
        bi[p + "err"] = np.array(err or "")
        if res is not None:
            TG, TS, join = res
            bi[p + "TG"] = TG
            bi[p + "TS"] = TS
            bi[p + "join"] = join.astype(np.uint32)
            pg, eg = run(FM.getPathGDM, TG, join, goal, 0.5)
            ps, es = run(FM.getPathGDM, TS, join, start, 0.5)
            bi[p + "pathG"] = pg if pg is not None else np.zeros((0, 2))
            bi[p + "pathS"] = ps if ps is not None else np.zeros((0, 2))
            bi[p + "pathG_err"] = np.array(eg or "")
            bi[p + "pathS_err"] = np.array(es or "")
            print(f"[bi] {p} {kind} join={join} pathG={None if pg is None else pg.shape} "
                  f"pathS={None if ps is None else ps.shape} t={time.time()-t0:.1f}s", flush=True)
        else:
            print(f"[bi] {p} {kind} reference raised {err}", flush=True)
    bi["n_cases"] = np.array(len(kinds))
    np.savez_compressed(os.path.join(OUT, "fmm2d_bidir.npz"), **bi)

    # ---------------------------------------------------------------- 3. 3D volumes + paths
    v3 = {}
    vcases = [("layers", 48, 48, 5, 0), ("layers", 40, 56, 5, 1), ("cube", 20, 20, 20, 2), ("cube", 16, 24, 12, 3)]
    for vi, (kind, h, w, L, seed) in enumerate(vcases):
        r = np.random.default_rng(900 + seed)
        c = r.uniform(1.0, 4.0, (h, w, L))
        if kind == "layers":
            c[:, :, 2] *= 1.5  # per-mode factors (3 locomotion layers: z = 1..3)
            c[:, :, 3] *= 0.75
            c[r.random((h, w, L)) < 0.06] = np.inf
        c = c.astype(np.float32).astype(np.float64)  # float32-exact, stored losslessly
        c[0, :, :] = np.inf
        c[-1, :, :] = np.inf
        c[:, 0, :] = np.inf
        c[:, -1, :] = np.inf
        c[:, :, 0] = np.inf
        c[:, :, -1] = np.inf
        while True:
            goal = np.array([r.integers(2, w - 2), r.integers(2, h - 2), r.integers(1, L - 1)], np.uint32)
            start = np.array([r.integers(2, w - 2), r.integers(2, h - 2), r.integers(1, L - 1)], np.uint32)
            if np.isfinite(c[goal[1], goal[0], goal[2]]) and np.isfinite(c[start[1], start[0], start[2]]) \
                    and np.abs(goal.astype(int) - start.astype(int)).sum() > (h + w) // 3:
                break
        # full field: an unreachable (inf) start means the band empties before an early exit
        Tfull, e1 = run(FM3D.computeTmap, c, goal, np.array([0, 0, 0], np.uint32))
        Tearly, e2 = run(FM3D.computeTmap, c, goal, start)
        p = f"v{vi}_"
        v3[p + "cost"] = c.astype(np.float32)
        v3[p + "goal"] = goal.astype(np.int64)
        v3[p + "start"] = start.astype(np.int64)
        v3[p + "T"] = Tfull
        v3[p + "T_early"] = Tearly
        v3[p + "err"] = np.array((e1 or "") + "|" + (e2 or ""))
        path, e3 = run(FM3D.getPathGDM, Tearly, start, goal, 0.5)
        v3[p + "path"] = path if path is not None else np.zeros((0, 3))
        v3[p + "path_err"] = np.array(e3 or "")
        print(f"[3d] {p} {kind} {h}x{w}x{L} err={e1},{e2} path={None if path is None else path.shape} "
              f"perr={e3} t={time.time()-t0:.1f}s", flush=True)
    v3["n_cases"] = np.array(len(vcases))
    np.savez_compressed(os.path.join(OUT, "fmm3d.npz"), **v3)

    # ---------------------------------------------------------------- 4. scalar helpers
    hp = {}
    ins, outs = [], []
    vals = [0.0, 0.5, 1.0, 2.0, 3.75, 10.0, np.inf]
    for a in vals:
        for b in vals:
            for c in (0.25, 1.0, 2.5, 7.0):
                ins.append((a, b, c))
                outs.append(float(FM.getEikonal(np.float64(a), np.float64(b), np.float64(c))))
    r = np.random.default_rng(7)
    for _ in range(2000):
        a, b = r.uniform(0, 50, 2)
        c = r.uniform(0.01, 20)
        ins.append((a, b, c))
        outs.append(float(FM.getEikonal(np.float64(a), np.float64(b), np.float64(c))))
    hp["eik_in"] = np.array(ins)
    hp["eik_out"] = np.array(outs)
    # computeGradient over a whole small field (point=[]), with infs in it
    Tg = f2["c1_T"][:40, :44].copy()
    Tg[10:14, 20:23] = np.inf
    gnx, gny = FM.computeGradient(Tg)
    hp["grad_T"] = Tg
    hp["grad_nx"] = gnx
    hp["grad_ny"] = gny
    # windowed form at a point
    gnx_w, gny_w = FM.computeGradient(Tg, np.array([17.3, 22.8]))
    hp["gradw_pt"] = np.array([17.3, 22.8])
    hp["gradw_nx"] = gnx_w
    hp["gradw_ny"] = gny_w
    pts = np.column_stack([r.uniform(0, 42, 300), r.uniform(0, 38, 300)])
    pts[:20, 0] = np.floor(pts[:20, 0])  # exercise the a == 0 / b == 0 branches
    pts[10:30, 1] = np.floor(pts[10:30, 1])
    hp["interp_pts"] = pts
    hp["interp_map"] = f2["c1_T"][:40, :44]
    hp["interp_out"] = np.array([float(FM.interpolatePoint(p_, hp["interp_map"])) for p_ in pts])
    M3 = r.uniform(-3, 3, (9, 10, 6))
    pts3 = np.column_stack([r.uniform(0, 8.5, 200), r.uniform(0, 7.5, 200), r.uniform(0, 4.5, 200)])
    hp["interp3_map"] = M3
    hp["interp3_pts"] = pts3
    hp["interp3_out"] = np.array([float(FM3D.interpolatePoint(p_, M3)) for p_ in pts3])
    np.savez_compressed(os.path.join(OUT, "helpers.npz"), **hp)
    print(f"done in {time.time()-t0:.1f}s")


if __name__ == "__main__":
    main()
