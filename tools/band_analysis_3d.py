"""FM3D's early-exit band values (FastMarching3D.py:126-145, the planner's call at
Coupled_motion_planner.py:1636) against the reference's own (tests/golden/fm3d_early.npz): the
full-field value (the GPU's choice) vs the band relaxation (fixed point of the n-D local solve,
:59-75, over closed + band cells, every other cell +inf).  CPU only (oracle/); DESIGN §3.7."""
import math
import sys

import numpy as np

sys.path.insert(0, "oracle")
import oracle as O  # noqa: E402


def solve_nd(ts, c):
    """:59-75 on the axis minima ts (inf allowed)."""
    ta = [t for t in ts if not math.isinf(t)]
    while ta:
        n = len(ta)
        tmax = max(ta)
        if c * c > sum((tmax - t) ** 2 for t in ta):
            s = sum(ta)
            q = sum(t * t for t in ta)
            return (s + math.sqrt(n * c * c + s * s - n * q)) / n
        ta.remove(tmax)
    return math.inf


d = np.load("tests/golden/fm3d_early.npz")
cases = [k[:-5] for k in d.files if k.endswith("_cost")]
for p in sorted(cases):
    cost = d[p + "_cost"].astype(float)
    goal, start, R = d[p + "_goal"], d[p + "_start"], d[p + "_T_early"]
    H, W, L = cost.shape
    Tf = O.fmm3d(cost, goal)
    sx, sy, sz = (int(v) for v in start)
    if [sx, sy, sz] == [int(v) for v in goal] or not (0 <= sx < W and 0 <= sy < H and 0 <= sz < L):
        continue
    ts = Tf[sy, sx, sz]
    closed = Tf < ts
    closed[sy, sx, sz] = True
    P = np.pad(closed, 1, constant_values=False)
    nb = (P[1:-1, :-2, 1:-1] | P[1:-1, 2:, 1:-1] | P[:-2, 1:-1, 1:-1] | P[2:, 1:-1, 1:-1] | P[1:-1, 1:-1, :-2] |
          P[1:-1, 1:-1, 2:])
    band = nb & ~closed & np.isfinite(cost)
    T = np.where(closed, Tf, np.inf)
    cells = list(zip(*np.nonzero(band)))
    for it in range(1000):
        ch = False
        for (y, x, z) in cells:
            def v(yy, xx, zz):
                return T[yy, xx, zz] if 0 <= yy < H and 0 <= xx < W and 0 <= zz < L else math.inf
            w = solve_nd([min(v(y, x - 1, z), v(y, x + 1, z)), min(v(y - 1, x, z), v(y + 1, x, z)),
                          min(v(y, x, z - 1), v(y, x, z + 1))], cost[y, x, z])
            if w < T[y, x, z] * (1 - 2 ** -40):
                ch = True
            T[y, x, z] = min(T[y, x, z], w)
        if not ch:
            break
    sel = band & np.isfinite(R)
    if not sel.any():
        continue
    rf, rj = R[sel] / Tf[sel], R[sel] / T[sel]
    print(f"{p} ({str(d[p + '_kind'])}): band {int(sel.sum())}, full-field ratio max {rf.max():.4f} exact {np.mean(np.abs(rf - 1) < 1e-12):.2f}"
          f" | relaxed ratio min {rj.min():.4f} max {rj.max():.4f} exact {np.mean(np.abs(rj - 1) < 1e-12):.2f} ({it + 1} sweeps)")
