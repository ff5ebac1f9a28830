"""Study: rebuild FastMarching3D.computeTmap's early-exit field (:126-145, break at :141) from the
full field.  Compares reconstructions with the oracle's exact early-exit run (pop order traced).
Test infrastructure / design study only."""
import sys, os, math
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O

OFF = [(0, 0, -1), (0, 0, 1), (-1, 0, 0), (1, 0, 0), (0, 1, 0), (0, -1, 0)]  # (dx,dy,dz) child order :21-33


def sumlist(v):
    return v[0] if len(v) == 1 else v[0] + sumlist(v[1:])


def solve3(tx, ty, tz, C):
    arr = [tx, ty, tz]
    tr = math.inf
    while tr == math.inf:
        n = len(arr)
        if n == 0:
            raise ValueError
        tmax = max(arr)
        s = 0.0
        for a in arr:
            s = s + math.pow(tmax - a, 2)
        if math.pow(C, 2) > s:
            S = sumlist(arr); Q = sumlist([a * a for a in arr])
            tr = (S + math.sqrt(n * math.pow(C, 2) + math.pow(S, 2) - n * Q)) / n
        arr.remove(tmax)
    return tr


def tget(T, x, y, z):
    H, W, L = T.shape
    if 0 <= x < W and 0 <= y < H and 0 <= z < L:
        return T[y, x, z]
    return math.inf


def local_solve(T, cost, x, y, z):
    tx = min(tget(T, x - 1, y, z), tget(T, x + 1, y, z))
    ty = min(tget(T, x, y - 1, z), tget(T, x, y + 1, z))
    tz = min(tget(T, x, y, z - 1), tget(T, x, y, z + 1))
    return solve3(tx, ty, tz, cost[y, x, z])


def reconstruct(cost, Tf, start, mode, order=None):
    """order: per-cell pop key (lower = earlier); default Tf itself."""
    H, W, L = cost.shape
    sx, sy, sz = (int(v) for v in start)
    Ts = Tf[sy, sx, sz]
    key = Tf if order is None else order
    ks = key[sy, sx, sz]
    closed = np.isfinite(cost) & (key < ks)
    closed[sy, sx, sz] = True
    E = np.where(closed, Tf, np.inf)
    # band: finite-cost, not closed, next to a closed cell
    band = []
    for y in range(H):
        for x in range(W):
            for z in range(L):
                if closed[y, x, z] or not np.isfinite(cost[y, x, z]):
                    continue
                for dx, dy, dz in OFF:
                    if 0 <= x + dx < W and 0 <= y + dy < H and 0 <= z + dz < L and closed[y + dy, x + dx, z + dz]:
                        band.append((x, y, z))
                        break
    if mode == "A":  # closed-only solve
        for (x, y, z) in band:
            E[y, x, z] = local_solve(E, cost, x, y, z)
        # (in-place: later band cells see earlier ones -- undo by using a copy)
        E2 = np.where(closed, Tf, np.inf)
        for (x, y, z) in band:
            E[y, x, z] = local_solve(E2, cost, x, y, z)
    elif mode == "B":  # Jacobi fixed point over the band
        for it in range(50):
            Ep = E.copy()
            for (x, y, z) in band:
                E[y, x, z] = min(Ep[y, x, z], local_solve(Ep, cost, x, y, z))
            if np.array_equal(E, Ep):
                break
    elif mode == "C":  # event replay on band cells, closed cells at their final values
        ev = []
        for (x, y, z) in band:
            for k, (dx, dy, dz) in enumerate(OFF):
                qx, qy, qz = x - dx, y - dy, z - dz  # q's child k is this cell
                if 0 <= qx < W and 0 <= qy < H and 0 <= qz < L and closed[qy, qx, qz]:
                    ev.append((key[qy, qx, qz], k, (x, y, z)))
        ev.sort(key=lambda e: (e[0], e[1]))
        for _, _, (x, y, z) in ev:
            v = local_solve(E, cost, x, y, z)
            if v < E[y, x, z]:
                E[y, x, z] = v
    return E, closed


def compare(name, cost, goal, start):
    Tf = O.fmm3d(cost, goal)
    Tee, pop = O.fmm3d_trace(cost, goal, start)
    tclosed = pop >= 0
    tband = np.isfinite(Tee) & ~tclosed
    res = {}
    for mode in ("A", "B", "C"):
        for oname, order in (("Tf", None), ("pop", np.where(pop >= 0, pop.astype(float), np.inf))):
            if oname == "pop" and mode != "C":
                continue
            E, closed = reconstruct(cost, Tf, start, mode, order)
            cm = int((closed != (tclosed & np.isfinite(cost))).sum())
            fin = np.array_equal(np.isfinite(E), np.isfinite(Tee))
            both = np.isfinite(E) & np.isfinite(Tee)
            err = np.abs(E[both] - Tee[both])
            nbad = int((err > 1e-9).sum())
            bandbad = int((np.abs(E - Tee)[tband & both] > 1e-9).sum())
            pa, sa = O.gdm3d(Tee, np.array(start, float), np.array(goal, float))
            pb, sb = O.gdm3d(E, np.array(start, float), np.array(goal, float))
            same = pa.shape == pb.shape and np.allclose(pa, pb, atol=1e-9)
            if pa.size and pb.size:
                from scipy.spatial.distance import cdist
                dm = cdist(pa, pb)
                haus = max(dm.min(0).max(), dm.min(1).max())
            else:
                haus = np.nan
            print(f"{name} mode {mode}/{oname}: closed mismatch {cm}, finite-mask equal {fin}, cells >1e-9: {nbad} "
                  f"(band {bandbad} of {int(tband.sum())}), max err {err.max() if err.size else 0:.3g}, "
                  f"path equal {same} ({len(pa)} vs {len(pb)}), Hausdorff {haus:.3g}", flush=True)


if __name__ == "__main__":
    d = np.load(os.path.join(ROOT, "tests/golden/fmm3d.npz"))
    for i in range(int(d["n_cases"])):
        compare(f"v{i}", d[f"v{i}_cost"].astype(np.float64), d[f"v{i}_goal"], d[f"v{i}_start"])
