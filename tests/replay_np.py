"""numpy restatement of the exact band replay's formulation (test infrastructure, not product code:
the product is csrc/bidir_exact.hip).  It is the CPU prototype the kernels were written from, kept so
that the formulation itself is pinned to the reference's outputs on the CPU:

  every value the reference's narrow band ever writes (FastMarching.py:44-80) is an EVENT
      g(y, d) = getEikonal (:17-29) over y's neighbours as they stand when y's neighbour in direction d
                pops (rank t), updateNode's children being y-1, y+1, x-1, x+1 (:46-54),
  where a cell z holds, at time t, V(z, t) = min over its events of time < min(t, rank z) (0 for the
  source); the events are a DAG in pop order (Jacobi sweeps reach its unique solution), a popped
  cell's value is V(y, rank y), and pops follow (value, -seq) with seq the insertion time of the value
  (bisect_left: latest insertion first among equal T, :65 / :76).  The ranks are iterated to their
  fixed point from a field's (T, node) order.

The device additionally orders exact-tie runs as stacks and handles rounding inversions
(bidir_exact.hip exact_ties_kernel / exact_keys_kernel); the reference fixtures used here need neither,
and the GPU tests cover both (tests/test_gpu_bidir_exact.py integer rasters, fm3d_early c3)."""
import numpy as np

INF = np.inf
DXY = [(0, -1), (0, 1), (-1, 0), (1, 0)]  # updateNode's children (x, y), FastMarching.py:46-54
BIG = np.iinfo(np.int64).max


def eik(a, b, c):
    """getEikonal FastMarching.py:17-29, elementwise (np.power(., 2): exact products)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    with np.errstate(invalid="ignore"):
        d = a - b
        two = .5 * (a + b + np.sqrt(2 * (c * c) - d * d))
        r = np.where(c < np.abs(d), np.minimum(a, b) + c, two)
    return np.where(np.isinf(a), np.where(np.isinf(b), INF, b + c), np.where(np.isinf(b), a + c, r))


def shift(A, dx, dy, fill):
    """B[y, x] = A[y + dy, x + dx] (fill outside)."""
    H, W = A.shape[:2]
    B = np.full_like(A, fill)
    B[max(0, -dy):H - max(0, dy), max(0, -dx):W - max(0, dx)] = A[max(0, dy):H - max(0, -dy), max(0, dx):W - max(0, -dx)]
    return B


def relax(cost, src, rank, g):
    """Jacobi sweeps of every event g[y, x, d] to the DAG's fixed point for the given ranks."""
    H, W = cost.shape
    sx, sy = src
    t = np.stack([shift(rank, dx, dy, BIG) for dx, dy in DXY], -1)  # time of event (y, d)
    valid = (t < rank[..., None]) & np.isfinite(cost)[..., None] & (t < BIG)
    valid[sy, sx, :] = False
    issrc = np.zeros((H, W), bool)
    issrc[sy, sx] = True
    nb = []
    for dx, dy in DXY:  # per neighbour: its rank, its events' times, source flag
        nb.append((shift(rank, dx, dy, BIG), [shift(t[..., k], dx, dy, BIG) for k in range(4)], shift(issrc, dx, dy, False), dx, dy))
    it = 0
    while True:
        it += 1
        gn = np.full((H, W, 4), INF)
        for d in range(4):
            vals = []
            for rz, tz, sz, dx, dy in nb:
                lim = np.minimum(t[..., d], rz)
                m = np.full((H, W), INF)
                for k in range(4):
                    gz = shift(g[..., k], dx, dy, INF)
                    m = np.where(tz[k] < lim, np.minimum(m, gz), m)
                vals.append(np.where(sz, 0.0, m))
            e = eik(np.minimum(vals[3], vals[2]), np.minimum(vals[1], vals[0]), cost)  # :57-63
            gn[..., d] = np.where(valid[..., d], e, INF)
        if np.array_equal(gn, g):
            return gn, t, valid, it
        g = gn


def keys(g, t, valid, src):
    """each cell's value (min over its events) and seq = 4 t + child index of the first event reaching it"""
    H, W = g.shape[:2]
    T = np.full((H, W), INF)
    seq = np.full((H, W), -1, np.int64)
    order = np.argsort(np.where(valid, t, BIG), axis=-1, kind="stable")
    for k in range(4):
        d = order[..., k]
        gv = np.take_along_axis(g, d[..., None], -1)[..., 0]
        tv = np.take_along_axis(t, d[..., None], -1)[..., 0]
        ok = np.take_along_axis(valid, d[..., None], -1)[..., 0] & (gv < T)  # a strict decrease (:70)
        T = np.where(ok, gv, T)
        seq = np.where(ok, tv * 4 + np.array([1, 0, 3, 2])[d], seq)
    T[src[1], src[0]] = 0.0
    seq[src[1], src[0]] = BIG
    return T, seq


def ranks(T, seq):
    H, W = T.shape
    f = np.nonzero(np.isfinite(T).ravel())[0]
    o = np.lexsort((-seq.ravel()[f], T.ravel()[f]))
    r = np.full(H * W, BIG, np.int64)
    r[f[o]] = np.arange(f.size)
    return r.reshape(H, W)


def replay(cost, src, T0, max_outer=1000):
    """One front: the pop ranks, events, event times and validity, from a field T0."""
    r = ranks(T0, np.zeros(T0.shape, np.int64))
    vals = [shift(T0, dx, dy, INF) for dx, dy in DXY]
    g = np.repeat(eik(np.minimum(vals[3], vals[2]), np.minimum(vals[1], vals[0]), cost)[..., None], 4, -1)
    for _ in range(max_outer):
        g, t, valid, _ = relax(cost, src, r, g)
        T, seq = keys(g, t, valid, src)
        r2 = ranks(T, seq)
        if np.array_equal(r2, r):
            return T, r, g, t, valid
        r = r2
    raise RuntimeError("ranks did not settle")


def bidir(cost, goal, start, TG0, TS0):
    """biComputeTmap FastMarching.py:114-162 from two fields: (TG, TS, nodeJoin)."""
    H, W = cost.shape
    fr = [replay(cost, goal, TG0), replay(cost, start, TS0)]
    rG, rS = fr[0][1].ravel(), fr[1][1].ravel()
    oG, oS = np.argsort(rG, kind="stable"), np.argsort(rS, kind="stable")
    nG, nS = int((rG < BIG).sum()), int((rS < BIG).sum())
    lastG, lastS = goal[1] * W + goal[0], start[1] * W + start[0]
    j = 0
    while True:  # :141-155
        j += 1
        if j >= nG and j >= nS:
            raise RuntimeError("the fronts never meet")
        if j < nG:
            lastG = int(oG[j])
        if j < nS:
            lastS = int(oS[j])
        if rS[lastG] <= j:
            join = lastG
            break
        if rG[lastS] <= j:
            join = lastS
            break
    out = []
    for T, r, g, t, valid in fr:
        P = np.full((H, W), INF)
        closed = r <= j
        P[closed] = T[closed]
        ev = valid & (t <= j)
        band = ~closed & ev.any(-1)
        P[band] = np.where(ev, g, INF).min(-1)[band]
        out.append(P)
    return out[0], out[1], np.array([join % W, join // W], np.uint32)
