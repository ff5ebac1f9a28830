"""GPU parity of the bidirectional join alone (eik_bidir_join_f64: the step of biComputeTmap,
FastMarching.py:141-162, that turns the two fronts' fields into nodeJoin and the partial fields).

The oracle is the join's definition on the same fields, in numpy: rank = position in the stable
(T, node) order of the finite cells, k* = min over cells of max(rankG, rankS), the join = the
goal front's pop of rank k* when it qualifies (the G test runs first, :150-152) else the start
front's, the partial fields = cells of rank <= k* plus their 4-neighbours, +inf elsewhere.  The
device join ranks only the cells under a bound on k* (csrc/bidir.hip); these cases stress the
bound: exact ties, fronts of very different density (the threshold in the open-ended bucket),
goal == start, disjoint fields.  Bit-exact: index work.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import eikonal

    c = eikonal.Context(0)
    yield c
    c.close()


def ranks(T):
    n = T.size
    f = T.reshape(-1)
    fin = np.isfinite(f)
    order = np.lexsort((np.arange(n), f))  # by T, then node
    order = order[fin[order]]
    r = np.full(n, np.iinfo(np.int64).max, np.int64)
    r[order] = np.arange(order.size)
    return r


def join_oracle(TG, TS):
    H, W = TG.shape
    rg, rs = ranks(TG), ranks(TS)
    both = (rg != np.iinfo(np.int64).max) & (rs != np.iinfo(np.int64).max)
    assert both.any()
    m = np.maximum(rg, rs)
    packed = np.where(both, (2 * m + (rg != m)) * (1 << 29) + np.arange(TG.size), np.iinfo(np.int64).max)
    best = int(packed.min())
    node = best & ((1 << 29) - 1)
    k = best >> 30

    def partial(T, r):
        keep = (r <= k).reshape(H, W)
        nb = np.zeros_like(keep)
        nb[1:, :] |= keep[:-1, :]
        nb[:-1, :] |= keep[1:, :]
        nb[:, 1:] |= keep[:, :-1]
        nb[:, :-1] |= keep[:, 1:]
        return np.where(keep | nb, T, np.inf)

    return partial(TG, rg), partial(TS, rs), np.array([node % W, node // W], np.uint32), k


def cone(H, W, x, y, rng, noise=0.0, aniso=1.0):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    T = np.sqrt((xx - x) ** 2 * aniso + (yy - y) ** 2)
    if noise:
        T += noise * rng.random((H, W)) * (T > 0)
    return T


def make(case, rng):
    if case == "smooth":
        H, W = 300, 340
        TG, TS = cone(H, W, 250, 200, rng, 0.3), cone(H, W, 30, 40, rng, 0.3)
    elif case == "obstacles":
        H, W = 1024, 1024
        TG, TS = cone(H, W, 800, 700, rng, 0.5), cone(H, W, 100, 90, rng, 0.5)
        blk = rng.random((H, W)) < 0.1
        blk[700, 800] = blk[90, 100] = False
        TG[blk] = TS[blk] = np.inf
    elif case == "ties":  # integer fields: masses of exact ties, broken by node index
        H, W = 257, 263
        TG = np.floor(cone(H, W, 200, 100, rng))
        TS = np.floor(cone(H, W, 20, 220, rng))
    elif case == "manhattan":  # |dx| + |dy|: diamond fronts, every level a tie class
        H, W = 512, 384
        yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
        TG = np.abs(xx - 300) + np.abs(yy - 400)
        TS = np.abs(xx - 10) + np.abs(yy - 5)
    elif case == "lopsided":  # the start front is dense at small T: its threshold in the open bucket
        H, W = 768, 640
        TG = cone(H, W, 600, 700, rng, 0.2)
        TS = 1e-3 * cone(H, W, 20, 30, rng, 0.2)
        TS[TS > 0] += 5e3 * (TS[TS > 0] > 0.4)
    elif case == "corridor":  # a narrow strip of finite cells joining the two sources
        H, W = 256, 2048
        TG, TS = cone(H, W, 2000, 128, rng, 0.1), cone(H, W, 40, 128, rng, 0.1)
        wall = np.ones((H, W), bool)
        wall[120:136, :] = False
        TG[wall] = TS[wall] = np.inf
    elif case == "same_source":  # goal == start: k* = 0, the join is the source
        H, W = 200, 220
        TG = cone(H, W, 50, 60, rng, 0.2)
        TS = TG.copy()
    elif case == "float_ties":  # distinct doubles that round to one float: the sort's run fix-up
        H, W = 200, 220
        TG = np.floor(cone(H, W, 150, 120, rng)) + 1e-9 * rng.random((H, W))
        TS = np.floor(cone(H, W, 30, 40, rng)) + 1e-9 * rng.random((H, W))
        TG[120, 150] = TS[40, 30] = 0.0
    elif case == "zero_cost_patch":  # a zero-cost region around the goal -- ~1e5 distinct
        # T of ~2^-500 (the fp64 solver's staged cost floor) all round to the float 0, one run of
        # equal 32-bit keys in no node order: the fix-up hands the field to the 64-bit sort
        H, W = 400, 400
        TG = cone(H, W, 200, 200, rng, 0.3) + 1.0
        yy, xx = np.mgrid[0:H, 0:W]
        patch = (np.abs(xx - 200) < 160) & (np.abs(yy - 200) < 160)
        TG[patch] = 2.0 ** -500 * (1.0 + cone(H, W, 200, 200, rng, 0.9)[patch])
        TG[200, 200] = 0.0
        TS = cone(H, W, 8, 12, rng, 0.3)
    elif case == "large":
        H, W = 2048, 1536
        TG, TS = cone(H, W, 1400, 1800, rng, 0.4, 1.3), cone(H, W, 100, 200, rng, 0.4)
        blk = rng.random((H, W)) < 0.05
        blk[1800, 1400] = blk[200, 100] = False
        TG[blk] = TS[blk] = np.inf
    else:
        raise KeyError(case)
    return TG, TS


CASES = ["smooth", "obstacles", "ties", "manhattan", "lopsided", "corridor", "same_source", "float_ties",
         "zero_cost_patch", "large"]


@pytest.mark.parametrize("case", CASES)
def test_join_matches_definition(ctx, case):
    rng = np.random.default_rng(CASES.index(case))
    TG, TS = make(case, rng)
    gp, sp, join, members = ctx.bidir_join(TG, TS)
    rgp, rsp, rjoin, k = join_oracle(TG, TS)
    assert np.array_equal(join, rjoin), (case, join, rjoin)
    assert np.array_equal(gp, rgp) and np.array_equal(sp, rsp)
    n_fin = int(np.isfinite(TG).sum()), int(np.isfinite(TS).sum())
    for f in range(2):
        assert k + 1 <= members[f] <= n_fin[f], (case, k, members, n_fin)
    print(f"{case}: k* {k}, members {members.tolist()} of {TG.size} cells")


def test_join_disjoint_fields_raise(ctx):
    import eikonal

    TG = np.full((64, 80), np.inf)
    TS = np.full((64, 80), np.inf)
    TG[:, :40] = 1.0
    TS[:, 40:] = 1.0
    with pytest.raises(eikonal.EikError):
        ctx.bidir_join(TG, TS)


def test_join_members_bounded_on_terrain(ctx):
    """On real fronts (the solver's own fields of a random-cost raster) the ranked set stays a
    fraction of the raster: the bound is what makes the join cheaper than sorting the raster."""
    rng = np.random.default_rng(11)
    H = W = 1024
    cost = rng.uniform(1, 4, (H, W))
    cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
    goal, start = (700, 650), (300, 380)
    TG = ctx.tmap2d(cost, goal, dtype=np.float64)
    TS = ctx.tmap2d(cost, start, dtype=np.float64)
    gp, sp, join, members = ctx.bidir_join(TG, TS)
    rgp, rsp, rjoin, k = join_oracle(TG, TS)
    assert np.array_equal(join, rjoin) and np.array_equal(gp, rgp) and np.array_equal(sp, rsp)
    assert members.max() <= 0.5 * H * W, members


# ---- capped fronts (eikonal_api.cpp solve_fronts): biComputeTmap on rasters of >= 2^20 cells
# solves each front only up to a cap estimated on a coarse copy; the result must be the full
# fronts' (the FIM is not bit-deterministic between two schedules: fields within 1e-9, and the
# join and masks equal)
def _raster(kind, rng):
    H = W = 1024
    cost = rng.uniform(1, 4, (H, W))
    if kind == "wall_gap":  # a one-cell wall with a 3-cell gap: invisible to the 4 x 4 coarse blocks
        cost[:, 500] = np.inf
        cost[700:703, 500] = 1.0
    elif kind == "obstacles":
        cost[rng.random((H, W)) < 0.15] = np.inf
    elif kind == "blocky":  # large impassable blocks and a high-cost band
        cost[200:800, 300:340] = np.inf
        cost[100:900, 600:620] = 300.0
    cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
    return cost


FRONT_CASES = [("uniform_far", (900, 880), (60, 50)), ("uniform_near", (520, 500), (480, 530)),
               ("wall_gap", (900, 100), (100, 900)), ("obstacles", (800, 700), (150, 200)),
               ("blocky", (950, 500), (50, 500)), ("same_node", (400, 400), (400, 400))]


@pytest.fixture(scope="module")
def ctx_full():
    import eikonal

    c = eikonal.Context(0, options="FRONTS_CAP=0")
    yield c
    c.close()


@pytest.mark.parametrize("kind,goal,start", FRONT_CASES, ids=[c[0] for c in FRONT_CASES])
def test_capped_fronts_equal_full_fronts(ctx, ctx_full, kind, goal, start):
    rng = np.random.default_rng(100 + [c[0] for c in FRONT_CASES].index(kind))
    cost = _raster(kind.split("_")[0] if kind.startswith("uniform") else kind, rng)
    if kind == "obstacles":
        cost[goal[1], goal[0]] = cost[start[1], start[0]] = 1.0
    TG, TS, join = ctx.tmap2d_bidir(cost, goal, start)
    info = ctx.fronts_info()
    FG, FS, fjoin = ctx_full.tmap2d_bidir(cost, goal, start)
    assert not ctx_full.fronts_info()["capped"]
    assert np.array_equal(join, fjoin), (kind, join, fjoin, info)
    for a, b in ((TG, FG), (TS, FS)):
        assert np.array_equal(np.isfinite(a), np.isfinite(b)), (kind, info)
        f = np.isfinite(a)
        assert np.abs(a[f] - b[f]).max() <= 1e-9, kind
    print(f"{kind}: {info}, finite cells {int(np.isfinite(TG).sum())} / {int(np.isfinite(TS).sum())}")
    if kind in ("uniform_far", "uniform_near", "same_node"):
        assert info["capped"] and not info["fallback"], info
        assert max(info["kept"]) < cost.size, info


def test_capped_fronts_disconnected(ctx):
    import eikonal

    cost = np.ones((1024, 1024))
    cost[:, 512] = np.inf
    with pytest.raises(eikonal.EikError):
        ctx.tmap2d_bidir(cost, (100, 100), (900, 900))
