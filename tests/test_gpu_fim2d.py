"""GPU parity of the HIP block-FIM (libeikonal, through the C ABI) against the oracle.

Tolerances (BASELINE.md "Parity tolerance"):
  * reachability masks (isfinite) identical, T[goal] == 0;
  * fp32 field: max relative error <= 2e-5 over finite cells;
  * fp64 field: max absolute error <= 1e-9.
The golden fields were produced by the reference FastMarching.py itself (tests/golden/); larger
maps are checked against the C oracle (bit-exact restatement of the reference, pinned by
tests/test_oracle_golden.py).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

RTOL32 = 2e-5
ATOL64 = 1e-9


@pytest.fixture(scope="module", params=["persistent", "list"])
def ctx(request):
    """Both solver drivers: one persistent launch over the device FIFO (default), and one
    launch per outer iteration over the active list."""
    import eikonal
    from eikonal import _lib as L

    c = eikonal.Context(0)
    c.set_option(L.OPT_MODE, L.MODE_PERSISTENT if request.param == "persistent" else L.MODE_LIST)
    yield c
    c.close()


def check_field(T, R, goal, f64):
    assert T.shape == R.shape
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin), "reachability mask differs"
    assert T[goal[1], goal[0]] == 0
    if not fin.any():
        return
    err = np.abs(T[fin].astype(np.float64) - R[fin])
    if f64:
        assert err.max() <= ATOL64, err.max()
    else:
        rel = err / np.maximum(np.abs(R[fin]), 1e-30)
        rel[R[fin] == 0] = err[R[fin] == 0]
        assert rel.max() <= RTOL32, rel.max()


def oracle_field(cost, goal):
    O.set_strict(False)  # intended semantics (no StopIteration on tied decrease-keys)
    try:
        return O.fmm2d(np.asarray(cost, np.float64), goal)
    finally:
        O.set_strict(True)


@pytest.mark.parametrize("i", range(13))
@pytest.mark.parametrize("f64", [False, True])
def test_golden_fields(ctx, golden, i, f64):
    d = golden("fmm2d_fields")
    p = f"c{i}_"
    cost = d[p + "cost"].astype(np.float64)
    goal = d[p + "goal"]
    R = d[p + "T"] if not str(d[p + "err"]) else oracle_field(cost, goal)  # blobs_ties: ref raised
    T = ctx.tmap2d(cost, goal, dtype=np.float64 if f64 else np.float32)
    check_field(T, R, goal, f64)


@pytest.mark.parametrize("name", ["uniform", "random"])
@pytest.mark.parametrize("f64", [False, True])
def test_c1_config(ctx, golden, name, f64):
    """BASELINE configs[0] (C1): 256^2 uniform / U(1, 10) seed 0, goal (128, 128) -- the field
    against the reference's own (tests/golden/c1.npz) and, end to end on the GPU (its field, its
    path kernel), the reference's getPathGDM path from (30, 40)."""
    d = golden("c1")
    cost = d[name + "_cost"].astype(np.float64)
    goal, start = d["goal"], d["start"]
    T = ctx.tmap2d(cost, goal, dtype=np.float64 if f64 else np.float32)
    check_field(T, d[name + "_T"], goal, f64)
    if f64:
        path, st = ctx.path2d(T, start.astype(np.float64), goal.astype(np.float64))
        ref = d[name + "_path"]
        assert st == 0 and path.shape == ref.shape and np.abs(path - ref).max() <= 1e-6


@pytest.mark.parametrize("shape,kind,seed", [
    ((517, 1031), "obst", 1),      # ragged: neither side a multiple of the 64-cell tile
    ((1024, 1024), "random", 2),
    ((300, 70), "maze", 3),        # long winding front: many outer iterations
    ((64, 64), "random", 4),       # exactly one tile
    ((1, 200), "random", 5),       # degenerate strip
    ((37, 1), "random", 6),
    ((2048, 2048), "blobs", 7),
])
def test_vs_oracle(ctx, shape, kind, seed):
    rng = np.random.default_rng(seed)
    H, W = shape
    c = rng.uniform(1, 10, shape)
    if kind == "obst":
        c[rng.random(shape) < 0.15] = np.inf
    elif kind == "maze":
        for x in range(4, W - 2, 8):  # walls with alternating gaps
            c[:, x] = np.inf
            gap = 2 if (x // 8) % 2 == 0 else H - 3
            c[gap, x] = 3.0
    elif kind == "blobs":
        yy, xx = np.mgrid[0:H, 0:W]
        for _ in range(40):
            cy, cx, r = rng.integers(0, H), rng.integers(0, W), rng.integers(10, 80)
            c[(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 300.0
    c = c.astype(np.float32).astype(np.float64)
    goal = [W // 3, H // 2] if W > 1 else [0, H // 2]
    c[goal[1], goal[0]] = 1.0
    R = oracle_field(c, goal)
    check_field(ctx.tmap2d(c, goal, dtype=np.float32), R, goal, False)
    if H * W <= 1 << 20:
        check_field(ctx.tmap2d(c, goal, dtype=np.float64), R, goal, True)


def test_enclosed_goal_and_unreachable(ctx):
    c = np.full((90, 130), 2.0)
    c[40:50, 60] = c[40:50, 70] = np.inf
    c[40, 60:71] = c[49, 60:71] = np.inf  # goal boxed in
    goal = [65, 45]
    T = ctx.tmap2d(c, goal, dtype=np.float32)
    R = oracle_field(c, goal)
    check_field(T, R, goal, False)
    assert np.isfinite(T).sum() == np.isfinite(R).sum() == 8 * 9


def test_non_inf_border_matches_oob_as_inf(ctx):
    rng = np.random.default_rng(11)
    c = rng.uniform(0.5, 3, (150, 160))  # no inf border: out-of-range reads as +inf
    check_field(ctx.tmap2d(c, [0, 0], dtype=np.float32), oracle_field(c, [0, 0]), [0, 0], False)


def test_zero_cost_cells(ctx):
    c = np.ones((80, 80))
    c[30:50, 30:50] = 0.0  # free region: T constant across it
    check_field(ctx.tmap2d(c, [40, 40], dtype=np.float64), oracle_field(c, [40, 40]), [40, 40], True)


def test_bad_inputs_raise(ctx):
    import eikonal

    c = np.ones((10, 10))
    with pytest.raises(eikonal.EikError):
        ctx.tmap2d(c, [10, 3])  # goal outside
    c[3, 3] = -1.0
    with pytest.raises(eikonal.EikError):
        ctx.tmap2d(c, [1, 1])  # negative cost rejected (reference semantics undefined)
    c[3, 3] = np.nan
    with pytest.raises(eikonal.EikError):
        ctx.tmap2d(c, [1, 1])


def test_bad_cost_reports_first_index(ctx):
    """The cost check runs on the device copy (one kernel, an 8-byte read-back) in every host
    entry that takes a cost array: EIK_ERR_ARG naming the FIRST bad index and its value, and the
    context stays usable afterwards."""
    import eikonal
    from eikonal import _lib as L

    rng = np.random.default_rng(3)
    c = rng.uniform(1, 2, (300, 500))
    c[250, 7] = -2.0
    c[41, 333] = np.nan  # first in row-major order: 41 * 500 + 333
    c[200, 100] = -0.5
    want = f"cost[{41 * 500 + 333}] = nan"
    calls = [lambda: ctx.tmap2d(c, [1, 1]), lambda: ctx.tmap2d(c.astype(np.float32), [1, 1], dtype=np.float32),
             lambda: ctx.tmap2d_batch(np.stack([np.ones_like(c), c]), [[1, 1], [2, 2]]),
             lambda: ctx.tmap2d_bidir(c, [1, 1], [400, 290]),
             lambda: ctx.tmap3d(c.reshape(300, 50, 10), [1, 1, 1]),
             lambda: ctx.tmap3d_batch(c.reshape(1, 300, 50, 10), [[1, 1, 1]])]
    for k, call in enumerate(calls):
        with pytest.raises(eikonal.EikError) as e:
            call()
        assert e.value.code == L.EIK_ERR_ARG
        w = want if k != 2 else f"cost[{300 * 500 + 41 * 500 + 333}] = nan"
        assert w in str(e.value), (k, str(e.value))
    ok = np.ones((40, 60))
    T = ctx.tmap2d(ok, [0, 0])
    assert T[0, 0] == 0 and np.isfinite(T).all()


def test_batch_matches_single(ctx):
    rng = np.random.default_rng(5)
    B, H, W = 6, 190, 260
    costs = rng.uniform(1, 8, (B, H, W)).astype(np.float32)
    costs[:, rng.random((H, W)) < 0.1] = np.inf
    goals = np.array([[rng.integers(0, W), rng.integers(0, H)] for _ in range(B)], np.int64)
    for b in range(B):
        costs[b, goals[b, 1], goals[b, 0]] = 1.0
    T = ctx.tmap2d_batch(costs, goals)
    for b in range(B):
        check_field(T[b], oracle_field(costs[b], goals[b]), goals[b], False)


def test_repeatable(ctx):
    """Monotone min-updates: racing sweeps may differ only in the last bits between runs."""
    rng = np.random.default_rng(9)
    c = rng.uniform(1, 10, (700, 900)).astype(np.float32)
    a = ctx.tmap2d(c, [450, 350], dtype=np.float32)
    b = ctx.tmap2d(c, [450, 350], dtype=np.float32)
    fin = np.isfinite(a)
    assert np.array_equal(fin, np.isfinite(b))
    assert (np.abs(a[fin] - b[fin]) / np.maximum(a[fin], 1e-30)).max() <= 1e-5


def test_stats_count_visits(ctx):
    c = np.ones((512, 512), np.float32)
    ctx.tmap2d(c, [256, 256], dtype=np.float32)
    s = ctx.stats()
    assert s["tile_visits"] >= 64 and s["iterations"] >= 1 and s["solve_ms"] > 0


@pytest.mark.parametrize("shape,f64", [((512, 512), False), ((512, 512), True), ((300, 500), True)])
def test_fresh_visits_read_no_T(ctx, shape, f64):
    """A persistent visit of a full tile nobody has written yet stages only the cost (fim2d.hip
    kFreshSkip): on a uniform raster every full tile but the goal's is first visited that way,
    exactly once, and the byte model leaves out their T reads.  (List mode always reads T.)"""
    from eikonal import _lib as L
    H, W = shape
    dt = np.float64 if f64 else np.float32
    c = np.ones(shape, dt)
    goal = [256, 256]
    T = ctx.tmap2d(c, goal, dtype=dt)
    s = ctx.stats()
    persistent = s["iterations"] == 1
    full = (H // 64) * (W // 64)
    goal_full = goal[1] // 64 < H // 64 and goal[0] // 64 < W // 64
    assert s["fresh_visits"] == ((full - goal_full) if persistent else 0)
    esz = 8 if f64 else 4
    alg = esz * (s["tile_visits"] * (3 * 4096 + 256) - s["fresh_visits"] * 4096 + s["inplace_passes"] * (4096 + 256)
                 + H * W)
    assert s["bytes_alg"] == alg
    check_field(T, oracle_field(c, goal), goal, f64)


@pytest.mark.parametrize("passes", [1, 2, 8, 16])
def test_pass_cap_option(passes):
    """EIK_OPT_PASSES (in-place passes per persistent visit) changes the schedule, not the field:
    a single map and a batch against the oracle at caps other than the defaults (24 for a single
    map -- 16 for one of >= 16384 tiles --, 2 for a batch; 2 is also run here on the single map and
    1 / 16 on the batch)."""
    import eikonal
    from eikonal import _lib as L

    c = eikonal.Context(0)
    try:
        c.set_option(L.OPT_PASSES, passes)
        rng = np.random.default_rng(11)
        cost = rng.uniform(1, 10, (700, 900))
        cost[rng.random(cost.shape) < 0.12] = np.inf
        cost = cost.astype(np.float32).astype(np.float64)
        goal = [300, 350]
        cost[goal[1], goal[0]] = 1.0
        check_field(c.tmap2d(cost, goal, dtype=np.float32), oracle_field(cost, goal), goal, False)
        costs = rng.uniform(1, 8, (4, 150, 210)).astype(np.float32)
        goals = np.array([[20, 30], [200, 140], [100, 75], [5, 149]], np.int64)
        for b in range(4):
            costs[b, goals[b, 1], goals[b, 0]] = 1.0
        T = c.tmap2d_batch(costs, goals)
        for b in range(4):
            check_field(T[b], oracle_field(costs[b], goals[b]), goals[b], False)
    finally:
        c.close()


@pytest.mark.parametrize("opts", [(("SCHED", 0),), (("SCHED", 2),), (("SCHED", 3),), (("FRESH_FIRST", 1),),
                                  (("SCHED", 0), ("FRESH_FIRST", 1)), (("PRIO", 0.1),), (("PRIO", 1),),
                                  (("PRIO", 1e4),), (("PRIO", 1), ("SCHED", 0)),
                                  (("PRIO", 0.1), ("PRIO_DISPATCH", 128)), (("PRIO", 1), ("PRIO_DISPATCH", 100))])
def test_schedule_options(opts):
    """The queue-scheduling options (EIK_OPT_SCHED other than the default 1, EIK_OPT_FRESH_FIRST, the
    priority bands and their dispatch batch past 64 entries -- two per lane, fim_engine.hpp band_dispatch)
    change the order of tile visits, never the fixed point: single map and batch vs the oracle."""
    import eikonal
    from eikonal import _lib as L

    c = eikonal.Context(0)
    try:
        for name, v in opts:
            c.set_option(getattr(L, "OPT_" + name), v)
        rng = np.random.default_rng(12)
        cost = rng.uniform(1, 10, (640, 770))
        cost[rng.random(cost.shape) < 0.15] = np.inf
        cost = cost.astype(np.float32).astype(np.float64)
        goal = [500, 120]
        cost[goal[1], goal[0]] = 1.0
        check_field(c.tmap2d(cost, goal, dtype=np.float32), oracle_field(cost, goal), goal, False)
        costs = rng.uniform(1, 8, (3, 130, 260)).astype(np.float32)
        goals = np.array([[3, 4], [250, 120], [128, 64]], np.int64)
        for b in range(3):
            costs[b, goals[b, 1], goals[b, 0]] = 1.0
        T = c.tmap2d_batch(costs, goals)
        for b in range(3):
            check_field(T[b], oracle_field(costs[b], goals[b]), goals[b], False)
    finally:
        c.close()


@pytest.mark.parametrize("neg", [False, True])
def test_visit_budget_device_buffers(neg):
    """EIK_OPT_MAX_VISITS on the device-buffer entry (eik_fim2d_solve: no host-side cost check).
    In-place passes are charged to the budget like full visits, so a single-map solve (24 passes
    per visit by default) whose workgroups never reach 64 full visits each still stops with
    EIK_ERR_NOCONVERGE.  neg: a negative-cost block (reference semantics undefined) must end in
    NOCONVERGE or a finished solve -- never a hang (the test's own timeout)."""
    import torch
    import eikonal
    from eikonal import _lib as L

    rng = np.random.default_rng(3)
    cost = rng.uniform(1, 10, (1024, 1024)).astype(np.float32)
    cost[rng.random(cost.shape) < 0.15] = np.inf
    if neg:
        cost[400:600, 400:600] = -2.0
    goal = np.array([[512, 300]], np.int64)
    cost[300, 512] = 1.0
    c = eikonal.Context(0)
    try:
        c.set_option(L.OPT_MAX_VISITS, 128)
        dev = torch.device("cuda", 0)
        cd = torch.from_numpy(cost).to(dev)
        Td = torch.empty_like(cd)
        f = L.Fim2d(c, 1, 1024, 1024, L.EIK_F32)
        try:
            if neg:
                try:
                    f.solve(cd.data_ptr(), Td.data_ptr(), goal, torch.cuda.current_stream(dev).cuda_stream)
                except eikonal.EikError as e:
                    assert e.code == L.EIK_ERR_NOCONVERGE, e
            else:
                with pytest.raises(eikonal.EikError) as ei:
                    f.solve(cd.data_ptr(), Td.data_ptr(), goal, torch.cuda.current_stream(dev).cuda_stream)
                assert ei.value.code == L.EIK_ERR_NOCONVERGE
            # the context stays usable: default budget, same map, solves
            c.set_option(L.OPT_MAX_VISITS, 0)
            if not neg:
                f.solve(cd.data_ptr(), Td.data_ptr(), goal, torch.cuda.current_stream(dev).cuda_stream)
                torch.cuda.synchronize()
                check_field(Td.cpu().numpy(), oracle_field(cost, goal[0]), goal[0], False)
        finally:
            f.close()
    finally:
        c.close()


@pytest.mark.parametrize("delta", [0.02, 1.0, 20.0])
@pytest.mark.parametrize("kind", ["maze", "blobs", "obst"])
def test_priority_bands_fp64(kind, delta):
    """EIK_OPT_PRIO (priority bands, fim_engine.hpp): waiting tiles taken lowest entering T first,
    with second entries on a key drop and stale entries dropped at the claim -- a different visit
    order, the same fixed point: fp64 fields against the oracle (<= 1e-9), incl. a maze (keys far
    beyond the last band: the open-ended band is a FIFO) and band widths of a few cells' cost."""
    import eikonal
    from eikonal import _lib as L

    rng = np.random.default_rng(int(100 * delta) + len(kind))
    H, W = 777, 1100
    c = rng.uniform(1, 10, (H, W))
    if kind == "obst":
        c[rng.random((H, W)) < 0.2] = np.inf
    elif kind == "maze":
        for x in range(6, W - 2, 10):
            c[:, x] = np.inf
            c[3 if (x // 10) % 2 == 0 else H - 4, x] = 2.0
    else:
        yy, xx = np.mgrid[0:H, 0:W]
        for _ in range(30):
            cy, cx, r = rng.integers(0, H), rng.integers(0, W), rng.integers(10, 90)
            c[(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 300.0
    goal = [W // 2, H // 3]
    c[goal[1], goal[0]] = 1.0
    R = oracle_field(c, goal)
    fin = np.isfinite(R)
    ctx = eikonal.Context(0)
    try:
        errs = []
        for prio in (0.0, delta):  # the FIFO beside it: the same order of rounding differences
            ctx.set_option(L.OPT_PRIO, prio)
            T = ctx.tmap2d(c, goal, dtype=np.float64)
            assert np.array_equal(np.isfinite(T), fin) and T[goal[1], goal[0]] == 0
            errs.append(np.abs(T[fin] - R[fin]))
        # fp64 rounding of the device's step (eik_common.hpp EIK_CHAIN: one more rounding at T's
        # magnitude than the reference) accumulated along the maze's ~1e5-cell paths: 1e-9 absolute,
        # or 1e-13 relative where T is large (T ~ 5e5 there: 1e-9 would be 2e-15, a few ulps) -- the
        # FIFO solve measures 5.8e-14
        lim = np.maximum(1e-9, 1e-13 * R[fin])
        for name, e in zip(("fifo", "prio"), errs):
            assert (e <= lim).all(), (name, e.max(), (e / np.maximum(R[fin], 1)).max())
    finally:
        ctx.close()


def test_priority_band_ring_overflow_falls_back():
    """A priority band whose ring fills (EIK_OPT_PRIO_RING forced to 8 slots on a raster of ~200
    tiles) stops the launch with qerror bit 4 and eik_fim2d_solve solves again with the FIFO: the
    same field as a plain FIFO solve (<= 1e-9 / 1e-13 relative vs the oracle), no error raised."""
    import eikonal
    from eikonal import _lib as L

    rng = np.random.default_rng(77)
    H, W = 777, 1100
    c = rng.uniform(1, 10, (H, W))
    goal = [W // 3, H // 2]
    R = oracle_field(c, goal)
    fin = np.isfinite(R)
    ctx = eikonal.Context(0)
    try:
        ctx.set_option(L.OPT_PRIO, 1.0)
        ctx.set_option(L.OPT_PRIO_RING, 8)
        T = ctx.tmap2d(c, goal, dtype=np.float64)
        T2 = ctx.tmap2d(c, goal, dtype=np.float64)  # the same solver again: FIFO from the start
    finally:
        ctx.close()
    lim = np.maximum(1e-9, 1e-13 * R[fin])
    for X in (T, T2):
        assert np.array_equal(np.isfinite(X), fin)
        assert (np.abs(X[fin] - R[fin]) <= lim).all()
