"""GPU parity of the path-extraction kernel (getPathGDM, FastMarching.py:164-236), the full-field
gradient (computeGradient, :242-300) and the bidirectional drop-in (biComputeTmap, :114-162).

Path tolerance on the SAME fp64 field: identical length and exit status, pointwise <= 1e-9
cells.  (The reference squares numpy scalars with `x**2` -> glibc pow(), not always correctly
rounded; the kernel uses exact products, so bit-identity is not claimed -- the oracle, which
does call pow(), is bit-exact to the reference.)
Bidirectional: the GPU returns FULL goal/start fields and the join from their pop ranks; the
rover path (planner glue, Coupled_motion_planner.py:1229-1232) must stay within a Hausdorff
distance of 3 cells of the reference's.
"""
import numpy as np
import pytest

import oracle as O
from band import BAND_BRACKET, band_ratio

pytestmark = pytest.mark.gpu
PATH_ATOL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    import eikonal

    c = eikonal.Context(0)
    yield c
    c.close()


def _f(a):
    return np.asarray(a, np.float64)


@pytest.mark.parametrize("i", range(12))
def test_path_on_golden_field(ctx, golden, i):
    d = golden("fmm2d_fields")
    p = f"c{i}_"
    path, st = ctx.path2d(d[p + "T"], _f(d[p + "start"]), _f(d[p + "goal"]), 0.5)
    ref = d[p + "path"]
    _, ost = O.gdm2d(d[p + "T"], _f(d[p + "start"]), _f(d[p + "goal"]), 0.5)
    assert st == ost
    assert path.shape == ref.shape
    assert np.abs(path - ref).max() <= PATH_ATOL


@pytest.mark.parametrize("i", range(6))
def test_path_on_golden_bidir_fields(ctx, golden, i):
    d = golden("fmm2d_bidir")
    p = f"b{i}_"
    for fld, end, key in (("TG", "goal", "pathG"), ("TS", "start", "pathS")):
        path, _ = ctx.path2d(d[p + fld], _f(d[p + "join"]), _f(d[p + end]), 0.5)
        ref = d[p + key]
        assert path.shape == ref.shape and np.abs(path - ref).max() <= PATH_ATOL


def test_gradient_full_field(ctx, golden):
    h = golden("helpers")
    gx, gy = ctx.gradient2d(h["grad_T"])
    for g, r in ((gx, h["grad_nx"]), (gy, h["grad_ny"])):
        assert np.array_equal(np.isnan(g), np.isnan(r))
        m = ~np.isnan(r)
        assert np.abs(g[m] - r[m]).max() <= 1e-15


def hausdorff(a, b):
    d = np.sqrt(((a[:, None, :] - b[None, :, :]) ** 2).sum(-1))
    return max(d.min(1).max(), d.min(0).max())


@pytest.mark.parametrize("i", range(6))
def test_bidirectional(ctx, golden, i):
    """biComputeTmap (FastMarching.py:114-162) and the planner's two descents from nodeJoin
    (Coupled_motion_planner.py:1225-1232) against the reference's own outputs: nodeJoin, the
    fronts' PARTIAL fields (finite masks; closed values equal, band values at their final value,
    bracketed GPU <= reference <= 1.03 x GPU) and the rover path, truncated or not, as the
    reference returns it.  Maps with exact ties of T (uniform, b0/b1): the reference pops ties
    LIFO, the default mode by node index, so a few tied cells at the fronts' edges may differ
    (EIK_OPT_EXACT_BAND removes both tolerances: tests/test_gpu_bidir_exact.py)."""
    d = golden("fmm2d_bidir")
    p = f"b{i}_"
    ties = i < 2
    cost = d[p + "cost"].astype(np.float64)
    goal, start = d[p + "goal"], d[p + "start"]
    TG, TS, join = ctx.tmap2d_bidir(cost, goal, start)
    assert join.dtype == np.uint32
    if ties:
        assert np.abs(join.astype(int) - d[p + "join"].astype(int)).max() <= 2
    else:
        assert np.array_equal(join, d[p + "join"])
    for T, R in ((TG, d[p + "TG"]), (TS, d[p + "TS"])):
        assert int((np.isfinite(T) != np.isfinite(R)).sum()) <= (4 if ties else 0)
        f = np.isfinite(T) & np.isfinite(R)
        assert np.all(T[f] <= R[f] + 1e-9)
        r = band_ratio(T, R, f)
        assert r <= BAND_BRACKET, f"band: reference / GPU up to {r:.4f} (bracket {BAND_BRACKET})"
    pg, sg = ctx.path2d(TG, _f(join), _f(goal))
    ps, ss = ctx.path2d(TS, _f(join), _f(start))
    for got, st, key in ((pg, sg, "pathG"), (ps, ss, "pathS")):
        ref = d[p + key]
        _, rst = O.gdm2d(d[p + ("TG" if key == "pathG" else "TS")], _f(d[p + "join"]),
                         _f(goal if key == "pathG" else start))
        assert st == rst, (key, st, rst)  # b4: the reference's start-side walk is truncated (numpy-2 fallback)
        assert got.shape == ref.shape and np.abs(got - ref).max() <= 0.01, (key, got.shape, ref.shape)
    rover = np.vstack((np.flipud(ps), pg[1:]))
    ref = np.vstack((np.flipud(d[p + "pathS"]), d[p + "pathG"][1:]))
    assert hausdorff(rover, ref) <= 0.01


def test_path_device_fp32_field(ctx):
    """eik_path2d_dev on a device-resident fp32 field (the bench's ms-to-path route)."""
    import ctypes
    import torch

    import eikonal
    from eikonal import _lib as L

    rng = np.random.default_rng(4)
    cost = rng.uniform(1, 3, (300, 340)).astype(np.float32)
    cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
    goal, start = (250, 200), (30, 40)
    T64 = ctx.tmap2d(cost.astype(np.float64), goal, dtype=np.float64)
    ref, rst = ctx.path2d(T64, start, goal)
    dev = torch.device("cuda", 0)
    T = torch.from_numpy(T64.astype(np.float32)).to(dev)
    cap = 30004
    out = torch.empty((cap, 2), dtype=torch.float64, device=dev)
    n = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    ctx._chk(L.lib().eik_path2d_dev(ctx._h, T.data_ptr(), L.EIK_F32, 300, 340, np.array(start, np.float64),
                                    np.array(goal, np.float64), 0.5, out.data_ptr(), cap, n.data_ptr(),
                                    st.data_ptr(), s.cuda_stream))
    k = int(n.item())
    path = out[:k].cpu().numpy()
    assert k == len(ref) and int(st.item()) == rst
    assert np.abs(path - ref).max() < 1e-3  # fp32 field vs fp64 field (BASELINE.md path tolerance)


def _walker_fields():
    """Fields for the walker-loop check: the golden fields (ties, obstacles, NaN
    fallbacks), a large smooth field (many windows), a V-shaped valley (interpolated gradients
    cancel: |g| < 0.01 unit steps, tiny operands) and fields with obstacles."""
    import oracle as O2

    out = []
    rng = np.random.default_rng(21)
    for H, W, p_inf in ((1500, 1700, 0.0), (600, 500, 0.08), (300, 900, 0.2)):
        cost = rng.uniform(1, 6, (H, W))
        cost[rng.random((H, W)) < p_inf] = np.inf
        cost[0, :] = cost[-1, :] = cost[:, 0] = cost[:, -1] = np.inf
        goal = (W - 40, H - 30)
        cost[goal[1], goal[0]] = 1.0
        O2.set_strict(False)
        out.append((O2.fmm2d(cost, goal), (25.3, 31.7), goal))
    yy, xx = np.mgrid[0:400, 0:400].astype(np.float64)
    valley = np.abs(xx - 200.0) * 3 + (399 - yy)  # descent runs into the x = 200 crease
    out.append((valley, (37.5, 12.25), (200.0, 395.0)))
    return out


@pytest.mark.parametrize("form", [1, 2, 3, 4])
@pytest.mark.parametrize("tau", [0.5, 1.7])
def test_walker_loop_forms_bit_identical(golden, tau, form):
    """EIK_OPT_PATH_LOOP: the single-exit step loop (1), that loop with the range-free f64
    sqrt / division (2, gdm.hip sqrt_core / div_core) and with the divisions taken from the square
    roots' reciprocals (3, div_rs) and that arithmetic on lane pairs (4: x on even lanes, y on odd)
    return the SAME bits as the loop in the
    reference's statement order (0) (array_equal, same status) -- on the golden fields and on
    fields that exercise window switches, NaN fallbacks, |g| < 0.01 unit steps and, at tau = 1.7,
    points that move more than one cell per step (the walker's slow path)."""
    import eikonal
    from eikonal import _lib as L

    cases = []
    d = golden("fmm2d_fields")
    for i in range(12):
        p = f"c{i}_"
        cases.append((d[p + "T"], _f(d[p + "start"]), _f(d[p + "goal"])))
    cases += _walker_fields()
    c0, c1 = eikonal.Context(0), eikonal.Context(0)
    try:
        c0.set_option(L.OPT_PATH_LOOP, 0)
        c1.set_option(L.OPT_PATH_LOOP, form)
        for T, s, g in cases:
            a, sa = c0.path2d(T, _f(s), _f(g), tau)
            b, sb = c1.path2d(T, _f(s), _f(g), tau)
            assert sa == sb and a.shape == b.shape and np.array_equal(a, b)
    finally:
        c0.close()
        c1.close()


def test_walker_fast_math_exact():
    """The 2D walker's fast-path arithmetic (gdm.hip sqrt_core, div_core, div_rs, interp2_general) equals
    the exact forms it replaces -- the correctly rounded f64 sqrt and division and interpolatePoint's
    special cases (FastMarching.py:327-336) -- bit for bit (a zero quotient up to its sign) on 4M
    pseudo-random inputs each from the domain the walker uses them on (walk_odd false)."""
    import eikonal
    from eikonal import _lib as L

    c = eikonal.Context(0)
    try:
        for seed in (1, 0x9E3779B97F4A7C15):
            counts = np.zeros(6, np.int64)
            c._chk(L.lib().eik_selftest_walker_math(c._h, 1 << 22, seed, counts))
            assert counts.tolist() == [0, 0, 0, 1 << 22, 0, 0], counts
        counts = np.zeros(6, np.int64)  # the one-correction square root and div_rs: 2^28 samples
        c._chk(L.lib().eik_selftest_walker_math(c._h, 1 << 28, 77, counts))
        assert counts[[0, 1, 2, 4, 5]].tolist() == [0, 0, 0, 0, 0] and counts[3] == 1 << 28, counts
    finally:
        c.close()


def test_pinned_results_round_trip(ctx):
    """Fields of >= 16 MiB come back in recycled page-locked blocks (eikonal._lib.result_empty) and
    cross PCIe as one DMA each way: the field and the path from it equal the pageable route's
    (a plain copy of the same field), and blocks are reused after the arrays are gone."""
    from eikonal import _lib as L

    rng = np.random.default_rng(12)
    N = 1536  # 18 MiB of float64
    cost = rng.uniform(1, 4, (N, N))
    cost[rng.random((N, N)) < 0.05] = np.inf
    goal, start = (N // 2, N // 3), (40, N - 60)
    cost[goal[1], goal[0]] = cost[start[1], start[0]] = 1.0
    T = ctx.tmap2d(cost, goal)
    assert T.nbytes >= L.PINNED_MIN_BYTES and T.flags.c_contiguous and T.flags.writeable
    Tp = np.array(T, copy=True)  # pageable
    assert np.array_equal(T, Tp, equal_nan=True)
    p1, s1 = ctx.path2d(T, start, goal)
    p2, s2 = ctx.path2d(Tp, start, goal)
    assert s1 == s2 and np.array_equal(p1, p2)
    n_free = sum(len(v) for v in L._pin_free.values())
    del T
    assert sum(len(v) for v in L._pin_free.values()) == n_free + 1  # back in the pool
    T2 = ctx.tmap2d(cost, goal)  # reuses it (a second solve: equal up to the fp64 rounding of its schedule)
    fin = np.isfinite(Tp)
    assert np.array_equal(np.isfinite(T2), fin) and np.abs(T2[fin] - Tp[fin]).max() <= 1e-9


@pytest.mark.parametrize("form", [2, 4])
def test_walker_forms_budget_and_stop_edges(form):
    """The lane-pair loop's own exits against the reference-order loop (form 0), bit for bit with the
    same point count and status: point budgets that end the walk mid-way (cap 2, 3, 50, 1001: the
    loop's 32-bit budget count), starts inside and just outside the stop radius (the safe-step count
    is 0 or a few steps), a large and a tiny tau, and a start on a NaN point."""
    import torch

    import eikonal
    from eikonal import _lib as L

    (T, _, goal), = _walker_fields()[:1]
    dev = torch.device("cuda", 0)
    Td = torch.from_numpy(np.ascontiguousarray(T)).to(dev)
    H, W = T.shape
    g = np.array(goal, np.float64)
    cases = [((25.3, 31.7), 0.5, cap) for cap in (2, 3, 50, 1001)]
    cases += [((goal[0] + 1.0, goal[1] + 0.5), 0.5, 30004), ((goal[0] + 1.6, goal[1]), 0.5, 30004),
              ((goal[0] - 2.9, goal[1] + 2.9), 0.5, 30004), ((400.5, 300.25), 2.3, 30004),
              ((400.5, 300.25), 1e-3, 3000), ((float("nan"), 300.0), 0.5, 100)]
    res = {}
    for f in (0, form):
        c = eikonal.Context(0)
        try:
            c.set_option(L.OPT_PATH_LOOP, f)
            s = torch.cuda.current_stream(dev)
            for q, (start, tau, cap) in enumerate(cases):
                out = torch.full((cap, 2), -7.0, dtype=torch.float64, device=dev)
                n = torch.zeros(1, dtype=torch.int64, device=dev)
                st = torch.zeros(1, dtype=torch.int32, device=dev)
                c._chk(L.lib().eik_path2d_dev(c._h, Td.data_ptr(), L.EIK_F64, H, W, np.array(start, np.float64), g,
                                              tau, out.data_ptr(), cap, n.data_ptr(), st.data_ptr(), s.cuda_stream))
                k = int(n.item())
                res.setdefault(q, []).append((k, int(st.item()), out[:k].cpu().numpy()))
        finally:
            c.close()
    for q, ((k0, s0, p0), (k1, s1, p1)) in res.items():
        assert (k0, s0) == (k1, s1), (cases[q], k0, s0, k1, s1)
        assert np.array_equal(p0, p1, equal_nan=True), cases[q]
