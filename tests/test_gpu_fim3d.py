"""GPU parity of the 3D block-FIM (FastMarching3D.computeTmap :126-145) and the 3D path kernel
(FastMarching3D.getPathGDM :198-271) against reference-generated fixtures and the oracle.
Tolerances as in 2D: masks equal; fp64 <= 1e-9 abs; fp32 <= 2e-5 rel; paths <= 1e-9."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import eikonal

    c = eikonal.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_list():
    """The 3D solver's list driver (one launch per outer iteration); the default is persistent."""
    import eikonal
    from eikonal import _lib as L

    c = eikonal.Context(0, options={"MODE": L.MODE_LIST})
    yield c
    c.close()


def check(T, R, f64):
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin)
    err = np.abs(T[fin].astype(np.float64) - R[fin])
    if f64:
        assert err.max() <= 1e-9, err.max()
    else:
        assert (err / np.maximum(R[fin], 1e-30)).max() <= 2e-5


@pytest.mark.parametrize("i", range(4))
@pytest.mark.parametrize("f64", [False, True])
def test_golden_volumes(ctx, golden, i, f64):
    d = golden("fmm3d")
    p = f"v{i}_"
    cost = d[p + "cost"].astype(np.float64)
    T = ctx.tmap3d(cost, d[p + "goal"], dtype=np.float64 if f64 else np.float32)
    check(T, d[p + "T"], f64)
    # every node the early-exit reference closed (T <= T[start]) has the same value here
    Te = d[p + "T_early"]
    s = d[p + "start"]
    closed = np.isfinite(Te) & (Te <= Te[s[1], s[0], s[2]])
    if f64:
        assert np.abs(T[closed] - Te[closed]).max() <= 1e-9


@pytest.mark.parametrize("i", range(4))
def test_path3d(ctx, golden, i):
    d = golden("fmm3d")
    p = f"v{i}_"
    s, g = d[p + "start"].astype(float), d[p + "goal"].astype(float)
    path, st = ctx.path3d(d[p + "T_early"], s, g)
    ref = d[p + "path"]
    assert st == 0 and path.shape == ref.shape and np.abs(path - ref).max() <= 1e-9
    # end to end, layered and cube volumes alike: the GPU's early-exit field (computeTmap breaks
    # once `start` is popped, FastMarching3D.py:141) descended by the GPU path kernel
    assert str(d[p + "path_err"]) == ""
    T = ctx.tmap3d(d[p + "cost"].astype(np.float64), d[p + "goal"], dtype=np.float64, start=d[p + "start"])
    path2, _ = ctx.path3d(T, s, g)
    assert path2.shape == ref.shape and np.abs(path2 - ref).max() <= 1e-9


@pytest.mark.parametrize("driver", ["persistent", "list"])
@pytest.mark.parametrize("shape,seed", [((200, 230, 5), 1), ((40, 44, 36), 2), ((64, 64, 3), 3), ((33, 70, 9), 4)])
def test_vs_oracle(ctx, ctx_list, shape, seed, driver):
    ctx = ctx if driver == "persistent" else ctx_list
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 4, shape)
    c[rng.random(shape) < 0.08] = np.inf
    H, W, L = shape
    goal = np.array([W // 2, H // 3, L // 2])
    c[goal[1], goal[0], goal[2]] = 1.0
    O.set_strict(False)
    try:
        R = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    check(ctx.tmap3d(c, goal, dtype=np.float32), R, False)
    check(ctx.tmap3d(c, goal, dtype=np.float64), R, True)


# --- layered solver (fim2dl.hip): fp32 volumes with <= 4 layers, or z-padded with all-inf
# first/last layers (the reference's padding), go to the 2D-tile engine with per-cell layers.
def _layered_case(shape, seed, pad=False, switch=False):
    rng = np.random.default_rng(seed)
    H, W, L = shape
    c = rng.uniform(1, 4, shape)
    c[rng.random(shape) < 0.08] = np.inf
    if switch:  # layer 0 cheap on the left, layer 1 cheap on the right: paths change layer
        c[:, : W // 2, 0] *= 0.3
        c[:, W // 2 :, 1 % L] *= 0.3
    if pad:
        c = np.concatenate([np.full((H, W, 1), np.inf), c, np.full((H, W, 1), np.inf)], axis=2)
    goal = np.array([W // 3, H // 2, (1 if pad else 0) + (L - 1) // 2])
    c[goal[1], goal[0], goal[2]] = 1.0
    return c, goal


@pytest.mark.parametrize("shape,seed,pad,switch", [((130, 150, 2), 11, False, True), ((200, 230, 3), 12, False, False),
                                                     ((64, 64, 4), 13, False, True), ((90, 140, 3), 14, True, True),
                                                     ((300, 257, 3), 15, False, True), ((70, 65, 1), 16, False, False)])
def test_layered_vs_oracle(ctx, shape, seed, pad, switch):
    """fp32 (<= 4 layers, 64-row tiles) and fp64 (<= 3 layers, 40-row tiles; 4 layers go to fim3d)."""
    c, goal = _layered_case(shape, seed, pad, switch)
    O.set_strict(False)
    try:
        R = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    for f64 in (False, True):
        T = ctx.tmap3d(c, goal, dtype=np.float64 if f64 else np.float32)
        check(T, R, f64)
        if pad:
            assert np.all(np.isinf(T[:, :, 0])) and np.all(np.isinf(T[:, :, -1]))


@pytest.fixture(scope="module")
def ctx_volume():
    """The layered solver in the volume's own [y][x][L] layout (EIK_OPT_LAYER_PLANAR 0; the default
    solves on layer-planar copies of the solved layers)."""
    import eikonal

    c = eikonal.Context(0, options={"LAYER_PLANAR": 0})
    yield c
    c.close()


@pytest.mark.parametrize("opts", [{"PRIO": 0.0}, {"PRIO": 1.0}, {"PRIO": 0.05}, {"PRIO": 1.0, "LAYER_PLANAR": 0},
                                  {"PRIO": 1.0, "PRIO_RING": 8}])
@pytest.mark.parametrize("shape,seed,pad,switch", [((300, 257, 3), 15, False, True), ((90, 140, 3), 14, True, True),
                                                     ((64, 64, 4), 13, False, True)])
def test_layered_priority_bands(shape, seed, pad, switch, opts):
    """EIK_OPT_PRIO on the layered solver (fim2dl.hip: the entering keys of the write-back, the
    whole-wave band grab): a different visit order, the same fields against the oracle in both dtypes,
    incl. bands a few cells wide, the volume layout and a ring forced to overflow (qerror bit 4: the
    solve runs again on the FIFO, no error raised)."""
    import eikonal

    c, goal = _layered_case(shape, seed, pad, switch)
    O.set_strict(False)
    try:
        R = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    cx = eikonal.Context(0, options=opts)
    try:
        for f64 in (False, True):
            check(cx.tmap3d(c, goal, dtype=np.float64 if f64 else np.float32), R, f64)
    finally:
        cx.close()


@pytest.mark.parametrize("shape,seed,pad,switch", [((130, 150, 2), 11, False, True), ((90, 140, 3), 14, True, True),
                                                     ((300, 257, 3), 15, False, True), ((70, 65, 1), 16, False, False),
                                                     ((5, 3, 2), 42, False, False), ((39, 65, 3), 43, True, False)])
def test_layered_volume_layout_vs_oracle(ctx_volume, shape, seed, pad, switch):
    """EIK_OPT_LAYER_PLANAR 0: the solve in the volume's [y][x][L] layout (the default solves on
    [nl][H][W] copies, test_layered_vs_oracle) -- fields against the oracle in both dtypes."""
    c, goal = _layered_case(shape, seed, pad, switch)
    O.set_strict(False)
    try:
        R = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    for f64 in (False, True):
        T = ctx_volume.tmap3d(c, goal, dtype=np.float64 if f64 else np.float32)
        check(T, R, f64)
        if pad:
            assert np.all(np.isinf(T[:, :, 0])) and np.all(np.isinf(T[:, :, -1]))


@pytest.mark.parametrize("shape,seed", [((1, 1, 1), 41), ((5, 3, 2), 42), ((39, 65, 3), 43), ((41, 64, 1), 44),
                                        ((80, 129, 2), 45)])
def test_layered_edge_shapes(ctx, shape, seed):
    """Layered solver at the tile edges: volumes smaller than one tile, one row / column past a
    tile (fp64 tiles are 40 rows, fp32 64), a single cell; +inf islands and cheap cells (0.5; a zero
    cost has no reference result -- FastMarching3D.py:62-73 empties its list and raises -- and at
    costs << 1 the reference's 3-axis form (S + sqrt(nC^2 + S^2 - nQ))/n cancels: at C = 1e-3 and
    T ~ 100 its own error is ~1e-8, above the 1e-9 tolerance; the layered solver solves relative to
    the smallest neighbour, fim3d.hip's fp64 path in the reference's arithmetic)."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 4, shape)
    c[rng.random(shape) < 0.05] = 0.5
    c[rng.random(shape) < 0.08] = np.inf
    H, W, L = shape
    goal = np.array([W // 2, H // 2, L // 2])
    c[goal[1], goal[0], goal[2]] = 1.0
    O.set_strict(False)
    try:
        R = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    for f64 in (False, True):
        check(ctx.tmap3d(c, goal, dtype=np.float64 if f64 else np.float32), R, f64)


@pytest.mark.parametrize("f64", [False, True])
def test_layered_device_entry(ctx, f64):
    """eik_fim3d_solve on device buffers (the bench's C5 route) equals the host entry point."""
    import torch
    from eikonal import _lib as L

    c, goal = _layered_case((257, 300, 3), 21, pad=True, switch=True)
    dev = torch.device("cuda", 0)
    cd = torch.from_numpy(c.astype(np.float64 if f64 else np.float32)).to(dev)
    Td = torch.empty_like(cd)
    H, W, Lz = c.shape
    st = torch.cuda.current_stream(dev)
    ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cd.data_ptr(), Td.data_ptr(), H, W, Lz, L.EIK_F64 if f64 else L.EIK_F32,
                                     np.ascontiguousarray(goal, np.int64), st.cuda_stream))
    torch.cuda.synchronize()
    s = ctx.stats()
    assert s["iterations"] == 1 and s["tile_visits"] > 0  # one persistent launch (layered solver)
    T = Td.cpu().numpy()
    O.set_strict(False)
    try:
        R = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    check(T, R, f64)


@pytest.mark.parametrize("passes", [1, 8])
def test_layered_pass_cap_option(passes):
    """EIK_OPT_PASSES also sets the layered solver's in-place pass cap (default 24): the schedule
    changes, the field does not."""
    import eikonal
    from eikonal import _lib as L

    c3, goal = _layered_case((200, 230, 3), 31, pad=True, switch=True)
    c = eikonal.Context(0)
    try:
        c.set_option(L.OPT_PASSES, passes)
        O.set_strict(False)
        try:
            R = O.fmm3d(c3, goal, None)
        finally:
            O.set_strict(True)
        check(c.tmap3d(c3, goal, dtype=np.float32), R, False)
        if passes == 1:
            assert c.stats()["inplace_passes"] == 0
    finally:
        c.close()


def test_layered_visit_budget():
    """A tiny EIK_OPT_MAX_VISITS stops the layered solver (device-buffer entry, no host-side cost
    check) with EIK_ERR_NOCONVERGE: its in-place passes are charged to the budget too."""
    import torch
    import eikonal
    from eikonal import _lib as L

    c3, goal = _layered_case((700, 700, 3), 32, pad=True, switch=True)
    c = eikonal.Context(0)
    try:
        c.set_option(L.OPT_MAX_VISITS, 128)
        dev = torch.device("cuda", 0)
        cd = torch.from_numpy(c3.astype(np.float32)).to(dev)
        Td = torch.empty_like(cd)
        H, W, Lz = c3.shape
        rc = L.lib().eik_fim3d_solve(c._h, cd.data_ptr(), Td.data_ptr(), H, W, Lz, L.EIK_F32,
                                     np.ascontiguousarray(goal, np.int64), torch.cuda.current_stream(dev).cuda_stream)
        assert rc == L.EIK_ERR_NOCONVERGE, rc
    finally:
        c.close()


@pytest.mark.parametrize("shape,seed,pad", [((300, 280, 3), 5, True), ((70, 90, 40), 6, False), ((20, 23, 70), 7, False)])
def test_path3d_windowed(ctx, shape, seed, pad):
    """Walks longer than the path kernel's LDS window (recentred reloads, back-tracking through
    the point ring): layered z-padded volumes (integer descent), cubes with trilinear steps and a
    volume taller in z than the window; the same field through the oracle's walk, <= 1e-9."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 3, shape)
    if pad:  # cubes stay obstacle-free: their walk takes trilinear steps all the way
        c[rng.random(shape) < 0.05] = np.inf
        inf = np.full(shape[:2] + (1,), np.inf)
        c = np.concatenate([inf, c, inf], axis=2)
    H, W, L = c.shape
    z = 1 if pad else L // 2
    goal = np.array([W - 6, H - 5, z])
    start = np.array([4.0, 5.0, float(z if pad else 2)])
    c[goal[1], goal[0], goal[2]] = 1.0
    c[5, 4, int(start[2])] = 1.0
    O.set_strict(False)
    try:
        T = O.fmm3d(c, goal, None)
    finally:
        O.set_strict(True)
    ref, rst = O.gdm3d(T, start, goal.astype(float), 0.5)
    path, st = ctx.path3d(T, start, goal.astype(float))
    assert st == rst and path.shape == ref.shape, (st, rst, path.shape, ref.shape)
    assert np.abs(path - ref).max() <= 1e-9
    assert len(path) > 40


@pytest.mark.parametrize("f64", [False, True])
def test_layered_nan_cost_blocks(ctx, f64):
    """A NaN cost on the device-buffer entry (no host cost check) acts as a blocked cell: the fp64
    cost clamp of the layered solver (>= 2^-500 for the range-free square root) must not turn NaN
    into a near-zero passable cost.  Field = the oracle's with those cells at +inf."""
    import torch
    from eikonal import _lib as L

    c, goal = _layered_case((150, 170, 3), 23, pad=True, switch=False)
    cn = c.copy()
    cn[40:70, 50:120, 1:4] = np.nan  # a wall across the volume, every layer
    dev = torch.device("cuda", 0)
    cd = torch.from_numpy(cn.astype(np.float64 if f64 else np.float32)).to(dev)
    Td = torch.empty_like(cd)
    H, W, Lz = c.shape
    ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cd.data_ptr(), Td.data_ptr(), H, W, Lz, L.EIK_F64 if f64 else L.EIK_F32,
                                     np.ascontiguousarray(goal, np.int64), torch.cuda.current_stream(dev).cuda_stream))
    torch.cuda.synchronize()
    ci = np.where(np.isnan(cn), np.inf, cn)
    O.set_strict(False)
    try:
        R = O.fmm3d(ci, goal, None)
    finally:
        O.set_strict(True)
    T = Td.cpu().numpy()
    assert np.all(np.isinf(T[np.isnan(cn)]))
    check(T, R, f64)
