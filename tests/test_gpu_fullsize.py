"""GPU parity at BASELINE.json's full sizes (configs[1..4]), on the bench's own synthetic rasters.

* C2, 4096^2 DEM raster: the fp64 field (the headline arithmetic) against the oracle's heap FMM
  (fp64, the reference's algorithm, ~3 s on one core) -- masks equal, max abs <= 1e-9 -- and its
  path against the oracle's walk on the oracle's field; the fp32 field -- masks equal, max
  relative error <= 2e-5 -- and the path kernel on it against the oracle's walk on
  the same field, <= 1e-9 cells.
* C2 bidirectional with EIK_OPT_EXACT_BAND: nodeJoin and both partial fields bit-identical to the
  oracle's sequential band (biComputeTmap, goal at the centre, start at (256, 256)).
* C3, 128 x 1024^2 batch: one batched solve, four of its maps against the oracle.
* C4, 16384^2 DEM raster on one GPU: too large for the oracle inside a test, so size-independent
  properties of the converged field, evaluated on the device in fp64: T[goal] = 0; every reached
  cell satisfies the reference's local solve (FastMarching.py:17-29) of its own neighbours to
  2e-5 relative (the Godunov fixed point the reference FMM also reaches);
  every reached cell other than the goal has a strictly smaller reached neighbour (a descent to
  the goal exists) and no unreached finite-cost cell touches a reached one (the reached set is
  closed, i.e. exactly the goal's component).
* C5, 4096^2 x 3 layered volume: the same properties with FastMarching3D's n-D local solve and
  six neighbours, and the 3D path kernel against the oracle's walk on the field, <= 1e-9.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch

    import eikonal
    from eikonal import _lib as L
    from eikonal import terrain

    dev = torch.device("cuda", 0)
    ctx = eikonal.Context(0)
    yield torch, eikonal, L, terrain, dev, ctx
    ctx.close()


def local_solve(torch, T, c):
    """FastMarching.getEikonal of every cell's own neighbours, fp64 (+inf outside the raster)."""
    inf = float("inf")
    P = torch.nn.functional.pad(T, (1, 1, 1, 1), value=inf)
    a = torch.minimum(P[1:-1, :-2], P[1:-1, 2:])  # Thor: x neighbours (:57-62)
    b = torch.minimum(P[:-2, 1:-1], P[2:, 1:-1])  # Tver
    lo, hi = torch.minimum(a, b), torch.maximum(a, b)
    d = hi - lo
    two = 0.5 * (a + b + torch.sqrt(torch.clamp(2 * c * c - d * d, min=0)))
    w = torch.where(c < d, lo + c, two)  # :26-29 (one inf: d = inf, lo + c)
    return torch.where(torch.isinf(lo), torch.full_like(lo, inf), w)


def check_properties(torch, T32, c32, goal, rows=2048, tol=2e-5):
    H, W = T32.shape
    gx, gy = goal
    assert float(T32[gy, gx]) == 0.0
    worst = 0.0
    for y0 in range(0, H, rows):
        ya, yb = max(y0 - 1, 0), min(y0 + rows + 1, H)
        T = T32[ya:yb].double()
        c = c32[ya:yb].double()
        s, e = y0 - ya, y0 - ya + min(rows, H - y0)
        fin = torch.isfinite(T)
        w = local_solve(torch, T, c)[s:e]
        Tc, finc = T[s:e], fin[s:e]
        # the goal is the source (T = 0); every other reached cell is its neighbours' local solve
        src = torch.zeros_like(finc)
        if ya <= gy < yb and s <= gy - ya < e:
            src[gy - ya - s, gx] = True
        chk = finc & ~src
        assert bool(torch.isfinite(c[s:e][finc]).all()), "a reached cell has infinite cost"
        rel = ((Tc[chk] - w[chk]).abs() / Tc[chk].clamp(min=1e-30))
        if rel.numel():
            worst = max(worst, float(rel.max()))
        # descent: a reached non-source cell has a strictly smaller reached neighbour
        inf = float("inf")
        P = torch.nn.functional.pad(T, (1, 1, 1, 1), value=inf)
        nmin = torch.minimum(torch.minimum(P[1:-1, :-2], P[1:-1, 2:]), torch.minimum(P[:-2, 1:-1], P[2:, 1:-1]))[s:e]
        assert bool((nmin[chk] < Tc[chk]).all()), "a reached cell without a descent neighbour"
        # closure: an unreached finite-cost cell has no reached neighbour
        open_ = ~finc & torch.isfinite(c[s:e])
        assert not bool(torch.isfinite(nmin[open_]).any()), "an unreached cell next to a reached one"
    assert worst <= tol, worst
    return worst


def test_c2_full_size_fp64_vs_oracle(env):
    """The headline configuration in the headline arithmetic (bench.py --dtype f64, the reference's
    float64): the device-resident fp64 solve of the 4096^2 C2 raster against the oracle's fp64 heap
    FMM, masks equal and max abs <= 1e-9; then the end-to-end path (fp64 field -> path kernel,
    device-resident, the bench's ms-to-path route) against the oracle's walk on the ORACLE's field."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 4096
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).double().contiguous()
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F64)
    goal, start = (N // 2, N // 2), (256, 256)
    stream = torch.cuda.current_stream(dev)
    fim.solve(cost.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)
    torch.cuda.synchronize()
    fim.close()
    Tg = T.cpu().numpy()
    O.set_strict(False)
    try:
        R = O.fmm2d(cost.cpu().numpy(), goal)
    finally:
        O.set_strict(True)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(Tg), fin)
    err = np.abs(Tg[fin] - R[fin]).max()
    assert err <= 1e-9, err
    path, st = ctx.path2d(Tg, start, goal)
    ref, rst = O.gdm2d(R, np.array(start, float), np.array(goal, float))
    assert st == rst == 0 and path.shape == ref.shape and len(path) > 1000
    assert np.abs(path - ref).max() <= 1e-6


def test_c2_full_size_bidirectional_exact_band(env):
    """biComputeTmap on the 4096^2 C2 raster with EIK_OPT_EXACT_BAND (goal at the centre, start at
    (256, 256), the bench's ms-to-path query): nodeJoin and both partial fields bit-identical to the
    oracle's sequential band (orc_fmm2d_bidir, the reference's algorithm) -- the replay at full size,
    ~2 M pops per front, on the capped-fronts path."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 4096
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).double().contiguous().cpu().numpy()
    goal, start = (N // 2, N // 2), (256, 256)
    c = eikonal.Context(0)
    try:
        c.set_option(L.OPT_EXACT_BAND, 1)
        TG, TS, join = c.tmap2d_bidir(cost, goal, start)
        info, fr = c.exact_info(), c.fronts_info()
    finally:
        c.close()
    O.set_strict(False)
    try:
        RG, RS, rj = O.fmm2d_bidir(cost, goal, start)
    finally:
        O.set_strict(True)
    assert info["passes"] >= 1 and fr["capped"], (info, fr)
    assert np.array_equal(join, rj), (join, rj)
    for A, B in ((TG, RG), (TS, RS)):
        assert np.array_equal(np.isfinite(A), np.isfinite(B))
        assert np.array_equal(A.view(np.uint64), B.view(np.uint64)), int((A != B).sum())


def test_c2_full_size_fp64_priority_bands(env):
    """The headline solve with EIK_OPT_PRIO (priority bands at the default width) against
    the default FIFO solve of the same raster: the same fixed point up to rounding (masks equal,
    <= 1e-11 relative), and the Godunov properties of check_properties."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 4096
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).double().contiguous()
    goal = (N // 2, N // 2)
    stream = torch.cuda.current_stream(dev)
    out = []
    for prio in (0.0, 1.0):
        c2 = eikonal.Context(0)
        try:
            c2.set_option(L.OPT_PRIO, prio)
            T = torch.empty_like(cost)
            fim = eikonal.Fim2d(c2, 1, N, N, L.EIK_F64)
            fim.solve(cost.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)
            torch.cuda.synchronize()
            out.append((T, fim.stats()))
            fim.close()
        finally:
            c2.close()
    (T0, s0), (T1, s1) = out
    fin = torch.isfinite(T0)
    assert torch.equal(fin, torch.isfinite(T1))
    rel = ((T1[fin] - T0[fin]).abs() / T0[fin].clamp(min=1e-30)).max().item()
    assert rel <= 1e-11, rel
    check_properties(torch, T1, cost, goal, tol=1e-11)
    print(f"C2 fp64 FIFO: {s0['tile_visits']} visits + {s0['inplace_passes']} passes; priority bands: "
          f"{s1['tile_visits']} + {s1['inplace_passes']}")


def test_c2_full_size_vs_oracle(env):
    torch, eikonal, L, terrain, dev, ctx = env
    N = 4096
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
    goal, start = (N // 2, N // 2), (256, 256)
    stream = torch.cuda.current_stream(dev)
    fim.solve(cost.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)
    torch.cuda.synchronize()
    fim.close()
    check_properties(torch, T, cost, goal)
    c64 = cost.double().cpu().numpy()
    Tg = T.cpu().numpy()
    O.set_strict(False)
    try:
        R = O.fmm2d(c64, goal)
    finally:
        O.set_strict(True)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(Tg), fin)
    rel = np.abs(Tg[fin].astype(np.float64) - R[fin]) / np.maximum(R[fin], 1e-30)
    assert rel.max() <= 2e-5, rel.max()
    # the path kernel on the GPU field vs the oracle's walk on the same field
    path, st = ctx.path2d(Tg, start, goal)
    ref, rst = O.gdm2d(Tg.astype(np.float64), np.array(start, float), np.array(goal, float))
    assert st == rst == 0 and path.shape == ref.shape and len(path) > 1000
    assert np.abs(path - ref).max() <= 1e-9


@pytest.mark.parametrize("f64", [False, True])
def test_c3_full_batch_vs_oracle(env, f64):
    """configs[2] as the bench runs it (bench.py bench_batch: 128 maps of 1024^2, seeds 1000..1127,
    the same goals) in ONE batched persistent solve, fp32 and fp64 (the bench's credited
    arithmetic); four of its maps against the oracle's fp64 heap FMM: masks equal, fp32 <= 2e-5
    relative, fp64 <= 1e-9 absolute."""
    torch, eikonal, L, terrain, dev, ctx = env
    import bench

    B, N = 128, 1024
    dt = torch.float64 if f64 else torch.float32
    cost = torch.empty((B, N, N), dtype=dt, device=dev)
    goals = []
    for b in range(B):
        cost[b] = terrain.cost_block(0, 0, N, N, N, N, seed=1000 + b, device=dev).to(dt)
        goals.append(bench.c3_goal(cost[b], b, N))
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, B, N, N, L.EIK_F64 if f64 else L.EIK_F32)
    fim.solve(cost.data_ptr(), T.data_ptr(), goals, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    fim.close()
    assert float(torch.isfinite(T).float().mean()) > 0.5
    O.set_strict(False)
    try:
        for b in (0, 37, 90, 127):
            R = O.fmm2d(cost[b].double().cpu().numpy(), goals[b])
            Tg = T[b].cpu().numpy().astype(np.float64)
            fin = np.isfinite(R)
            assert np.array_equal(np.isfinite(Tg), fin), b
            if f64:
                err = np.abs(Tg[fin] - R[fin]).max()
                assert err <= 1e-9, (b, err)
            else:
                rel = np.abs(Tg[fin] - R[fin]) / np.maximum(R[fin], 1e-30)
                assert rel.max() <= 2e-5, (b, rel.max())
    finally:
        O.set_strict(True)
    del cost, T
    torch.cuda.empty_cache()


@pytest.mark.parametrize("f64", [False, True])
def test_c4_full_size_properties(env, f64):
    """configs[3] on one GPU (bench.py bench_c4: the 16384^2 raster, seed 7, goal at the centre),
    fp32 (the 4-waves-per-SIMD kernel) and fp64: T[goal] = 0, the Godunov fixed point of every
    reached cell's own neighbours (fp32 <= 2e-5, fp64 <= 1e-11 relative), descent and closure."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 16384
    dt = torch.float64 if f64 else torch.float32
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).to(dt).contiguous()
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F64 if f64 else L.EIK_F32)
    goal = (N // 2, N // 2)
    fim.solve(cost.data_ptr(), T.data_ptr(), [goal], torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    fim.close()
    assert float(torch.isfinite(T).float().mean()) > 0.9
    worst = check_properties(torch, T, cost, goal, tol=1e-11 if f64 else 2e-5)
    print(f"C4 {'fp64' if f64 else 'fp32'} worst fixed-point residual {worst:.3e}")
    del cost, T
    torch.cuda.empty_cache()


def local_solve3(torch, T, c):
    """FastMarching3D's n-D local solve (:59-75) of every cell's own six neighbours, fp64: the
    axis minima sorted, the 3-axis root when C^2 > (s2-s0)^2 + (s2-s1)^2, else the 2-axis root when
    C^2 > (s1-s0)^2, else s0 + C (an inf maximum is dropped by the same tests)."""
    inf = float("inf")
    P = torch.nn.functional.pad(T, (1, 1, 1, 1, 1, 1), value=inf)
    ty = torch.minimum(P[:-2, 1:-1, 1:-1], P[2:, 1:-1, 1:-1])
    tx = torch.minimum(P[1:-1, :-2, 1:-1], P[1:-1, 2:, 1:-1])
    tz = torch.minimum(P[1:-1, 1:-1, :-2], P[1:-1, 1:-1, 2:])
    s = torch.sort(torch.stack([tx, ty, tz]), dim=0).values
    s0, s1, s2 = s[0], s[1], s[2]
    C2 = c * c
    S2, Q2 = s0 + s1, s0 * s0 + s1 * s1
    S3, Q3 = S2 + s2, Q2 + s2 * s2
    t1 = s0 + c
    t2 = (S2 + torch.sqrt(torch.clamp(2 * C2 + S2 * S2 - 2 * Q2, min=0))) / 2
    t3 = (S3 + torch.sqrt(torch.clamp(3 * C2 + S3 * S3 - 3 * Q3, min=0))) / 3
    w = torch.where(C2 > (s2 - s0) ** 2 + (s2 - s1) ** 2, t3, torch.where(C2 > (s1 - s0) ** 2, t2, t1))
    nmin = torch.minimum(torch.minimum(tx, ty), tz)
    return torch.where(torch.isinf(s0), torch.full_like(s0, inf), w), nmin


@pytest.mark.parametrize("f64", [False, True])
def test_c5_planar_matches_volume_layout(env, f64):
    """configs[4] with EIK_OPT_LAYER_PLANAR (the layered solver on [nl][H][W] copies): the field equals
    the volume-layout solve's (masks equal; fp32 <= 1e-5, fp64 <= 1e-11 relative -- a different
    tile order rounds differently), the padding layers +inf."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 4096
    c0 = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
    if f64:
        c0 = c0.double()
    inf = torch.full_like(c0, float("inf"))
    c1 = torch.where(c0 > 100, inf, 1.6 * c0)
    yy = torch.arange(N, device=dev)[:, None] // 64
    xx = torch.arange(N, device=dev)[None, :] // 64
    c2 = torch.where(((yy + 2 * xx) % 5) == 0, inf, 0.8 * c0)
    cost = torch.stack([inf, c0, c1, c2, inf], dim=-1).contiguous()
    del c1, c2, inf
    goal = np.array((N // 2, N // 2, 1), np.int64)
    stream = torch.cuda.current_stream(dev)
    out = []
    for planar in (0, 1):
        c = eikonal.Context(0, options={"LAYER_PLANAR": planar})
        try:
            T = torch.full_like(cost, 7.0)  # the planar solve writes every value (padding +inf)
            c._chk(L.lib().eik_fim3d_solve(c._h, cost.data_ptr(), T.data_ptr(), N, N, 5,
                                           L.EIK_F64 if f64 else L.EIK_F32, goal, stream.cuda_stream))
            torch.cuda.synchronize()
            out.append(T)
        finally:
            c.close()
    T0, T1 = out
    assert bool(torch.isinf(T1[:, :, 0]).all()) and bool(torch.isinf(T1[:, :, 4]).all())
    fin = torch.isfinite(T0)
    assert torch.equal(fin, torch.isfinite(T1))
    rel = ((T1[fin].double() - T0[fin].double()).abs() / T0[fin].double().clamp(min=1e-30)).max().item()
    assert rel <= (1e-11 if f64 else 1e-5), rel


@pytest.mark.parametrize("f64", [False, True])
def test_c5_full_size_properties(env, f64):
    """configs[4]: the bench's 4096 x 4096 x 3 layered volume (z padded with +inf layers, 5 in
    memory) through the layered solver, fp32 (64-row tiles) and fp64 (40-row tiles, the reference's
    precision); the FM3D fixed point (fp32 <= 2e-5, fp64 <= 1e-11 relative), descent and closure
    as for C4; the 3D path kernel on that field against the oracle's walk on the same field."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 4096
    c0 = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
    if f64:
        c0 = c0.double()
    inf = torch.full_like(c0, float("inf"))
    c1 = torch.where(c0 > 100, inf, 1.6 * c0)
    yy = torch.arange(N, device=dev)[:, None] // 64
    xx = torch.arange(N, device=dev)[None, :] // 64
    c2 = torch.where(((yy + 2 * xx) % 5) == 0, inf, 0.8 * c0)
    cost = torch.stack([inf, c0, c1, c2, inf], dim=-1).contiguous()
    del c1, c2, inf
    T = torch.empty_like(cost)
    goal = (N // 2, N // 2, 1)
    stream = torch.cuda.current_stream(dev)
    ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cost.data_ptr(), T.data_ptr(), N, N, 5, L.EIK_F64 if f64 else L.EIK_F32,
                                     np.array(goal, np.int64), stream.cuda_stream))
    torch.cuda.synchronize()
    assert ctx.stats()["iterations"] == 1  # one persistent launch: the layered solver
    check_layered_properties(torch, T, cost, goal, f64)
    Th = T.cpu().numpy()
    del cost
    start = np.array([256.0, 256.0, 1.0])
    end = np.array([float(goal[0]), float(goal[1]), 1.0])
    path, st = ctx.path3d(Th, start, end)
    ref, rst = O.gdm3d(Th.astype(np.float64), start, end, 0.5)
    assert st == rst == 0 and path.shape == ref.shape and len(path) > 1000
    assert np.abs(path - ref).max() <= 1e-9


def check_layered_properties(torch, T, cost, goal, f64, tol64=1e-11):
    """The FM3D fixed point of a layered solve, block by block of rows (fp32 <= 2e-5, fp64 <= 1e-11
    relative), a descent neighbour for every reached cell, the reached set closed, > 80 % reached."""
    N = T.shape[0]
    assert float(T[goal[1], goal[0], goal[2]]) == 0.0
    worst, rows = 0.0, 512
    for y0 in range(0, N, rows):
        ya, yb = max(y0 - 1, 0), min(y0 + rows + 1, N)
        s, e = y0 - ya, y0 - ya + min(rows, N - y0)
        Tb, cb = T[ya:yb].double(), cost[ya:yb].double()
        w, nmin = local_solve3(torch, Tb, cb)
        w, nmin, Tc, cc = w[s:e], nmin[s:e], Tb[s:e], cb[s:e]
        fin = torch.isfinite(Tc)
        src = torch.zeros_like(fin)
        if y0 <= goal[1] < y0 + rows:
            src[goal[1] - y0, goal[0], goal[2]] = True
        chk = fin & ~src
        assert bool(torch.isfinite(cc[fin]).all())
        if bool(chk.any()):
            worst = max(worst, float(((Tc[chk] - w[chk]).abs() / Tc[chk].clamp(min=1e-30)).max()))
        assert bool((nmin[chk] < Tc[chk]).all()), "a reached cell without a descent neighbour"
        assert not bool(torch.isfinite(nmin[~fin & torch.isfinite(cc)]).any()), "reached set not closed"
    assert worst <= (tol64 if f64 else 2e-5), worst
    assert float(torch.isfinite(T[:, :, 1:4]).float().mean()) > 0.8


@pytest.mark.parametrize("f64", [False, True])
def test_c5_volume_over_4gib(env, f64):
    """configs[4]'s volume at 16384 x 16384 (5 layers: 5.4 GB fp32, 10.7 GB fp64 -- past the 4 GiB a
    32-bit buffer offset spans): the layered solver addresses T per tile and layer (fim2dl.hip), so
    the volume stays on it (one launch; it went to fim3d.hip's cube solver at 0.3 Gcells/s before),
    and the field has the FM3D properties of test_c5_full_size_properties."""
    torch, eikonal, L, terrain, dev, ctx = env
    N = 16384
    c0 = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).contiguous()
    if f64:
        c0 = c0.double()
    inf = torch.full_like(c0, float("inf"))
    c1 = torch.where(c0 > 100, inf, 1.6 * c0)
    yy = torch.arange(N, device=dev)[:, None] // 64
    xx = torch.arange(N, device=dev)[None, :] // 64
    c2 = torch.where(((yy + 2 * xx) % 5) == 0, inf, 0.8 * c0)
    cost = torch.stack([inf, c0, c1, c2, inf], dim=-1).contiguous()
    del c0, c1, c2, inf, yy, xx
    T = torch.empty_like(cost)
    goal = (N // 2, N // 2, 1)
    stream = torch.cuda.current_stream(dev)
    ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cost.data_ptr(), T.data_ptr(), N, N, 5, L.EIK_F64 if f64 else L.EIK_F32,
                                     np.array(goal, np.int64), stream.cuda_stream))
    torch.cuda.synchronize()
    s = ctx.stats()
    assert s["iterations"] == 1 and s["tile_visits"] < 16 * (N // 64) * (N // 64), s  # the layered solver
    # fp64: the check's own 3-axis form (S + sqrt(3C^2 + S^2 - 3Q)) / 3 cancels by ~eps T / C, and T
    # runs 4x further than on the 4096 raster: 4e-11 (measured 1.15e-11; the solver solves relative
    # to the smallest neighbour, local_solve3 does not)
    check_layered_properties(torch, T, cost, goal, f64, tol64=4e-11)
    del T, cost
    torch.cuda.empty_cache()
