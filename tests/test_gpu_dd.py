"""GPU domain decomposition (eikonal/dd.py + the solver's ghost / pack / merge entry points).

Every block of a px x py split gets its own eikonal.Fim2d on cuda:0 and the halo exchange is
done in-process (recv[r][side] <- send[neighbour][opposite side]) in the same order as
dd.solve (iterate -> pack -> exchange -> merge -> active count), so the device-side ghost
merge and re-activation of BOTH solver drivers are checked without a second GPU.  The
assembled field must equal the oracle's single-domain field (fp64: 1e-9 absolute; fp32:
2e-5 relative).  The rank-parallel exchange itself is covered by test_dd_gloo.py.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
OPP = {0: 1, 1: 0, 2: 3, 3: 2}


def solve_blocks(cost, goal, px, py, f64, mode, exchange_every=4):
    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    dev = torch.device("cuda", 0)
    H, W = cost.shape
    R = px * py
    ctx = eikonal.Context(0)
    ctx.set_option(L.OPT_MODE, mode)
    dt = torch.float64 if f64 else torch.float32
    blocks = [dd.Block(H, W, px, py, r) for r in range(R)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    locs, sends, recvs, Ts, costs = [], [], [], [], []
    for b in blocks:
        c = torch.from_numpy(np.ascontiguousarray(cost[b.y0:b.y1, b.x0:b.x1])).to(dev, dt)
        send, recv, ghost = dd.make_strips(b, dt, dev, float("inf"))
        fim = eikonal.Fim2d(ctx, 1, b.h, b.w, L.EIK_F64 if f64 else L.EIK_F32)
        loc = dd.GpuLocal(fim, ghost)
        T = torch.empty_like(c)
        loc.start(c, T, b.local_goal(*goal), stream)
        locs.append(loc), sends.append(send), recvs.append(recv), Ts.append(T), costs.append(c)
    for rounds in range(1, 100000):
        for loc, send in zip(locs, sends):
            loc.iterate(exchange_every)
            loc.pack_edges(*send)
        for r, b in enumerate(blocks):
            for s in range(4):
                if b.nb[s] is not None:
                    recvs[r][s].copy_(sends[b.nb[s]][OPP[s]])
        for r, b in enumerate(blocks):
            for s in range(4):
                if b.nb[s] is not None:
                    locs[r].merge_ghost(s, recvs[r][s])
        if sum(loc.active() for loc in locs) == 0:
            break
    torch.cuda.synchronize()
    out = np.empty((H, W), np.float64)
    for b, T in zip(blocks, Ts):
        out[b.y0:b.y1, b.x0:b.x1] = T.cpu().double().numpy()
    ctx.close()
    return out, rounds


def oracle_field(cost, goal):
    O.set_strict(False)
    try:
        return O.fmm2d(cost, goal)
    finally:
        O.set_strict(True)


@pytest.mark.parametrize("mode", ["persistent", "list"])
@pytest.mark.parametrize("px,py", [(2, 1), (1, 2), (2, 2), (4, 2)])
@pytest.mark.parametrize("f64", [True, False])
def test_dd_blocks_match_single_domain(mode, px, py, f64):
    from eikonal import _lib as L

    rng = np.random.default_rng(px * 10 + py)
    H, W = 390, 455  # blocks not multiples of the 64-cell tile
    cost = rng.uniform(1, 6, (H, W))
    cost[rng.random((H, W)) < 0.08] = np.inf
    goal = (W // 3, H // 4)
    cost[goal[1], goal[0]] = 1.0
    if not f64:
        cost = cost.astype(np.float32).astype(np.float64)
    T, rounds = solve_blocks(cost, goal, px, py, f64, L.MODE_PERSISTENT if mode == "persistent" else L.MODE_LIST)
    R = oracle_field(cost, goal)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin)
    err = np.abs(T[fin] - R[fin])
    if f64:
        assert err.max() <= 1e-9, err.max()
    else:
        assert (err / np.maximum(R[fin], 1e-30)).max() <= 2e-5
    assert rounds >= 2


@pytest.mark.parametrize("f64", [True, False])
def test_solve_then_merge_then_iterate(f64):
    """The C ABI allows set_ghosts -> solve -> pack_edges -> exchange -> merge_ghost -> iterate:
    eik_fim2d_solve launches without the queue rewind, so the merge's activations must not land
    behind tickets the launch's idle waiters already took (the next launch would spin
    until the queue timeout, or lose the ghost update).  2 x 1 blocks, the first local solve by
    eik_fim2d_solve, then dd.solve's rounds; the assembled field equals the oracle's."""
    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    rng = np.random.default_rng(77)
    H, W = 260, 330
    cost = rng.uniform(1, 6, (H, W))
    cost[rng.random((H, W)) < 0.08] = np.inf
    goal = (W // 5, H // 2)
    cost[goal[1], goal[0]] = 1.0
    if not f64:
        cost = cost.astype(np.float32).astype(np.float64)
    dev = torch.device("cuda", 0)
    dt = torch.float64 if f64 else torch.float32
    ctx = eikonal.Context(0)
    ctx.set_option(L.OPT_QTIMEOUT, 5.0)  # a lost / stuck queue entry fails fast instead of hanging
    stream = torch.cuda.current_stream(dev).cuda_stream
    blocks = [dd.Block(H, W, 2, 1, r) for r in range(2)]
    fims, sends, recvs, Ts, costs = [], [], [], [], []
    for b in blocks:
        c = torch.from_numpy(np.ascontiguousarray(cost[b.y0:b.y1, b.x0:b.x1])).to(dev, dt)
        send, recv, ghost = dd.make_strips(b, dt, dev, float("inf"))
        fim = eikonal.Fim2d(ctx, 1, b.h, b.w, L.EIK_F64 if f64 else L.EIK_F32)
        fim.set_ghosts(*[g.data_ptr() if g is not None else None for g in ghost])
        T = torch.empty_like(c)
        fim.solve(c.data_ptr(), T.data_ptr(), [b.local_goal(*goal)], stream)  # no rewind after it
        fims.append(fim), sends.append(send), recvs.append(recv), Ts.append(T), costs.append(c)
    for rounds in range(1, 1000):
        for fim, send in zip(fims, sends):
            fim.pack_edges(*[t.data_ptr() if t is not None else None for t in send])
        for r, b in enumerate(blocks):
            for s in range(4):
                if b.nb[s] is not None:
                    recvs[r][s].copy_(sends[b.nb[s]][OPP[s]])
        for r, b in enumerate(blocks):
            for s in range(4):
                if b.nb[s] is not None:
                    fims[r].merge_ghost(s, recvs[r][s].data_ptr())
        if sum(f.active() for f in fims) == 0:
            break
        for f in fims:
            f.iterate(1)
    torch.cuda.synchronize()
    out = np.empty((H, W), np.float64)
    for b, T in zip(blocks, Ts):
        out[b.y0:b.y1, b.x0:b.x1] = T.cpu().double().numpy()
    ctx.close()
    R = oracle_field(cost, goal)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(out), fin)
    err = np.abs(out[fin] - R[fin])
    if f64:
        assert err.max() <= 1e-9, err.max()
    else:
        assert (err / np.maximum(R[fin], 1e-30)).max() <= 2e-5


@pytest.mark.parametrize("mode", ["persistent", "list"])
def test_nan_cost_blocks_fp64_device(mode):
    """fp64 device-buffer solve (eik_fim2d_solve, no host cost check) with a NaN block: the staged
    cost clamp (>= 2^-500) must keep NaN a blocked cell, as +inf; field = the oracle's on the
    raster with those cells at +inf."""
    import eikonal
    from eikonal import _lib as L

    rng = np.random.default_rng(31)
    H, W = 300, 280
    cost = rng.uniform(1, 5, (H, W))
    cost[100:140, 20:250] = np.nan
    goal = (W // 2, 40)
    dev = torch.device("cuda", 0)
    ctx = eikonal.Context(0)
    ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT if mode == "persistent" else L.MODE_LIST)
    ctx.set_option(L.OPT_QTIMEOUT, 5.0)
    c = torch.from_numpy(cost).to(dev)
    T = torch.empty_like(c)
    fim = eikonal.Fim2d(ctx, 1, H, W, L.EIK_F64)
    fim.solve(c.data_ptr(), T.data_ptr(), [goal], torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    fim.close()
    ctx.close()
    Tg = T.cpu().numpy()
    assert np.all(np.isinf(Tg[np.isnan(cost)]))
    R = oracle_field(np.where(np.isnan(cost), np.inf, cost), goal)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(Tg), fin)
    assert np.abs(Tg[fin] - R[fin]).max() <= 1e-9


def solve_blocks_layered(cost, goal, px, py, f64, z0, nl):
    """The in-process rounds schedule (as solve_blocks) over blocks of a [H][W][L] volume, each an
    eikonal.Fim3dLayered (the layered solver with ghost strips of nl values per edge cell)."""
    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    dev = torch.device("cuda", 0)
    H, W, Lz = cost.shape
    R = px * py
    ctx = eikonal.Context(0)
    dt = torch.float64 if f64 else torch.float32
    blocks = [dd.Block(H, W, px, py, r) for r in range(R)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    locs, sends, recvs, Ts = [], [], [], []
    for b in blocks:
        c = torch.from_numpy(np.ascontiguousarray(cost[b.y0:b.y1, b.x0:b.x1])).to(dev, dt)
        send, recv, ghost = dd.make_strips(b, dt, dev, float("inf"), per_cell=nl)
        fim = eikonal.Fim3dLayered(ctx, b.h, b.w, Lz, z0, nl, L.EIK_F64 if f64 else L.EIK_F32)
        loc = dd.GpuLocalLayered(fim, ghost)
        T = torch.empty_like(c)
        lg = b.local_goal(goal[0], goal[1])
        loc.start(c, T, (lg[0], lg[1], goal[2]), stream)
        locs.append((loc, c)), sends.append(send), recvs.append(recv), Ts.append(T)
    for rounds in range(1, 100000):
        for (loc, _), send in zip(locs, sends):
            loc.iterate(1)
            loc.pack_edges(*send)
        for r, b in enumerate(blocks):
            for s in range(4):
                if b.nb[s] is not None:
                    recvs[r][s].copy_(sends[b.nb[s]][OPP[s]])
        for r, b in enumerate(blocks):
            for s in range(4):
                if b.nb[s] is not None:
                    locs[r][0].merge_ghost(s, recvs[r][s])
        if sum(loc.active() for loc, _ in locs) == 0:
            break
    torch.cuda.synchronize()
    out = np.empty((H, W, Lz), np.float64)
    for b, T in zip(blocks, Ts):
        out[b.y0:b.y1, b.x0:b.x1] = T.cpu().double().numpy()
    ctx.close()
    return out, rounds


def _volume(H, W, seed, pad):
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 5, (H, W, 3))
    c[rng.random((H, W, 3)) < 0.08] = np.inf
    c[:, : W // 2, 0] *= 0.3
    c[:, W // 2:, 2] *= 0.3
    if pad:  # the planner's z padding (Coupled_motion_planner.py:355-356)
        inf = np.full((H, W, 1), np.inf)
        c = np.concatenate([inf, c, inf], axis=2)
    return c


@pytest.mark.parametrize("shape,px,py,pad", [((1024, 1024), 2, 1, True), ((1024, 1024), 2, 2, True),
                                             ((390, 455), 4, 2, False), ((300, 333), 1, 2, True)])
@pytest.mark.parametrize("f64", [True, False])
def test_dd_layered_blocks_match_single_domain(shape, px, py, pad, f64):
    """SURVEY §8(e), C5 across GPUs: a few-layer volume split in x-y, layers together (strips of nl
    values per edge cell, eik_fim3dl_create / eik_fim2d_pack_edges / eik_fim2d_merge_ghost), blocks
    not multiples of the tile (40-row fp64 / 64-row fp32 tiles cut by the block ends, where the
    south / east ghosts sit inside a tile).  The assembled field equals the single-domain layered
    solve of the same volume: masks equal, fp64 <= 1e-11 / fp32 <= 1e-5 relative."""
    import eikonal

    H, W = shape
    cost = _volume(H, W, px * 10 + py, pad)
    z0 = 1 if pad else 0
    goal = (W // 3, H // 2, z0 + 1)
    cost[goal[1], goal[0], goal[2]] = 1.0
    ctx = eikonal.Context(0)
    try:
        ref = ctx.tmap3d(cost, np.array(goal), dtype=np.float64 if f64 else np.float32).astype(np.float64)
    finally:
        ctx.close()
    T, rounds = solve_blocks_layered(cost, goal, px, py, f64, z0, 3)
    assert rounds >= 2
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(T), fin)
    rel = np.abs(T[fin] - ref[fin]) / np.maximum(ref[fin], 1e-30)
    assert rel.max() <= (1e-11 if f64 else 1e-5), rel.max()
