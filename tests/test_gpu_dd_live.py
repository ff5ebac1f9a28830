"""GPU live domain decomposition (dd.solve_live: one persistent launch per block stays up while
its halo agent runs the host's exchange rounds).

* single block, full grid: the halo agent (last workgroup of the launch) serves the host's
  pack / merge rounds while every other workgroup solves (the bench's per-rank configuration).
* 2 and 4 processes on cuda:0 (co-resident grids), dd.IpcHalo (hipIpc-shared strips) +
  dd.solve_live over gloo: the bench's N > 1 code path end to end, peer stores within one device.
  (One process per block: launches of one process on streams that share a hardware queue
  would serialise.)
Fields equal the oracle's single-domain field (fp64 1e-9 abs, fp32 2e-5 rel), and no cell is
left above the local solve of its own neighbours (a missed halo update: a ghost strip that lies
inside a tile cut by the block's end must be refreshed by the in-place passes' halo reload).
"""
import os
import socket

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
OPP = {0: 1, 1: 0, 2: 3, 3: 2}


def _cost(H, W, seed, goal):
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 6, (H, W))
    c[rng.random((H, W)) < 0.08] = np.inf
    c[goal[1], goal[0]] = 1.0
    return c


def _oracle(cost, goal):
    O.set_strict(False)
    try:
        return O.fmm2d(cost, goal)
    finally:
        O.set_strict(True)


def _residual(T, c):
    """max over reached non-goal cells of (T - local solve of its own neighbours) / T, fp64
    (FastMarching.py:17-29).  A converged field is a fixed point up to rounding (fp32: ~1e-7);
    a missed halo update leaves cells ABOVE their neighbours' solve (seen: 1e-5 .. 1e-3), which
    this catches even when the error against the oracle stays under the field tolerance."""
    P = np.pad(T, 1, constant_values=np.inf)
    a = np.minimum(P[1:-1, :-2], P[1:-1, 2:])
    b = np.minimum(P[:-2, 1:-1], P[2:, 1:-1])
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    with np.errstate(invalid="ignore", over="ignore"):
        d = hi - lo
        w = np.where(c < d, lo + c, 0.5 * (a + b + np.sqrt(np.clip(2 * c * c - d * d, 0, None))))
        w = np.where(np.isinf(lo), np.inf, w)
        m = np.isfinite(T) & (T > 0)
        return float(((T[m] - w[m]) / T[m]).max()) if m.any() else 0.0


def _check(T, R, f64, cost=None):
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin)
    err = np.abs(T[fin] - R[fin])
    if f64:
        assert err.max() <= 1e-9, err.max()
    else:
        assert (err / np.maximum(R[fin], 1e-30)).max() <= 2e-5
    if cost is not None:  # no cell left above its neighbours' local solve (missed update)
        res = _residual(T, cost)
        assert res <= (1e-9 if f64 else 1e-6), res


def test_live_single_block_full_grid():
    """One block, default (full-occupancy) grid, no neighbours: the halo agent answers the host's
    rounds while every other workgroup solves; the field equals the oracle's."""
    import types

    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    H, W = 700, 900
    goal = (W // 2, H // 2)
    cost = _cost(H, W, 5, goal).astype(np.float32).astype(np.float64)
    dev = torch.device("cuda", 0)
    ctx = eikonal.Context(0)
    ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
    ctx.set_option(L.OPT_QTIMEOUT, 10.0)
    c = torch.from_numpy(cost).to(dev, torch.float32)
    T = torch.empty_like(c)
    fim = eikonal.Fim2d(ctx, 1, H, W, L.EIK_F32)
    loc = dd.LiveGpuLocal(fim, [None] * 4)
    none = types.SimpleNamespace(targets=([None] * 4, [None] * 4), recvs=([None] * 4, [None] * 4))
    for _ in range(2):
        loc.start(c, T, goal, torch.cuda.current_stream(dev).cuda_stream)
        loc.launch(none)
        try:
            for r in range(1, 100000):
                loc.live_pack(r & 1)
                a, ch = loc.live_merge(r & 1)
                assert ch == 0
                if a == 0:
                    break
        finally:
            left = loc.release()
        assert left == 0
        torch.cuda.synchronize()
        _check(T.cpu().double().numpy(), _oracle(cost, goal), False, cost)
    ctx.close()


def _why(rank, e):
    """a worker's failure with its cause chain (dd.solve_live raises on every rank alike; the
    cause -- the eikonal error of the rank that failed, with its queue error word -- rides below)"""
    parts = [f"rank {rank}: {e!r}"]
    c = e.__cause__ or e.__context__
    while c is not None and len(parts) < 4:
        parts.append(repr(c))
        c = c.__cause__ or c.__context__
    return " <- ".join(parts)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ipc_worker(rank, world, port, H, W, goal, seed, q, f64):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "planning-motion_planning_amd"))
    import torch.distributed as dist

    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        px, py = dd.SPLITS[world]
        blk = dd.Block(H, W, px, py, rank)
        cost = _cost(H, W, seed, goal).astype(np.float64 if f64 else np.float32)[blk.y0:blk.y1, blk.x0:blk.x1]
        c = torch.from_numpy(np.ascontiguousarray(cost)).to(dev)
        T = torch.empty_like(c)
        ctx = eikonal.Context(0)
        ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
        ctx.set_option(L.OPT_GRID, 160 // world)  # the ranks share one GPU: co-resident grids
        ctx.set_option(L.OPT_QTIMEOUT, 10.0)
        dt = torch.float64 if f64 else torch.float32
        fim = eikonal.Fim2d(ctx, 1, blk.h, blk.w, L.EIK_F64 if f64 else L.EIK_F32)
        _, _, ghost = dd.make_strips(blk, dt, dev, float("inf"))
        loc = dd.LiveGpuLocal(fim, ghost)
        halo = dd.IpcHalo(ctx, blk, 8 if f64 else 4)
        vote = dd.NodeVote() if world > 2 else None  # shared-memory vote, else gloo all-reduce
        res = []
        for _ in range(2):  # twice: the strips and the solver are reused
            loc.start(c, T, blk.local_goal(*goal), torch.cuda.current_stream(dev).cuda_stream)
            rounds = dd.solve_live(loc, blk, halo, vote=vote)
            torch.cuda.synchronize()
            assert dd.halo_consistent(blk, T, ghost)
            res.append(T.cpu().double().numpy())
        dist.barrier()
        halo.close()
        q.put((rank, blk.y0, blk.y1, blk.x0, blk.x1, res, rounds, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, 0, 0, 0, 0, None, 0, _why(rank, e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,f64", [(2, False), (2, True), (4, False), (4, True), (8, True)])
def test_live_ipc_processes(world, f64):
    import torch.multiprocessing as mp

    H, W = 300, 520
    goal = (W // 4, H // 2)
    seed = 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, world, port, H, W, goal, seed, q, f64)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [x[-1] for x in parts if x[-1]]
    assert not errs, "\n".join(errs)
    cost = _cost(H, W, seed, goal)
    if not f64:
        cost = cost.astype(np.float32).astype(np.float64)
    R = _oracle(cost, goal)
    for k in range(2):
        T = np.full((H, W), np.nan)
        for _, y0, y1, x0, x1, res, rounds, _ in parts:
            T[y0:y1, x0:x1] = res[k]
            assert rounds >= 2
        _check(T, R, f64, cost)


def _terrain_worker(rank, world, port, N, q, ring=0):
    """One rank of bench.py's N > 1 configuration (configs[3] scaled to N^2): its block of the seed-7
    terrain raster generated on the device, fp64, the live schedule over IPC strips + the node vote.
    ring > 0: EIK_OPT_PRIO_RING, slots per priority band."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "planning-motion_planning_amd"))
    import torch.distributed as dist

    import eikonal
    from eikonal import _lib as L
    from eikonal import dd, terrain

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        px, py = dd.SPLITS[world]
        blk = dd.Block(N, N, px, py, rank)
        c = terrain.cost_block(blk.y0, blk.x0, blk.h, blk.w, N, N, seed=7, device=dev).double().contiguous()
        T = torch.empty_like(c)
        ctx = eikonal.Context(0)
        ctx.set_option(L.OPT_GRID, max(2, 3 * torch.cuda.get_device_properties(dev).multi_processor_count // (2 * world)))
        ctx.set_option(L.OPT_QTIMEOUT, 20.0)
        if ring:
            ctx.set_option(L.OPT_PRIO_RING, ring)
        fim = eikonal.Fim2d(ctx, 1, blk.h, blk.w, L.EIK_F64)
        _, _, ghost = dd.make_strips(blk, torch.float64, dev, float("inf"))
        loc = dd.LiveGpuLocal(fim, ghost)
        halo = dd.IpcHalo(ctx, blk, 8)
        vote = dd.NodeVote()
        loc.start(c, T, blk.local_goal(N // 2, N // 2), torch.cuda.current_stream(dev).cuda_stream)
        rounds = dd.solve_live(loc, blk, halo, vote=vote)
        torch.cuda.synchronize()
        ok = dd.halo_consistent(blk, T, ghost)
        dist.barrier()
        halo.close()
        vote.close()
        q.put((rank, blk.y0, blk.y1, blk.x0, blk.x1, T.cpu().numpy(), rounds, ok, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, 0, 0, 0, 0, None, 0, False, _why(rank, e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ring", [0, 64])
def test_c4_split_4x2_assembled_field(ring):
    """configs[3]'s 4 x 2 split at a real size: a 4096^2 fp64 raster of the bench's terrain (seed 7,
    goal at the centre) over 8 processes sharing cuda:0 (the bench's EIK_BENCH_SHARED_GPU grids, 3/4 of
    the co-resident workgroups), the live schedule (IPC peer stores + shared-memory vote).  The
    assembled blocks are compared with the single-domain solve of the same raster: masks equal,
    <= 1e-11 relative, and every reached cell a fixed point of its own neighbours (<= 1e-9 relative
    residual).
    ring=64: every priority band's ring forced to 64 slots, 1/8 of a block's 512 tiles (16 x 32 tiles
    of 1024 x 2048).  The band-membership bits (fim_engine.hpp band_put) bound a band to one entry per
    tile, so the default ring (>= 2 x the tiles) cannot lap; this case checks a long live launch on
    rings far below that (profiles/r06c_ring_probe.log: 512 / 256 / 128 / 64 slots, both the round-5
    and this library, no lap).  Round 5's failure of this test was not a ring lap but residency: 8
    launches of exactly the co-resident grid each, and one rank's halo agent -- then its LAST
    workgroup -- could not start while another rank's small kernels held a slot."""
    import torch.multiprocessing as mp

    import eikonal
    from eikonal import _lib as L
    from eikonal import terrain

    world, N = 8, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_terrain_worker, args=(r, world, port, N, q, ring)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = [q.get(timeout=300) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [x[-1] for x in parts if x[-1]]
    assert not errs, "\n".join(errs)
    assert all(x[7] for x in parts), "halo strips differ from the neighbours' final edges"
    Tdd = np.full((N, N), np.nan)
    for _, y0, y1, x0, x1, Tb, rounds, _, _ in parts:
        Tdd[y0:y1, x0:x1] = Tb
        assert rounds >= 2
    assert not np.isnan(Tdd).any()
    dev = torch.device("cuda", 0)
    c = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).double().contiguous()
    T = torch.empty_like(c)
    ectx = eikonal.Context(0)
    fim = eikonal.Fim2d(ectx, 1, N, N, L.EIK_F64)
    fim.solve(c.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    fim.close()
    ectx.close()
    Ts, cost = T.cpu().numpy(), c.cpu().numpy()
    fin = np.isfinite(Ts)
    assert np.array_equal(np.isfinite(Tdd), fin)
    rel = np.abs(Tdd[fin] - Ts[fin]) / np.maximum(Ts[fin], 1e-30)
    assert rel.max() <= 1e-11, rel.max()
    res = _residual(Tdd, cost)
    assert res <= 1e-9, res


def _layered_worker(rank, world, port, H, W, goal, q):
    """One rank of a C5-style volume split in x-y (layers together): eikonal.Fim3dLayered on its
    block with ghost strips of nl values per edge cell, the relaunch schedule (dd.solve) over gloo."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "planning-motion_planning_amd"))
    import torch.distributed as dist

    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        px, py = dd.SPLITS[world]
        blk = dd.Block(H, W, px, py, rank)
        vol = _volume5(H, W, goal)
        c = torch.from_numpy(np.ascontiguousarray(vol[blk.y0:blk.y1, blk.x0:blk.x1])).to(dev)
        T = torch.empty_like(c)
        ctx = eikonal.Context(0)
        ctx.set_option(L.OPT_GRID, max(2, 3 * torch.cuda.get_device_properties(dev).multi_processor_count // (2 * world)))
        nl = 3
        dsend, drecv, ghost = dd.make_strips(blk, torch.float64, dev, float("inf"), per_cell=nl)
        hsend, hrecv, _ = dd.make_strips(blk, torch.float64, "cpu", float("inf"), per_cell=nl)
        fim = eikonal.Fim3dLayered(ctx, blk.h, blk.w, 5, 1, nl, L.EIK_F64)
        loc = dd.GpuLocalLayered(fim, ghost)
        lg = blk.local_goal(goal[0], goal[1])
        loc.start(c, T, (lg[0], lg[1], goal[2]), torch.cuda.current_stream(dev).cuda_stream)
        rounds = dd.solve(dd.HostStaged(loc, dsend, drecv), blk, hsend, hrecv, exchange_every=4,
                          count_device="cpu")
        torch.cuda.synchronize()
        q.put((rank, blk.y0, blk.y1, blk.x0, blk.x1, T.cpu().numpy(), rounds, None))
        fim.close()
        ctx.close()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, 0, 0, 0, 0, None, 0, _why(rank, e)))
    finally:
        dist.destroy_process_group()


def _volume5(H, W, goal):
    """a z-padded [H][W][5] volume as the planner builds its FM3D volumes (Coupled_motion_planner.py:
    355-356): +inf first / last layers, three locomotion-mode layers of terrain-like cost"""
    rng = np.random.default_rng(23)
    c = rng.uniform(1, 5, (H, W, 3))
    c[rng.random((H, W, 3)) < 0.08] = np.inf
    c[:, : W // 2, 0] *= 0.3
    c[:, W // 2:, 2] *= 0.3
    inf = np.full((H, W, 1), np.inf)
    v = np.concatenate([inf, c, inf], axis=2)
    v[goal[1], goal[0], goal[2]] = 1.0
    return v


def test_c5_split_2x1_processes():
    """SURVEY §8(e), C5 across GPUs: a 1024^2 x 3 fp64 volume (z-padded to 5) split 2 x 1 over two
    processes sharing cuda:0, layers together, the relaunch schedule over gloo.  The assembled field
    equals the single-domain layered solve (eik_tmap3d): masks equal, <= 1e-11 relative."""
    import torch.multiprocessing as mp

    import eikonal

    world, H, W = 2, 1024, 1024
    goal = (W // 3, H // 2, 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_layered_worker, args=(r, world, port, H, W, goal, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [x[-1] for x in parts if x[-1]]
    assert not errs, "\n".join(errs)
    Tdd = np.full((H, W, 5), np.nan)
    for _, y0, y1, x0, x1, Tb, rounds, _ in parts:
        Tdd[y0:y1, x0:x1] = Tb
        assert rounds >= 2
    vol = _volume5(H, W, goal)
    ectx = eikonal.Context(0)
    try:
        ref = ectx.tmap3d(vol, np.array(goal), dtype=np.float64)
    finally:
        ectx.close()
    inner = (slice(None), slice(None), slice(1, 4))
    Tdd, ref = Tdd[inner], ref[inner]
    fin = np.isfinite(ref)
    assert fin.mean() > 0.5
    assert np.array_equal(np.isfinite(Tdd), fin)
    rel = np.abs(Tdd[fin] - ref[fin]) / np.maximum(ref[fin], 1e-30)
    assert rel.max() <= 1e-11, rel.max()


def _layered_live_worker(rank, world, port, H, W, goal, q, f64):
    """One rank of a C5-style volume split in x-y on the LIVE schedule: eikonal.Fim3dLayered on its
    block, the layered kernel's halo agent storing nl values per edge cell into the neighbours'
    hipIpc strips (dd.IpcHalo with nl x the element size), the per-round vote over shared memory."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "planning-motion_planning_amd"))
    import torch.distributed as dist

    import eikonal
    from eikonal import _lib as L
    from eikonal import dd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        px, py = dd.SPLITS[world]
        blk = dd.Block(H, W, px, py, rank)
        dt = torch.float64 if f64 else torch.float32
        vol = _volume5(H, W, goal)
        c = torch.from_numpy(np.ascontiguousarray(vol[blk.y0:blk.y1, blk.x0:blk.x1])).to(dev, dt)
        T = torch.empty_like(c)
        ctx = eikonal.Context(0)
        ctx.set_option(L.OPT_GRID, max(2, 3 * torch.cuda.get_device_properties(dev).multi_processor_count // (4 * world)))
        ctx.set_option(L.OPT_QTIMEOUT, 20.0)
        nl = 3
        _, _, ghost = dd.make_strips(blk, dt, dev, float("inf"), per_cell=nl)
        fim = eikonal.Fim3dLayered(ctx, blk.h, blk.w, 5, 1, nl, L.EIK_F64 if f64 else L.EIK_F32)
        loc = dd.LiveGpuLocalLayered(fim, ghost)
        halo = dd.IpcHalo(ctx, blk, (8 if f64 else 4) * nl)
        vote = dd.NodeVote() if world > 2 else None
        lg = blk.local_goal(goal[0], goal[1])
        res = []
        for _ in range(2):  # twice: the strips and the solver are reused
            loc.start(c, T, (lg[0], lg[1], goal[2]), torch.cuda.current_stream(dev).cuda_stream)
            rounds = dd.solve_live(loc, blk, halo, vote=vote)
            torch.cuda.synchronize()
            res.append(T.cpu().double().numpy())
        dist.barrier()
        halo.close()
        if vote is not None:
            vote.close()
        q.put((rank, blk.y0, blk.y1, blk.x0, blk.x1, res, rounds, None))
        fim.close()
        ctx.close()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, 0, 0, 0, 0, None, 0, _why(rank, e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,f64", [(2, True), (4, True), (4, False)])
def test_c5_split_live_processes(world, f64):
    """SURVEY §8(e), C5 across GPUs on the LIVE schedule (round 6): a 768 x 1024 x 3 volume (z-padded
    to 5) split 2 x 1 / 2 x 2 over processes sharing cuda:0, one persistent layered launch per block
    whose halo agent exchanges nl values per edge cell while the block solves.  The assembled field
    equals the single-domain layered solve (eik_tmap3d): masks equal, <= 1e-11 (fp64) / 1e-5 (fp32)
    relative, twice in a row on the same solvers and strips."""
    import torch.multiprocessing as mp

    import eikonal

    H, W = 768, 1024
    goal = (W // 3, H // 2, 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_layered_live_worker, args=(r, world, port, H, W, goal, q, f64)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [x[-1] for x in parts if x[-1]]
    assert not errs, "\n".join(errs)
    vol = _volume5(H, W, goal)
    if not f64:
        vol = vol.astype(np.float32).astype(np.float64)
    ectx = eikonal.Context(0)
    try:
        ref = ectx.tmap3d(vol if f64 else vol.astype(np.float32), np.array(goal),
                          dtype=np.float64 if f64 else np.float32).astype(np.float64)
    finally:
        ectx.close()
    inner = (slice(None), slice(None), slice(1, 4))
    for k in range(2):
        Tdd = np.full((H, W, 5), np.nan)
        for _, y0, y1, x0, x1, res, rounds, _ in parts:
            Tdd[y0:y1, x0:x1] = res[k]
            assert rounds >= 2
        Tk, R = Tdd[inner], ref[inner]
        fin = np.isfinite(R)
        assert fin.mean() > 0.5
        assert np.array_equal(np.isfinite(Tk), fin)
        rel = np.abs(Tk[fin] - R[fin]) / np.maximum(R[fin], 1e-30)
        assert rel.max() <= (1e-11 if f64 else 1e-5), rel.max()
