"""Multi-rank domain decomposition on CPU (gloo): the halo-exchange drivers of eikonal/dd.py
(dd.solve rounds and the dd.solve_live protocol over P2PHalo), run with 2, 4 and 8 ranks (the
bench's 2x1 / 2x2 / 4x2 splits) on blocks of one raster, must converge to the single-domain
solution (the oracle FMM field, <= 1e-9 abs: same Godunov fixed point).  The GPU bench plugs the HIP solver
into the same driver over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from eikonal import dd


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cost(H, W, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 6, (H, W))
    c[rng.random((H, W)) < 0.12] = np.inf
    c[0, :] = c[-1, :] = c[:, 0] = c[:, -1] = np.inf
    return c


def _worker(rank, world, port, H, W, goal, seed, q, live=False):
    from dd_cpu import CpuLocal

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    px, py = dd.SPLITS[world]
    blk = dd.Block(H, W, px, py, rank)
    cost = _cost(H, W, seed)[blk.y0:blk.y1, blk.x0:blk.x1]
    send, recv, ghost = dd.make_strips(blk, torch.float64, "cpu", float("inf"))
    loc = CpuLocal(cost, ghost)
    loc.start(blk.local_goal(*goal))
    if live:
        vote = dd.NodeVote() if live == "node" else None
        halo = dd.P2PHalo(blk, torch.float64, "cpu")
        rounds = dd.solve_live(loc, blk, halo, group=dd.control_group(), vote=vote)
        if vote is not None:  # a second solve on the same vote (round numbers carry on)
            loc.start(blk.local_goal(*goal))
            assert dd.solve_live(loc, blk, halo, vote=vote) == rounds
            vote.close()
    else:
        rounds = dd.solve(loc, blk, send, recv, exchange_every=4)
    q.put((rank, blk.y0, blk.y1, blk.x0, blk.x1, loc.T, rounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("live", [False, True, "node"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_dd_matches_single_domain(world, live):
    H, W, seed = 48, 70, 3
    goal = (9, 30)
    c = _cost(H, W, seed)
    c[goal[1], goal[0]] = 2.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, goal, seed, q, live)) for r in range(world)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = np.full((H, W), np.nan)
    for _, y0, y1, x0, x1, Tb, rounds in parts:
        T[y0:y1, x0:x1] = Tb
        assert rounds >= 2  # the front crossed at least one rank boundary
    O.set_strict(False)
    try:
        cc = c.copy()
        R = O.fmm2d(cc, goal)
    finally:
        O.set_strict(True)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin)
    assert np.abs(T[fin] - R[fin]).max() <= 1e-9


def _worker_layered(rank, world, port, H, W, goal, q):
    from dd_cpu import CpuLocalLayered

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    px, py = dd.SPLITS[world]
    blk = dd.Block(H, W, px, py, rank)
    c = _cost3(H, W)
    cost = c[blk.y0:blk.y1, blk.x0:blk.x1, 1:4]  # the three solved layers of the z-padded volume
    nl = cost.shape[2]
    send, recv, ghost = dd.make_strips(blk, torch.float64, "cpu", float("inf"), per_cell=nl)
    loc = CpuLocalLayered(cost, ghost)
    lg = blk.local_goal(goal[0], goal[1])
    loc.start((lg[0], lg[1], goal[2] - 1))
    rounds = dd.solve(loc, blk, send, recv, exchange_every=4)
    q.put((rank, blk.y0, blk.y1, blk.x0, blk.x1, loc.T, rounds))
    dist.barrier()
    dist.destroy_process_group()


def _cost3(H, W):
    """a z-padded 3-layer volume as the planner builds its FM3D volumes (Coupled_motion_planner.py:
    355-356): +inf first / last layers; mode 1 cheap on the left, mode 2 on the right"""
    rng = np.random.default_rng(9)
    c = rng.uniform(1, 4, (H, W, 3))
    c[rng.random((H, W, 3)) < 0.1] = np.inf
    c[:, : W // 2, 0] *= 0.3
    c[:, W // 2:, 1] *= 0.3
    inf = np.full((H, W, 1), np.inf)
    return np.concatenate([inf, c, inf], axis=2)


@pytest.mark.parametrize("world", [2, 4])
def test_dd_layered_matches_single_domain(world):
    """SURVEY §8(e), C5 across ranks: a few-layer volume split in x-y with its layers kept together
    (strips of nl values per edge cell, dd.make_strips(per_cell=nl)); the rounds driver over gloo
    must give the oracle's FM3D field (FastMarching3D.py:126-145) within 1e-9."""
    H, W = 36, 44
    goal = (30, 9, 2)
    c = _cost3(H, W)
    c[goal[1], goal[0], goal[2]] = 1.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker_layered, args=(r, world, port, H, W, goal, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = np.full((H, W, 5), np.inf)
    for _, y0, y1, x0, x1, Tb, rounds in parts:
        T[y0:y1, x0:x1, 1:4] = Tb
        assert rounds >= 2
    O.set_strict(False)
    try:
        R = O.fmm3d(c, np.array(goal), None)
    finally:
        O.set_strict(True)
    fin = np.isfinite(R)
    assert np.array_equal(np.isfinite(T), fin)
    assert np.abs(T[fin] - R[fin]).max() <= 1e-9


def test_block_partition_covers_raster():
    for world, (px, py) in dd.SPLITS.items():
        H, W = 100, 130
        cov = np.zeros((H, W), int)
        for r in range(world):
            b = dd.Block(H, W, px, py, r)
            cov[b.y0:b.y1, b.x0:b.x1] += 1
            for s, nb in enumerate(b.nb):
                if nb is not None:  # neighbour relation is symmetric
                    opp = {0: 1, 1: 0, 2: 3, 3: 2}[s]
                    assert dd.Block(H, W, px, py, nb).nb[opp] == r
        assert (cov == 1).all()
