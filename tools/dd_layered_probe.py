"""Layered decomposition blocks (the in-process rounds schedule of tests/test_gpu_dd.py
solve_blocks_layered over blocks of a few-layer volume) with the FIFO against the default priority
bands: rounds, summed tile visits / in-place passes, wall time.  python tools/dd_layered_probe.py [N px py]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal  # noqa: E402
from eikonal import _lib as L  # noqa: E402
from eikonal import dd  # noqa: E402

OPP = {0: 1, 1: 0, 2: 3, 3: 2}


def volume(H, W, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(1, 5, (H, W, 3))
    c[rng.random((H, W, 3)) < 0.08] = np.inf
    c[:, : W // 2, 0] *= 0.3
    c[:, W // 2:, 2] *= 0.3
    inf = np.full((H, W, 1), np.inf)
    return np.concatenate([inf, c, inf], axis=2)


def solve(cost, goal, px, py, f64, options):
    dev = torch.device("cuda", 0)
    H, W, Lz = cost.shape
    ctx = eikonal.Context(0, options=options)
    dt = torch.float64 if f64 else torch.float32
    blocks = [dd.Block(H, W, px, py, r) for r in range(px * py)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    locs, sends, recvs = [], [], []
    for b in blocks:
        c = torch.from_numpy(np.ascontiguousarray(cost[b.y0:b.y1, b.x0:b.x1])).to(dev, dt)
        send, recv, ghost = dd.make_strips(b, dt, dev, float("inf"), per_cell=3)
        fim = eikonal.Fim3dLayered(ctx, b.h, b.w, Lz, 1, 3, L.EIK_F64 if f64 else L.EIK_F32)
        loc = dd.GpuLocalLayered(fim, ghost)
        T = torch.empty_like(c)
        lg = b.local_goal(goal[0], goal[1])
        loc.start(c, T, (lg[0], lg[1], goal[2]), stream)
        locs.append((loc, c, T)), sends.append(send), recvs.append(recv)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for rounds in range(1, 100000):
        for (loc, _, _), send in zip(locs, sends):
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
        if sum(loc.active() for loc, _, _ in locs) == 0:
            break
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    st = [loc.fim.stats() for loc, _, _ in locs]
    ctx.close()
    return rounds, sum(s["tile_visits"] for s in st), sum(s["inplace_passes"] for s in st), ms


N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
px = int(sys.argv[2]) if len(sys.argv) > 2 else 2
py = int(sys.argv[3]) if len(sys.argv) > 3 else 2
cost = volume(N, N, 7)
goal = (N // 3, N // 2, 2)
cost[goal[1], goal[0], goal[2]] = 1.0
for f64 in (True, False):
    for opts in ({"PRIO": 0.0}, None, {"PRIO": 0.0}, None):
        rounds, vis, passes, ms = solve(cost, goal, px, py, f64, opts)
        print(f"{'f64' if f64 else 'f32'} {N}^2x3 {px}x{py} {'FIFO ' if opts else 'bands'}: rounds {rounds} "
              f"visits {vis} passes {passes} {ms:.1f} ms (the rounds loop, host-driven)", flush=True)
