"""Layered solver (C5, 4096^2 x 3 z-padded volume of bench.py) under in-place pass caps."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal
from eikonal import terrain, _lib as L

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
ctx = eikonal.Context(0)
N = 4096
c0 = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
inf = torch.full_like(c0, float("inf"))
c1 = torch.where(c0 > 100, inf, 1.6 * c0)
yy = torch.arange(N, device=dev)[:, None] // 64
xx = torch.arange(N, device=dev)[None, :] // 64
c2 = torch.where(((yy + 2 * xx) % 5) == 0, inf, 0.8 * c0)
cost = torch.stack([inf, c0, c1, c2, inf], dim=-1).contiguous()
T = torch.empty_like(cost)
g = np.array([N // 2, N // 2, 1], np.int64)
for p in (8, 16, 24, 8, 16, 24):
    ctx.set_option(L.OPT_PASSES, p)
    solve = lambda: ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cost.data_ptr(), T.data_ptr(), N, N, 5, L.EIK_F32, g,
                                                     st.cuda_stream))
    solve()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        solve()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    s = ctx.stats()
    print(f"C5 passes={p}: {ms:.3f} ms  {3 * N * N / ms / 1e6:.3f} Gcells/s  visits {s['tile_visits']}", flush=True)
