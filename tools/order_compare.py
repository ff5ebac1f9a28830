"""Ordered (delta-window) list mode vs the persistent FIFO on the throughput-bound configs:
C3 (batch 128 x 1024^2) and C4 at one GPU (16384^2): time, visits, in-place passes."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, 'planning-motion_planning_amd')
import eikonal
from eikonal import terrain, _lib as L

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
ctx = eikonal.Context(0)


def run(name, fim, cost, T, goals, K=3):
    for mode, delta in ((L.MODE_PERSISTENT, 0), (L.MODE_LIST, 0), (L.MODE_LIST, 3000), (L.MODE_LIST, 1000),
                        (L.MODE_LIST, 300), (L.MODE_LIST, 100)):
        ctx.set_option(L.OPT_MODE, mode)
        ctx.set_option(L.OPT_DELTA, delta)
        fim.solve(cost.data_ptr(), T.data_ptr(), goals, s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fim.solve(cost.data_ptr(), T.data_ptr(), goals, s)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / K * 1e3
        st = fim.stats()
        print(f"{name} mode={mode} delta={delta}: {el:.2f} ms  {cost.numel() / el / 1e6:.2f} Gcells/s  "
              f"launches={st['iterations']} visits={st['tile_visits']} inplace={st['inplace_passes']}", flush=True)
    ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
    ctx.set_option(L.OPT_DELTA, 0)


B, N = 128, 1024
cost = torch.empty((B, N, N), dtype=torch.float32, device=dev)
rng = np.random.default_rng(1000)
goals = []
for b in range(B):
    cost[b] = terrain.cost_block(0, 0, N, N, N, N, seed=1000 + b, device=dev)
    while True:
        gx, gy = (int(v) for v in rng.integers(N // 8, N - N // 8, 2))
        if float(cost[b, gy, gx]) < 50:
            break
    goals.append((gx, gy))
T = torch.empty_like(cost)
fim = eikonal.Fim2d(ctx, B, N, N, L.EIK_F32)
run("C3", fim, cost, T, goals)
fim.close()
del cost, T
torch.cuda.empty_cache()
N = 16384
cost = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).contiguous()
T = torch.empty_like(cost)
fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
run("C4", fim, cost, T, [(N // 2, N // 2)], K=2)
