"""Ordered (delta-window) list-mode scheduling vs the persistent FIFO on the bench DEM: time, visits."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, 'planning-motion_planning_amd')
import eikonal
from eikonal import terrain, _lib as L

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
ctx = eikonal.Context(0)
N = 4096
cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
T = torch.empty_like(cost)
for mode, delta in ((L.MODE_PERSISTENT, 0), (L.MODE_LIST, 0), (L.MODE_LIST, 100000), (L.MODE_LIST, 30000), (L.MODE_LIST, 10000), (L.MODE_LIST, 3000), (L.MODE_LIST, 1000), (L.MODE_LIST, 300)):
    ctx.set_option(L.OPT_MODE, mode)
    ctx.set_option(L.OPT_DELTA, delta)
    for _ in range(2):
        fim.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = 5
    for _ in range(K):
        fim.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], s)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / K * 1e3
    st = fim.stats()
    print(f"mode={mode} delta={delta}: {el:.3f} ms  launches={st['iterations']} visits={st['tile_visits']} "
          f"inplace={st['inplace_passes']}", flush=True)
print("Tmax", float(T[torch.isfinite(T)].max()))
Tf = T[torch.isfinite(T)]
print(f"T max {Tf.max().item():.1f} median {Tf.median().item():.1f}  cost median {cost[torch.isfinite(cost)].median().item():.2f}")
