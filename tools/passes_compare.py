"""In-place pass cap (EIK_OPT_PASSES) of the persistent driver, and the list driver, on C2 (4096^2
DEM), C3 (batch 128 x 1024^2) and C4 at one GPU (16384^2): time, visits, in-place passes."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, 'planning-motion_planning_amd')
import eikonal
from eikonal import terrain, _lib as L

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
ctx = eikonal.Context(0)
which = sys.argv[1:] or ["C2", "C3", "C4"]


def run(name, fim, cost, T, goals, K=5):
    import os
    caps = [int(v) for v in os.environ.get("PASSES", "0,8,2,16,0").split(",")]
    for mode, passes in [(L.MODE_PERSISTENT, p) for p in caps]:
        ctx.set_option(L.OPT_MODE, mode)
        ctx.set_option(L.OPT_PASSES, passes)
        fim.solve(cost.data_ptr(), T.data_ptr(), goals, s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fim.solve(cost.data_ptr(), T.data_ptr(), goals, s)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / K * 1e3
        st = fim.stats()
        print(f"{name} mode={mode} passes={passes}: {el:.3f} ms  {cost.numel() / el / 1e6:.2f} Gcells/s  "
              f"launches={st['iterations']} visits={st['tile_visits']} inplace={st['inplace_passes']}", flush=True)
    ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
    ctx.set_option(L.OPT_PASSES, 0)


if "C2" in which:
    N = 4096
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
    run("C2", fim, cost, T, [(N // 2, N // 2)], K=10)
    cu = torch.ones_like(cost)
    cu[0, :] = cu[-1, :] = cu[:, 0] = cu[:, -1] = float("inf")
    run("uniform4096", fim, cu, T, [(N // 2, N // 2)], K=10)
    fim.close()
    del cost, T, cu
if "C3" in which:
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
if "C4" in which:
    torch.cuda.empty_cache()
    N = 16384
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).contiguous()
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
    run("C4", fim, cost, T, [(N // 2, N // 2)], K=int(os.environ.get("C4K", "2")))
