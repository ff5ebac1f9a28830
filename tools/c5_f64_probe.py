"""C5 (4096^2 x 3 layered costmap, z padded to 5) in fp64: the general 3D solver (fim3d.hip, the
drop-in's default precision) -- time and agreement with the fp32 layered solver."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import numpy as np, torch
import eikonal
from eikonal import _lib as L, terrain

dev = torch.device("cuda", 0)
N = int(os.environ.get("N", "4096"))
ctx = eikonal.Context(0, options=os.environ.get("OPTS", ""))
stream = torch.cuda.current_stream(dev)
c0 = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).double()
inf = torch.full_like(c0, float("inf"))
c1 = torch.where(c0 > 100, inf, 1.6 * c0)
yy = torch.arange(N, device=dev)[:, None] // 64
xx = torch.arange(N, device=dev)[None, :] // 64
c2 = torch.where(((yy + 2 * xx) % 5) == 0, inf, 0.8 * c0)
goal = np.array([N // 2, N // 2, 1], np.int64)
for dt, tdt in ((L.EIK_F32, torch.float32), (L.EIK_F64, torch.float64)):
    cost = torch.stack([inf, c0, c1, c2, inf], dim=-1).to(tdt).contiguous()
    T = torch.empty_like(cost)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cost.data_ptr(), T.data_ptr(), N, N, 5, dt, goal, stream.cuda_stream))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        s = ctx.stats()
        print(f"dtype {dt}: {el*1e3:.1f} ms ({N*N*3/el/1e9:.3f} Gcells/s over 3 layers), visits {s['tile_visits']}, "
              f"passes {s['inplace_passes']}, launches {s['iterations']}", flush=True)
    if dt == L.EIK_F32:
        T32 = T.double()
    else:
        fin = torch.isfinite(T32)
        print("masks equal", bool(torch.equal(fin, torch.isfinite(T))), "max rel fp32 vs fp64",
              float(((T32[fin] - T[fin]).abs() / T[fin].clamp_min(1e-30)).max()), flush=True)
