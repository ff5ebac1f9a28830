"""Planner step 1 (eik_rover_path_f64, bench_costmap's query) under in-place pass caps: the two
fronts are ONE batch of B = 2 maps, whose default cap is the batch value (2)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import numpy as np, torch
import eikonal, planner
from eikonal import _lib as L, terrain

dev = torch.device("cuda", 0)
N, res = 4096, 0.05
Zh = terrain.dem_block(0, 0, N, N, seed=42, device=dev).double().contiguous().cpu().numpy()
g = (2048, 2048)
q = planner.query(res * (g[0] + 1), res * (g[1] + 1), res * (256 + 1), res * (256 + 1), 0.0, res, res * N)
for opts in os.environ.get("OPTS_LIST", ",PASSES=8,PASSES=24,,PASSES=8,PASSES=24").split(","):
    ctx = eikonal.Context(0, options=opts)
    ctx.rover_path(Zh, q)
    ts = []
    for _ in range(3):
        Zc = Zh.copy() if os.environ.get("FRESH") else Zh  # a fresh host array per plan, as the planner reads one
        t0 = time.perf_counter()
        r = ctx.rover_path(Zc, q)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"{opts or 'default'}: {np.median(ts):.2f} ms, waypoints {len(r[0])}, join {list(r[2])}, "
          f"fronts {ctx.fronts_info()}", flush=True)
    ctx.close()
if not os.environ.get("ROVER_ONLY"):
    # the two fronts alone on the planner's own cost raster (host entry, one B = 2 batch), and each
    # front as a single-map solve, with the solver stats
    import costmap
    cMap, _ = costmap.cost_map(Zh, res, res * N)
    cost = np.ascontiguousarray(cMap.T)
    gx, gy = 2048, 2048
    sx, sy = 256, 256
    ctx = eikonal.Context(0)
    for rep in range(3):
        cc = cost.copy() if os.environ.get("FRESH") else cost
        t0 = time.perf_counter()
        ctx.tmap2d_bidir(cc, (gx, gy), (sx, sy))
        s = ctx.stats()
        print(f"bidir batch: wall {(time.perf_counter() - t0) * 1e3:.2f} ms, solve {s['solve_ms']:.2f} ms, visits "
              f"{s['tile_visits']}, in-place {s['inplace_passes']}, fronts {ctx.fronts_info()}", flush=True)
    dc = torch.from_numpy(cost).to(dev)
    T = torch.empty_like(dc)
    f1 = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F64)
    for g in ((gx, gy), (sx, sy)):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f1.solve(dc.data_ptr(), T.data_ptr(), [g], torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize()
            s = ctx.stats()
            print(f"single front from {g}: {(time.perf_counter() - t0) * 1e3:.2f} ms, visits {s['tile_visits']}, "
                  f"in-place {s['inplace_passes']}", flush=True)
