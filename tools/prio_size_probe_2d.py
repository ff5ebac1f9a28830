"""fp64 2D single-map solves (the DEM-derived raster, goal at the centre) at several sizes under
EIK_OPT_PRIO widths: does default_prio's 0.25 x max(1, sqrt(H W) / 4096) hold between and below the
C2 / C4 sizes?  python tools/prio_size_probe_2d.py [N ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bench import L, eikonal, terrain  # noqa: E402

sizes = [int(s) for s in sys.argv[1:]] or [1024, 2048, 8192]
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
widths = os.environ.get("WIDTHS", "-1,0,0.25,0.5,1").split(",")
for N in sizes:
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).double().contiguous()
    T = torch.empty_like(cost)
    goal = (N // 2, N // 2)
    steps = max(3, int(2e9 // (N * N * 8)))
    for w in widths:
        ctx = eikonal.Context(0, options={"PRIO": float(w)})
        try:
            fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F64)
            solve = lambda: fim.solve(cost.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)  # noqa: E731
            sec = bench.timed_loop(solve, steps)
            st = fim.stats()
            print(f"f64 N={N} PRIO={w}: {N * N / sec / 1e9:.3f} Gcells/s {sec * 1e3:.3f} ms vis {st['tile_visits']} "
                  f"inpl {st['inplace_passes']}", flush=True)
            fim.close()
        finally:
            ctx.close()
    del cost, T
    torch.cuda.empty_cache()
