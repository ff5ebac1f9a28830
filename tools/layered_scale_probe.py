"""Layered solver (C5's volume: 3 modes + inf padding, bench.bench_layers) at 4096^2 / 8192^2 /
16384^2 under EIK_OPT_PRIO widths: does the layered band width hold on larger rasters (the 2D
solver's C4 collapses at narrow widths)?  python tools/layered_scale_probe.py [f32|f64] [N ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bench import eikonal, terrain  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "f32"
sizes = [int(s) for s in sys.argv[2:]] or [4096, 8192, 16384]
tdt = torch.float64 if dt == "f64" else torch.float32
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
widths = os.environ.get("WIDTHS", "0,0.25,0.5,1,2").split(",")
for N in sizes:
    seed = int(os.environ.get("SEED", "7"))
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=seed, device=dev).to(tdt).contiguous()
    goal = (N // 2, N // 2)
    for w in widths:
        ctx = eikonal.Context(0, options={"PRIO": float(w)})
        try:
            r = bench.bench_layers(ctx, dev, stream, cost, goal, 3)
            print(f"{dt} N={N} PRIO={w}: {r['value']} Gcells/s {r['ms_per_step']} ms vis {r.get('tile_visits_per_solve')} "
                  f"inpl {r['roofline'].get('inplace_passes_per_solve')} reach {r['reached_fraction']} seed {seed}",
                  flush=True)
        finally:
            ctx.close()
        torch.cuda.empty_cache()
    del cost
    torch.cuda.empty_cache()
