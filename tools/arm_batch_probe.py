"""The bench's 16-volume FM3D batch (bench_arm) before and after the costmap extra: wall time and
the solve's device time / visits, to see what the costmap run leaves behind."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import numpy as np, torch
import eikonal
import bench

dev = torch.device("cuda", 0)
ctx = eikonal.Context(0)
stream = torch.cuda.current_stream(dev)
cap = {}
orig = ctx.tmap3d_batch


def batch(costs, goals):
    cap["a"] = (costs, goals)
    return orig(costs, goals)


ctx.tmap3d_batch = batch


def measure(tag):
    costs, goals = cap["a"]
    for _ in range(3):
        t0 = time.perf_counter()
        orig(costs, goals)
        el = (time.perf_counter() - t0) * 1e3
        s = ctx.stats()
        print(f"{tag}: wall {el:.2f} ms, device {s['solve_ms']:.2f} ms, visits {s['tile_visits']}, "
              f"passes {s['inplace_passes']}, launches {s['iterations']}", flush=True)


bench.bench_arm(ctx, 2)
measure("before costmap")
goal = (2048, 2048)
bench.bench_costmap(ctx, dev, stream, 2, goal)
measure("after costmap")
