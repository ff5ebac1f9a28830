"""Diagnose fp32 error of the live-DD test case (tests/test_gpu_dd_live.py, 300 x 520, seed 9):
is a large relative error rounding (the field is a fixed point of the local solve) or a missed
update (some cell stays above the local solve of its neighbours)?  Runs the single-domain
persistent solve under the given EIK_OPTIONS variants, then REPS 4-rank live solves.
  python tools/dd_live_diag.py [REPS]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "planning-motion_planning_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def residual(T, c):
    """(T - local solve of its own neighbours) / T over reached non-goal cells, fp64."""
    inf = np.inf
    P = np.pad(T, 1, constant_values=inf)
    a = np.minimum(P[1:-1, :-2], P[1:-1, 2:])
    b = np.minimum(P[:-2, 1:-1], P[2:, 1:-1])
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    with np.errstate(invalid="ignore", over="ignore"):
        d = hi - lo
        two = 0.5 * (a + b + np.sqrt(np.clip(2 * c * c - d * d, 0, None)))
        w = np.where(c < d, lo + c, two)
        w = np.where(np.isinf(lo), inf, w)
        fin = np.isfinite(T) & (T > 0)
        return np.where(fin, (T - w) / np.where(fin, T, 1.0), 0.0)


def report(tag, T, R, c):
    fin = np.isfinite(R)
    same = np.array_equal(np.isfinite(T), fin)
    rel = np.where(fin, np.abs(T - R) / np.maximum(np.where(fin, R, 1.0), 1e-30), 0.0)
    k = np.unravel_index(np.argmax(rel), rel.shape)
    res = residual(T, c)
    kr = np.unravel_index(np.argmax(np.abs(res)), res.shape)
    print(f"{tag}: masks {'equal' if same else 'DIFFER'}; max rel {rel.max():.3e} at y,x={k} "
          f"(T {T[k]:.6f} R {R[k]:.6f}, sign {np.sign(T[k] - R[k]):+.0f}); cells rel>1e-5: {(rel > 1e-5).sum()}; "
          f"fixed-point residual max {res.max():.3e} min {res.min():.3e} at {kr}", flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    import torch.multiprocessing as mp

    import eikonal
    from eikonal import _lib as L
    import test_gpu_dd_live as TL

    H, W, seed = 300, 520, 9
    goal = (W // 4, H // 2)
    cost = TL._cost(H, W, seed, goal)
    c32 = cost.astype(np.float32).astype(np.float64)
    R = TL._oracle(c32, goal)
    dev = torch.device("cuda", 0)
    for opts in ("", "SCHED=0", "PASSES=1"):
        os.environ["EIK_OPTIONS"] = opts
        ctx = eikonal.Context(0, options=eikonal._lib.options_from_env())
        ctx.set_option(L.OPT_MODE, L.MODE_PERSISTENT)
        c = torch.from_numpy(c32).to(dev, torch.float32)
        T = torch.empty_like(c)
        fim = eikonal.Fim2d(ctx, 1, H, W, L.EIK_F32)
        for g in (None, 160):
            if g:
                ctx.set_option(L.OPT_GRID, g)
            fim.solve(c.data_ptr(), T.data_ptr(), goal, torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize()
            report(f"single [{opts or 'defaults'}] grid {g or 'full'}", T.cpu().double().numpy(), R, c32)
        ctx.close()
    os.environ["EIK_OPTIONS"] = ""
    for world in (2, 4):
        for rep in range(reps):
            q = mp.get_context("spawn").Queue()
            port = TL._port()
            procs = [mp.get_context("spawn").Process(target=TL._ipc_worker,
                                                     args=(r, world, port, H, W, goal, seed, q, False))
                     for r in range(world)]
            for p in procs:
                p.start()
            parts = [q.get(timeout=240) for _ in range(world)]
            for p in procs:
                p.join(timeout=60)
            errs = [x[-1] for x in parts if x[-1]]
            if errs:
                print("worker errors", errs)
                return 1
            for k in range(2):
                T = np.full((H, W), np.nan)
                for _, y0, y1, x0, x1, res, rounds, _ in parts:
                    T[y0:y1, x0:x1] = res[k]
                blocks = [(y0, y1, x0, x1) for _, y0, y1, x0, x1, *_ in parts]
                report(f"live world {world} rep {rep} solve {k} blocks {blocks}", T, R, c32)
    return 0


if __name__ == "__main__":
    sys.exit(main())
