"""Compare the solver drivers (list / persistent, grid sizes) on the bench DEM: time, visits, field agreement."""
import sys, time, numpy as np
sys.path.insert(0, 'planning-motion_planning_amd')
import torch
import eikonal
from eikonal import terrain, _lib as L

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
ctx = eikonal.Context(0)
for N in [int(x) for x in (sys.argv[1:] or ["4096"])]:
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).contiguous()
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
    ref = None
    for mode, grid in ((L.MODE_LIST, 0), (L.MODE_PERSISTENT, 0), (L.MODE_PERSISTENT, 512), (L.MODE_PERSISTENT, 256)):
        ctx.set_option(L.OPT_MODE, mode)
        ctx.set_option(L.OPT_GRID, grid)
        T = torch.empty_like(cost)
        for _ in range(2):
            fim.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], s)
        torch.cuda.synchronize()
        K = 10
        t0 = time.perf_counter()
        for _ in range(K):
            fim.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], s)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / K * 1e3
        st = fim.stats()
        Th = T.cpu().numpy()
        if ref is None:
            ref = Th
        fin = np.isfinite(ref)
        same = np.array_equal(fin, np.isfinite(Th))
        rel = float((np.abs(Th[fin] - ref[fin]) / np.maximum(ref[fin], 1e-30)).max())
        print(f"N={N} mode={mode} grid={grid}: {el:.3f} ms/solve  {N*N/el/1e6:.2f} Gcells/s  launches={st['iterations']} "
              f"visits={st['tile_visits']} solve_ms={st['solve_ms']:.3f} mask_same={same} maxrel_vs_list={rel:.2e}",
              flush=True)
    ctx.set_option(L.OPT_GRID, 0)
