"""Priority-band diagnostics (EIK_QDEBUG build): C2 fp64 solves with EIK_OPT_PRIO values, their
time, visits / passes and the queue counters (band claims, stale drops, lost CASes, FIFO claims,
FIFO stale, rescues, decrease-key entries, band puts).
  EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so python tools/prio_probe.py 0 250"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import eikonal  # noqa: E402
from eikonal import _lib as L  # noqa: E402
from eikonal import terrain  # noqa: E402

N = int(os.environ.get("N", "4096"))
dev = torch.device("cuda", 0)
cost = terrain.cost_block(0, 0, N, N, N, N, seed=42 if N == 4096 else 7, device=dev).double().contiguous()
T = torch.empty_like(cost)
lib = L.lib()
lib.eik_fim2d_qcount.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
names = ["-", "-", "-", "fifo_ok", "fifo_stale", "dispatches", "dup_push", "band_put"]
cf = cost[torch.isfinite(cost) & (cost > 0)]
print(f"cost geomean {float(torch.exp(torch.log(cf).mean())):.3f}: band width = multiplier x {64 * float(torch.exp(torch.log(cf).mean())):.1f}",
      flush=True)
for p in [float(v) for v in sys.argv[1:]]:
    ctx = eikonal.Context(0)
    ctx.set_option(L.OPT_PRIO, p)
    ctx.set_option(L.OPT_QTIMEOUT, 3.0)  # a stuck queue ends in an error, not a long hang
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F64)
    s = torch.cuda.current_stream(dev).cuda_stream
    fim.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], s)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fim.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], s)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    st = fim.stats()
    q = (C.c_uint64 * 8)()
    lib.eik_fim2d_qcount(fim._h, q)
    print(f"PRIO={p}: {np.median(ts) * 1e3:.3f} ms visits {st['tile_visits']} passes {st['inplace_passes']} "
          + " ".join(f"{n}={q[i]}" for i, n in enumerate(names)), flush=True)
    fim.close()
    ctx.close()
