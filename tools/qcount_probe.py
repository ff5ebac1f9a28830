"""Queue-counter probe of one throughput config (EIK_QDEBUG library: `make -C csrc FIMFLAGS=-DEIK_QDEBUG=1
OUT=../lib_qd/libeikonal.so BUILD=../build_qd`, selected with EIKONAL_LIB).  Solves C4 at one GPU
(16384^2, seed 7) or C3 (128 x 1024^2) like bench.py and prints the solve's eik_stats and queue
counters (fim_engine.hpp qcount: 0 FIFO slot polls, 1 tail polls, 2 band dispatch attempts, 3 / 4
claims won / stale, 5 dispatches that moved entries, 6 decrease-key entries, 7 band entries put),
for the attribution of the PMC traffic above the algorithmic bytes.

  EIKONAL_LIB=planning-motion_planning_amd/lib_qd/libeikonal.so python tools/qcount_probe.py C4 f64
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
import bench  # noqa: E402
import eikonal  # noqa: E402
from eikonal import _lib as L  # noqa: E402
from eikonal import terrain  # noqa: E402

NAMES = ["slot_polls", "tail_polls", "dispatch_attempts", "claims", "stale", "dispatches", "decrease_key", "band_puts"]


def main():
    cfg, dt = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream(dev)
    ctx = eikonal.Context(0, options=L.options_from_env())
    f64 = dt == "f64"
    tdt, edt = (torch.float64, L.EIK_F64) if f64 else (torch.float32, L.EIK_F32)
    if cfg == "C4":
        N = 16384
        cost = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).to(tdt).contiguous()
        goals = [(N // 2, N // 2)]
        fim = eikonal.Fim2d(ctx, 1, N, N, edt)
    else:
        B, N = 128, 1024
        cost = torch.empty((B, N, N), dtype=tdt, device=dev)
        goals = []
        for b in range(B):
            cost[b] = terrain.cost_block(0, 0, N, N, N, N, seed=1000 + b, device=dev).to(tdt)
            goals.append(bench.c3_goal(cost[b], b, N))
        fim = eikonal.Fim2d(ctx, B, N, N, edt)
    T = torch.empty_like(cost)
    lib = L.lib()
    lib.eik_fim2d_qcount.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    out = []
    for _ in range(reps):
        fim.solve(cost.data_ptr(), T.data_ptr(), goals, st.cuda_stream)
        torch.cuda.synchronize()
        q = (C.c_uint64 * 8)()
        lib.eik_fim2d_qcount(fim._h, q)
        s = fim.stats()
        out.append({"tile_visits": s["tile_visits"], "inplace_passes": s["inplace_passes"],
                    "fresh_visits": s["fresh_visits"], "solve_ms": s["solve_ms"],
                    **{NAMES[i]: int(q[i]) for i in range(8)}})
    print(json.dumps({"config": cfg, "dtype": dt, "lib": os.environ.get("EIKONAL_LIB", "lib"), "solves": out}))


if __name__ == "__main__":
    main()
