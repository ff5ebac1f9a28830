"""Priority-band ring probe (round 6): the 4 x 2 live split of the 4096^2 fp64
terrain raster (tests/test_gpu_dd_live.py's _terrain_worker: 8 processes on cuda:0, IPC strips, node
vote) with every band's ring forced to R slots (EIK_OPT_PRIO_RING), for a list of R.  Prints per R
whether the solve completed and, if not, the failing rank's error (its queue error word: bit 4 = a
ring lapped).  EIKONAL_LIB selects the library (the round-5 one in lib_alt for the A/B).

  python tools/ring_probe.py 512 256 128
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))


def run(ring, world=8, N=4096):
    import torch.multiprocessing as mp

    import test_gpu_dd_live as T

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = T._port()
    procs = [ctx.Process(target=T._terrain_worker, args=(r, world, port, N, q, ring)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = [q.get(timeout=200) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [x[-1] for x in parts if x[-1]]
    cause = [e for e in errs if "<-" in e]
    rounds = max((x[6] for x in parts), default=0)
    return (not errs), rounds, (cause or errs)[:2]


if __name__ == "__main__":
    lib = os.environ.get("EIKONAL_LIB", "lib/libeikonal.so")
    for r in [int(v) for v in sys.argv[1:]]:
        ok, rounds, errs = run(r)
        print(f"{lib} ring {r}: {'ok' if ok else 'FAILED'} rounds {rounds} {errs}", flush=True)
