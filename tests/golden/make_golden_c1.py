"""Golden fixtures for BASELINE.json configs[0] (C1): a 256 x 256 synthetic map, single goal at
(128, 128), solved by the reference's own src/FastMarching (uniform cost 1.0 and
U(1, 10) seed 0, +inf border), plus the reference's getPathGDM from (30, 40) to the goal.

Run ONCE in the build container (reference sources readable):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c1.py

The full field comes from the reference's updateNode / getMinNB driven by computeTmap's loop
(FastMarching.py:92-112 with a 3-value unpack: computeTmap itself raises at :107), as in
make_golden.py.  The reference's own failures (e.g. StopIteration on tied decrease-keys) are
recorded as data.  Output: c1.npz next to this script.
"""
import os
import sys
import time

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)
import make_golden as G  # noqa: E402  (imports the reference's FastMarching, read-only)


def main():
    t0 = time.time()
    out = {}
    n = 256
    goal, start = [128, 128], [30, 40]
    for name, cost in (("uniform", G.cost_uniform(n, n)), ("random", G.cost_random(n, n, 0))):
        T, err = G.run(G.ref_full_field, cost, goal)
        out[f"{name}_cost"] = cost.astype(np.float32)
        out[f"{name}_T"] = T[0] if T is not None else np.zeros((0, 0))
        out[f"{name}_err"] = np.array(err or "")
        path, perr = (None, "no field") if T is None else G.run(G.FM.getPathGDM, T[0], np.array(start),
                                                                 np.array(goal), 0.5)
        out[f"{name}_path"] = path if path is not None else np.zeros((0, 2))
        out[f"{name}_path_err"] = np.array(perr or "")
        print(f"{name}: err={err} path={None if path is None else path.shape} perr={perr} t={time.time() - t0:.1f}s",
              flush=True)
    out["goal"] = np.array(goal, np.int64)
    out["start"] = np.array(start, np.int64)
    np.savez_compressed(os.path.join(OUT, "c1.npz"), **out)


if __name__ == "__main__":
    main()
