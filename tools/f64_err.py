"""Max abs error of the fp64 C2 field (4096^2 DEM, goal centre) against the oracle's FMM, per library
build (EIKONAL_LIB).  Test infrastructure (imports the oracle)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np, torch
import eikonal, oracle as O
from eikonal import _lib as L, terrain
dev = torch.device("cuda", 0)
N = 4096
cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).double().contiguous()
O.set_strict(False)
R = O.fmm2d(cost.cpu().numpy(), (N // 2, N // 2))
fin = np.isfinite(R)
for lib in sys.argv[1:]:
    os.environ["EIKONAL_LIB"] = lib
    import subprocess
    code = f"""
import sys, numpy as np, torch
sys.path.insert(0, {os.path.join(ROOT, 'planning-motion_planning_amd')!r})
import eikonal
from eikonal import _lib as L, terrain
dev = torch.device('cuda', 0)
N = {N}
cost = terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).double().contiguous()
T = torch.empty_like(cost)
ctx = eikonal.Context(0)
f = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F64)
f.solve(cost.data_ptr(), T.data_ptr(), [(N // 2, N // 2)], torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
np.save('/tmp/Tg.npy', T.cpu().numpy())
"""
    subprocess.run([sys.executable, "-c", code], check=True, env=dict(os.environ, EIKONAL_LIB=lib))
    Tg = np.load("/tmp/Tg.npy")
    err = np.abs(Tg[fin] - R[fin])
    print(f"{lib}: masks equal {np.array_equal(np.isfinite(Tg), fin)}, max abs {err.max():.3e}, "
          f"p99.99 {np.quantile(err, 0.9999):.3e}, max T {R[fin].max():.1f}", flush=True)
