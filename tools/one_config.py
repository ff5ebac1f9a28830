"""One bench config alone (no C2 line), for rocprofv3 --pmc passes whose launches must be only
that config's (the C2 and C3 / C4 solves share a kernel name):
  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -- python tools/one_config.py C3 f64 3
  python tools/pmc_traffic.py <dir_f> <dir_w> "fim2d_persist_kernel<double" f64 > profiles/pmc_traffic_c3.json
Prints the bench's entry for the config (one JSON object)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import eikonal  # noqa: E402
from eikonal import _lib as L  # noqa: E402


def main():
    cfg, dt = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)  # the stream the inputs are generated on (a side stream raced them)
    ctx = eikonal.Context(0, options=L.options_from_env())  # EIK_OPTIONS A/B hook
    tdt, edt = (torch.float64, L.EIK_F64) if dt == "f64" else (torch.float32, L.EIK_F32)
    if cfg == "C2":  # configs[1], the headline raster
        from eikonal import terrain
        cost = terrain.cost_block(0, 0, 4096, 4096, 4096, 4096, seed=42, device=dev).to(tdt).contiguous()
        out = bench.bench_c2(ctx, dev, stream, cost, (2048, 2048), steps, dt)
    elif cfg == "C3":
        out = bench.bench_batch(ctx, dev, stream, steps, tdt, edt)
    elif cfg == "C4":
        out = bench.bench_c4(ctx, dev, stream, steps, tdt, edt)
    else:
        raise SystemExit(f"unknown config {cfg}")
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
