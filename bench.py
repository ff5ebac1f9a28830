"""Benchmark: Eikonal cost-to-go on MI355X (BASELINE.json metric), one JSON line on rank 0.

  python bench.py [--gpus N --steps K --warmup W]                   # N = 1 here
  torchrun --nproc-per-node N bench.py --gpus N ...                 # driver, N > 1

Workload (BASELINE.json configs): N = 1 -> config[1], a 4096 x 4096 DEM-derived cost raster
(terrain.py: fractal DEM seed 42 + the planner's cost recipe), single goal at the centre,
block-FIM in float64 -- the reference's arithmetic type (FastMarching.py:93-95 works on float64
rasters) and the drop-in's default; `--dtype f32` measures the fp32 solver instead (also reported
in extra_configs).  N > 1 -> config[3], strong scaling (default): ONE 16384 x 16384 raster
(terrain seed 7, goal at the centre) split over the ranks (px x py = 2x1, 2x2, 4x2 blocks of
16384 x 8192, 8192^2, 8192 x 4096); `--scaling weak` gives every rank a --block^2 block of a
growing raster instead.  A "step" = one full solve of the whole raster (T init -> converged),
inputs resident in HBM.  value = cells of the global raster x steps / max-over-ranks wall time
(Gcells/s).

Also reported: roofline of the dominant kernel (fim2d_persist_kernel, one launch per solve:
hipEvents around it on the solver stream over the timed region; algorithmic bytes = full tile
visits x 50176 B + in-place passes x 17408 B in fp32, twice that in fp64), ms-to-path
(host cost -> host path, N = 1), and the CPU baseline (oracle C heap FMM, 1 thread, N = 1).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))

import eikonal  # noqa: E402
from eikonal import dd, terrain  # noqa: E402
from eikonal import _lib as L  # noqa: E402

METRIC = "Eikonal Gcells/s + ms-to-path, 4k² & 16k² costmap at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# per element byte: cost read + T read + T write + halo read per full visit; T write + halo
# re-read per in-place pass (x 4 for fp32, x 8 for fp64); a tile's first visit reads no T (its T is
# still +inf: eik_stats.fresh_visits, fim2d.hip kFreshSkip)
CELLS_PER_VISIT = 3 * 64 * 64 + 4 * 64
CELLS_PER_PASS = 64 * 64 + 4 * 64
CELLS_T_READ = 64 * 64
WIDE_TILES = 16384  # fp32 maps of >= this many tiles run the 4-waves-per-SIMD kernel (csrc kWideTiles)


def env_int(k, d):
    return int(os.environ.get(k, d))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64",
                    help="solver arithmetic (the reference computes in float64)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="N > 1: strong = one --c4-size^2 raster split over the ranks (configs[3]); "
                         "weak = a --block^2 block per rank")
    ap.add_argument("--c4-size", type=int, default=16384, help="strong scaling: global raster side")
    ap.add_argument("--block", type=int, default=4096, help="weak scaling / N = 1: block side (cells)")
    ap.add_argument("--exchange-every", type=int, default=8, help="--dd rounds: outer iterations per exchange")
    ap.add_argument("--dd", choices=["live", "rounds"], default="live",
                    help="N > 1: live persistent launches + IPC halo rounds, or relaunch-per-round over RCCL")
    ap.add_argument("--sync-every", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-path", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-launch events (roofline)")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3 / C5 secondary measurements")
    ap.add_argument("--extra-steps", type=int, default=5)
    ap.add_argument("--extras", type=str, default="all",
                    help="comma list of extra_configs to run at N = 1 (C2_other,C3,C5,costmap,C4_1gpu,arm) or all")
    ap.add_argument("--pmc-traffic", type=str, default=None,
                    help="PMC summary (tools/pmc_traffic.py); default profiles/pmc_traffic_<dtype>.json")
    args = ap.parse_args()
    f64 = args.dtype == "f64"
    tdt = torch.float64 if f64 else torch.float32
    edt = L.EIK_F64 if f64 else L.EIK_F32
    esz = 8 if f64 else 4
    if args.pmc_traffic is None:
        args.pmc_traffic = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.dtype}.json")

    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local_rank = env_int("LOCAL_RANK", 0)
    # rehearsal knob (one-GPU box): every rank on cuda:0, gloo world group, the launches' grids
    # split so they are co-resident.  Timing under it is not a scaling measurement.
    shared = os.environ.get("EIK_BENCH_SHARED_GPU") == "1"
    if shared:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    px, py = dd.SPLITS[world]
    strong = world > 1 and args.scaling == "strong"
    if strong:  # configs[3]: one 16384^2 raster (seed 7), split over the ranks
        H = W = args.c4_size
        seed = 7
    else:
        H, W = args.block * py, args.block * px
        seed = 42
    blk = dd.Block(H, W, px, py, rank)
    goal_g = (W // 2, H // 2)

    cost = terrain.cost_block(blk.y0, blk.x0, blk.h, blk.w, H, W, seed=seed, device=dev).to(tdt).contiguous()
    T = torch.empty_like(cost)
    stream = torch.cuda.current_stream(dev)
    ctx = eikonal.Context(local_rank, options=eikonal._lib.options_from_env())  # A/B hook, opt-in
    ctx.set_option(L.OPT_SYNC_EVERY, args.sync_every)
    if shared and world > 1:
        ctx.set_option(L.OPT_GRID, max(2, 3 * torch.cuda.get_device_properties(dev).multi_processor_count // (2 * world)))
    fim = eikonal.Fim2d(ctx, 1, blk.h, blk.w, edt)
    lgoal = blk.local_goal(*goal_g)

    dd_mode = args.dd if world > 1 else None
    if world > 1:
        send, recv, ghost = dd.make_strips(blk, tdt, dev, float("inf"))
        ctrl = dd.control_group()
        halo, live_err, vote = None, None, None
        if dd_mode == "live":  # every rank must agree, or all fall back to rounds
            try:
                halo = dd.IpcHalo(ctx, blk, esz, group=ctrl)
            except Exception as e:
                live_err = repr(e)
            if env_int("LOCAL_WORLD_SIZE", world) == world and not live_err:
                try:  # one node: the per-round vote through shared memory, not gloo/TCP
                    vote = dd.NodeVote(group=ctrl)
                except Exception as e:
                    live_err = repr(e)
            ok = torch.tensor([0 if live_err else 1], dtype=torch.int64)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=ctrl)
            if ok.item() == 0:
                dd_mode = "rounds"
        live_local = dd.LiveGpuLocal(fim, ghost)
        local = dd.GpuLocal(fim, ghost)

        dd_rounds = []
        live_fail = {}  # a live solve that failed: its step index and error (then rounds for the rest)
        nstep = [0]

        def step():
            nonlocal dd_mode
            nstep[0] += 1
            if dd_mode == "live":
                try:
                    live_local.start(cost, T, lgoal, stream.cuda_stream)
                    dd_rounds.append(dd.solve_live(live_local, blk, halo, group=ctrl, vote=vote))
                    return
                except Exception as e:  # raised on every rank alike (dd.solve_live's error carry and
                    # release vote): every rank takes the relaunch schedule from here on, this step too
                    live_fail.update(step=nstep[0], error=repr(e)[:200])
                    dd_mode = "rounds"
                    ctx.set_option(L.OPT_QTIMEOUT, 30.0)
                    torch.cuda.synchronize()
            local.start(cost, T, lgoal, stream.cuda_stream)
            dd_rounds.append(dd.solve(local, blk, send, recv, exchange_every=args.exchange_every))
    else:
        def step():
            fim.solve(cost.data_ptr(), T.data_ptr(), [lgoal], stream.cuda_stream)

    if dd_mode == "live":
        ctx.set_option(L.OPT_QTIMEOUT, 5.0)  # a stuck live round ends in an error, not a hang
    step()  # (N > 1, live: a failure here falls back before the warmup)
    for _ in range(args.warmup):
        step()

    def timed(instrument):
        """K steps between barrier + synchronize; returns (max-over-ranks seconds, visits, passes,
        sweep_ms, launches)."""
        ctx.set_option(L.OPT_TIMING, 1 if instrument else 0)
        visits, passes, fresh, sweep_ms, iters = 0, 0, 0, 0.0, 0
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
            if instrument:
                s = fim.stats()
                visits += s["tile_visits"]
                passes += s["inplace_passes"]
                fresh += s["fresh_visits"]
                sweep_ms += s["sweep_ms"]
                iters += s["iterations"]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        ctx.set_option(L.OPT_TIMING, 0)
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=ctrl)
            el = tt.item()
        return el, visits, passes, fresh, sweep_ms, iters

    # 1) the measurement: no per-launch instrumentation inside the timed region
    el, _, _, _, _, _ = timed(False)
    # 2) the same K steps again with a hipEvent pair around every sweep launch (roofline)
    el_i, visits, passes, fresh, sweep_ms, iters = (0.0, 0, 0, 0, 0.0, 0) if args.no_timing else timed(True)

    if world > 1:  # the halo transport delivered every final edge (a wrong field cannot pass)
        dd_ok = dd.halo_consistent(blk, T, ghost, group=ctrl)
        # and the assembled field is the single-domain one: every rank solves the whole raster on
        # its own GPU and compares its block (no gather), then -- on RCCL -- one untimed solve of
        # the relaunch schedule (--dd rounds: batch_isend_irecv + all_reduce over RCCL), checked
        # the same way, so the north_star transport runs whenever the node has several GPUs
        dd_check = dd_field_check(args, ctx, dev, stream, blk, cost, T, H, W, seed, goal_g, tdt, edt, ctrl,
                                  local if (dd_mode == "live" and not shared) else None, send, recv, lgoal)
    value = H * W * args.steps / el / 1e9
    ms_per_step = el / args.steps * 1e3

    # roofline of the dominant kernel (rank-local: this rank's launches and its event time)
    launches = iters
    alg_bytes = esz * (visits * CELLS_PER_VISIT - fresh * CELLS_T_READ + passes * CELLS_PER_PASS)
    achieved = (alg_bytes / (sweep_ms * 1e-3) / 1e9) if sweep_ms > 0 else None
    traffic = None
    wide = not f64 and ((blk.h + 63) // 64) * ((blk.w + 63) // 64) >= WIDE_TILES
    kname = f"fim2d_persist_kernel<{'double' if f64 else 'float'}, {4 if wide else 1}>"
    if world == 1 and os.path.exists(args.pmc_traffic):  # measured on this workload (profiles/)
        try:
            pm = json.load(open(args.pmc_traffic))
            if pm.get("dtype", args.dtype) == args.dtype:
                traffic = pm.get("bytes_per_launch")
        except Exception:
            traffic = None
    roof = {
        "bound": "hbm",
        "kernel": kname,
        "achieved": round(achieved, 2) if achieved else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        "traffic": traffic,
        "alg_bytes_per_launch": round(alg_bytes / max(launches, 1)),
        # one read of cost + one write of T per cell, and the FIM redundancy over it
        "lower_bound_gbs": round(2 * esz * H * W / (el / args.steps) / 1e9, 2),
        "redundancy": round(alg_bytes / max(launches, 1) / (2 * esz * blk.h * blk.w), 2) if launches else None,
        "avg_launch_us": round(sweep_ms * 1e3 / max(launches, 1), 2),
        "instrumented_ms_per_step": round(el_i / args.steps * 1e3, 4),
        "launches_per_solve": round(launches / args.steps, 1),
        "tile_visits_per_solve": round(visits / args.steps, 1),
        "inplace_passes_per_solve": round(passes / args.steps, 1),
        "fresh_visits_per_solve": round(fresh / args.steps, 1),
    }

    out = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "Gcells/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        # N = 1: one GPU, nothing scales (null); N > 1: strong (configs[3]'s raster fixed) or weak
        "scaling": None if world == 1 else ("strong" if strong else "weak"),
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": f"synthetic (fractal DEM seed {seed} -> planner cost recipe, eikonal/terrain.py)",
        "config": {
            "workload": ("C2: 4096x4096 DEM-derived cost raster, single goal, FIM on 1 MI355X" if world == 1 else
                         (f"C4: {H}x{W} DEM-derived raster (seed 7), goal at the centre, {px}x{py} split over "
                          f"{world} GPUs" if strong else
                          f"C4-weak: {H}x{W} DEM-derived raster, {px}x{py} blocks of {args.block}^2")
                         + ", halo: " + ("live persistent launches + IPC peer stores over xGMI"
                                         if dd_mode == "live" else "RCCL point-to-point rounds")),
            "H": H, "W": W, "split": f"{px}x{py}", "block": [blk.h, blk.w], "goal": list(goal_g), "tile": 64,
            "parallelism": "single-gpu" if world == 1 else f"domain-decomposition {px}x{py}",
        },
        "roofline": roof,
    }
    if world > 1:
        out["config"]["dd_mode"] = dd_mode + (" (shm vote)" if dd_mode == "live" and vote is not None else "")
        out["config"]["halo_transport"] = ("hipIpc peer stores (xGMI) + node vote" if dd_mode == "live"
                                           else "RCCL batch_isend_irecv + all_reduce")
        out["config"]["dd_halo_consistent"] = dd_ok
        out["config"].update(dd_check)
        # every rank's work per solve (the decomposition's total against the single-domain solve's)
        if not args.no_timing:
            mine = torch.tensor([visits, passes, fresh, blk.h * blk.w], dtype=torch.float64) / \
                torch.tensor([args.steps, args.steps, args.steps, 1], dtype=torch.float64)
            allr = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allr, mine, group=ctrl)
            pr = torch.stack(allr)
            sd_v = dd_check.get("single_domain_tile_visits")
            sd_p = dd_check.get("single_domain_inplace_passes")
            out["config"]["dd_per_rank"] = {
                "tile_visits": [round(v, 1) for v in pr[:, 0].tolist()],
                "inplace_passes": [round(v, 1) for v in pr[:, 1].tolist()],
                "fresh_visits": [round(v, 1) for v in pr[:, 2].tolist()],
                "total_tile_visits": round(float(pr[:, 0].sum()), 1),
                "total_inplace_passes": round(float(pr[:, 1].sum()), 1),
                "visits_vs_single_domain": round(float(pr[:, 0].sum()) / sd_v, 3) if sd_v else None,
                "passes_vs_single_domain": (round(float(pr[:, 0].sum() + pr[:, 1].sum()) / (sd_v + sd_p), 3)
                                            if sd_v else None)}
        rr = dd_rounds[-args.steps:]
        out["config"]["dd_rounds_per_solve"] = round(sum(rr) / max(len(rr), 1), 1)
        out["config"]["dd_us_per_round"] = round(ms_per_step * 1e3 / max(sum(rr) / max(len(rr), 1), 1), 1)
        if live_err:  # the live transport could not be set up: rounds from the start
            out["config"]["dd_live_error"] = live_err[:200]
        if live_fail:  # a live solve failed at step k (1 = the first, untimed): rounds from there on
            out["config"]["dd_live_error"] = live_fail["error"]
            out["config"]["dd_live_failed_at_step"] = live_fail["step"]
            out["config"]["dd_live_failed_in_timed_region"] = live_fail["step"] > 1 + args.warmup

    if rank == 0 and world == 1 and not args.no_path:
        out.update(ms_to_path(cost, ctx, fim, dev, stream, goal_g, edt))

    if world > 1 and not args.no_extra:
        del T
        torch.cuda.empty_cache()
        xs = {}
        # configs[2] sharded: 128 / N maps per rank, no collective
        xs["C3_sharded"] = bench_batch(ctx, dev, stream, args.extra_steps, tdt, edt, rank=rank, world=world, group=ctrl)
        # configs[4] split in x-y: blocks of the layered volume, RCCL relaunch rounds
        try:
            xs["C5_split"] = bench_c5_split(ctx, dev, stream, args.extra_steps, tdt, edt, rank, world, ctrl, shared)
        except Exception as e:  # report; the measured line stands
            xs["C5_split"] = {"error": repr(e)[:200]}
        if rank == 0:
            out["extra_configs"] = xs

    if rank == 0 and world == 1 and not args.no_extra:
        del T
        torch.cuda.empty_cache()
        other = "f32" if f64 else "f64"
        want = set(args.extras.split(",")) if args.extras != "all" else None
        xs = {
            f"C2_{other}": lambda: bench_c2(ctx, dev, stream, cost, goal_g, args.extra_steps, other),
            "C3": lambda: bench_batch(ctx, dev, stream, args.extra_steps, tdt, edt),
            "C5": lambda: bench_layers(ctx, dev, stream, cost.to(tdt), goal_g, args.extra_steps),
            "costmap": lambda: bench_costmap(ctx, dev, stream, args.extra_steps, goal_g),
            "C4_1gpu": lambda: bench_c4(ctx, dev, stream, max(2, args.extra_steps // 2), tdt, edt),
            "arm": lambda: bench_arm(ctx, args.extra_steps),
            "C1": lambda: bench_c1(ctx),
        }
        if f64:
            xs["C4_1gpu_f32"] = lambda: bench_c4(ctx, dev, stream, max(2, args.extra_steps // 2), torch.float32,
                                                 L.EIK_F32)
            xs["C5_f32"] = lambda: bench_layers(ctx, dev, stream, cost.float(), goal_g, args.extra_steps)
        out["extra_configs"] = {k: fn() for k, fn in xs.items()
                                if want is None or k in want or (k.startswith("C2_") and "C2_other" in want)
                                or (k == "C5_f32" and "C5" in want)}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cost, goal_g, dev)

    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ms_to_path(cost, ctx, fim, dev, stream, goal, edt, start=(256, 256), reps=3):
    """Host cost raster -> arrival field -> path, two routes:
    * ms_to_path (the product's): the drop-in's own calls, FastMarching.computeTmap then
      getPathGDM, i.e. eik_tmap2d_f64 / eik_path2d_f64 on host numpy arrays (the C ABI copies
      through its pinned staging ring; the reference's API hands the field back to the host
      between the two calls, so it crosses PCIe three times: cost in, field out, field in);
    * ms_to_path_torch: pageable torch .to(dev) -> device solve -> eik_path2d_dev on the resident
      field -> path back (one host copy of the cost, none of the field).
    Also the path kernel alone on the resident field (hipEvents on the solver stream) and its
    time per path step."""
    host_cost = cost.cpu().numpy()
    f64 = edt == L.EIK_F64
    cap = 30004
    out_d = torch.empty((cap, 2), dtype=torch.float64, device=dev)
    n_d = torch.zeros(1, dtype=torch.int64, device=dev)
    st_d = torch.zeros(1, dtype=torch.int32, device=dev)
    H, W = host_cost.shape
    res = {}
    if f64:  # the drop-in computes in float64 (FastMarching.py:93-95)
        tot, lens = [], []
        for rep in range(reps + 2):  # two untimed calls first: the pinned result pool's first blocks
            t0 = time.perf_counter()
            Th = ctx.tmap2d(host_cost, goal)
            path, st = ctx.path2d(Th, start, goal)
            if rep >= 2:
                tot.append((time.perf_counter() - t0) * 1e3)
                lens.append(len(path))
        res.update({"ms_to_path": round(float(np.median(tot)), 3),
                    "ms_to_path_route": "drop-in: eik_tmap2d_f64 + eik_path2d_f64 on host arrays (pinned ring)"})
    tot, devs = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c = torch.from_numpy(host_cost).to(dev)
        T = torch.empty_like(c)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fim.solve(c.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)
        ctx._chk(L.lib().eik_path2d_dev(ctx._h, T.data_ptr(), edt, H, W, np.array(start, np.float64),
                                        np.array(goal, np.float64), 0.5, out_d.data_ptr(), cap, n_d.data_ptr(),
                                        st_d.data_ptr(), stream.cuda_stream))
        e1.record(stream)
        n = int(n_d.item())
        path = out_d[:n].cpu().numpy()
        t1 = time.perf_counter()
        tot.append((t1 - t0) * 1e3)
        devs.append(e0.elapsed_time(e1))
    # the walker alone on the resident field
    pk = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx._chk(L.lib().eik_path2d_dev(ctx._h, T.data_ptr(), edt, H, W, np.array(start, np.float64),
                                        np.array(goal, np.float64), 0.5, out_d.data_ptr(), cap, n_d.data_ptr(),
                                        st_d.data_ptr(), stream.cuda_stream))
        e1.record(stream)
        torch.cuda.synchronize()
        pk.append(e0.elapsed_time(e1))
    n = int(n_d.item())
    if "ms_to_path" not in res:
        res["ms_to_path"] = round(float(np.median(tot)), 3)
        res["ms_to_path_route"] = "torch .to(dev) + device solve + eik_path2d_dev"
    res.update({"ms_to_path_torch": round(float(np.median(tot)), 3),
                "ms_to_path_device": round(float(np.median(devs)), 3),
                "path_kernel_ms": round(float(np.median(pk)), 3),
                "path_us_per_step": round(float(np.median(pk)) * 1e3 / max(n, 1), 4),
                "path_points": n, "path_status": int(st_d.item()), "path_from": list(start)})
    return res


def dd_field_check(args, ctx, dev, stream, blk, cost, T, H, W, seed, goal_g, tdt, edt, group, rounds_local,
                   send, recv, lgoal):
    """N > 1, after the timed steps: (1) every rank solves the WHOLE raster on its own GPU and
    compares its block of the decomposed field with it (masks equal, fp64 <= 1e-11 / fp32 <= 1e-5
    relative; no gather), min over ranks -> dd_field_ok; (2) with RCCL (not the shared-GPU gloo
    rehearsal) one untimed solve of the relaunch schedule (dd.solve: batch_isend_irecv strips +
    all_reduce of the active count over RCCL), its field checked the same way -> dd_rounds_field_ok."""
    tol = 1e-11 if edt == L.EIK_F64 else 1e-5
    full_c = terrain.cost_block(0, 0, H, W, H, W, seed=seed, device=dev).to(tdt).contiguous()
    full_T = torch.empty_like(full_c)
    f1 = eikonal.Fim2d(ctx, 1, H, W, edt)
    f1.solve(full_c.data_ptr(), full_T.data_ptr(), [goal_g], stream.cuda_stream)
    torch.cuda.synchronize()
    s1 = f1.stats()  # the single-domain solve's work: the reference for the decomposition's total
    f1.close()
    ref = full_T[blk.y0:blk.y1, blk.x0:blk.x1].contiguous()
    del full_c, full_T
    torch.cuda.empty_cache()

    def err_of(Tb):
        fin = torch.isfinite(ref)
        if not torch.equal(fin, torch.isfinite(Tb)):
            return float("inf")
        if not bool(fin.any()):
            return 0.0
        return float(((Tb[fin].double() - ref[fin].double()).abs() / ref[fin].double().clamp(min=1e-30)).max())

    def worst(e):
        t = torch.tensor([e], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return t.item()

    out = {"single_domain_tile_visits": int(s1["tile_visits"]), "single_domain_inplace_passes": int(s1["inplace_passes"])}
    e = worst(err_of(T))
    out["dd_field_ok"] = bool(e <= tol)
    out["dd_field_max_rel"] = e
    if rounds_local is not None and os.environ.get("EIK_BENCH_DD_ROUNDS", "1") == "1":
        try:
            T2 = torch.empty_like(T)
            ctx.set_option(L.OPT_QTIMEOUT, 30.0)
            rounds_local.start(cost, T2, lgoal, stream.cuda_stream)
            t0 = time.perf_counter()
            nr = dd.solve(rounds_local, blk, send, recv, exchange_every=args.exchange_every)
            torch.cuda.synchronize()
            el = worst(time.perf_counter() - t0)
            e2 = worst(err_of(T2))
            out.update({"dd_rounds_field_ok": bool(e2 <= tol), "dd_rounds_field_max_rel": e2,
                        "dd_rounds_rccl_rounds": nr, "dd_rounds_rccl_ms": round(el * 1e3, 3)})
            del T2
        except Exception as ex:  # report; the measured line stands
            out["dd_rounds_error"] = repr(ex)[:200]
    return out


def timed_loop(fn, steps, warmup=1):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def c3_goal(cost_b, b, N):
    """A goal on a finite, low-cost cell of map b (its own generator: any rank can draw it)."""
    rng = np.random.default_rng(1000 + b)
    while True:
        gx, gy = (int(v) for v in rng.integers(N // 8, N - N // 8, 2))
        if float(cost_b[gy, gx]) < 50:
            return gx, gy


def solver_roofline(ctx, fim, solve, edt, kname, pmc_name, reps=3):
    """Roofline of one persistent solver launch (one launch per solve) on the throughput-bound
    configs: the launch's hipEvent time on the solver's stream (EIK_OPT_TIMING) and eik_stats'
    visits / first visits / in-place passes over `reps` solves, on the byte model of the C2 line
    (cost + T read + T write + halo per visit, no T read on a first visit, T write +
    halo per in-place pass).  traffic: the committed PMC pair of this config (profiles/pmc_name,
    tools/one_config.py under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, tools/pmc_traffic.py)."""
    esz = 8 if edt == L.EIK_F64 else 4
    ctx.set_option(L.OPT_TIMING, 1)
    ms, alg, vis, pas, fr = [], [], [], [], []
    try:
        for _ in range(reps):
            solve()
            st = fim.stats()
            ms.append(st["sweep_ms"])
            vis.append(st["tile_visits"])
            pas.append(st["inplace_passes"])
            fr.append(st["fresh_visits"])
            alg.append(esz * (st["tile_visits"] * CELLS_PER_VISIT - st["fresh_visits"] * CELLS_T_READ
                              + st["inplace_passes"] * CELLS_PER_PASS))
    finally:
        ctx.set_option(L.OPT_TIMING, 0)
    ms_k, alg_k = float(np.mean(ms)), float(np.mean(alg))
    ach = alg_k / (ms_k * 1e-3) / 1e9 if ms_k > 0 else None
    traffic = None
    pf = os.path.join(ROOT, "profiles", pmc_name)
    if os.path.exists(pf):
        try:
            pm = json.load(open(pf))
            if kname.split("<")[0] in pm.get("kernel", "") and pm.get("dtype") == ("f64" if esz == 8 else "f32"):
                traffic = pm.get("bytes_per_launch")
        except Exception:
            traffic = None
    return {"bound": "hbm", "kernel": kname, "achieved": round(ach, 2) if ach else None, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None, "traffic": traffic,
            "traffic_source": f"profiles/{pmc_name}" if traffic else None,
            "alg_bytes_per_launch": round(alg_k), "avg_launch_us": round(ms_k * 1e3, 2),
            "tile_visits_per_solve": round(float(np.mean(vis)), 1),
            "inplace_passes_per_solve": round(float(np.mean(pas)), 1),
            "fresh_visits_per_solve": round(float(np.mean(fr)), 1)}


def bench_batch(ctx, dev, stream, steps, tdt, edt, B=128, N=1024, rank=0, world=1, group=None):
    """configs[2]: 128 maps of 1024^2 (terrain seeds 1000..1127, one goal per map), ONE batched
    persistent solve (tiles of all maps share the device FIFO).  A step = the whole batch.  With
    world > 1 the batch is sharded (maps [rank * B / world, (rank + 1) * B / world) per rank, no
    collective in the solve); the time is the max over ranks."""
    lo, hi = rank * B // world, (rank + 1) * B // world
    nb = hi - lo
    cost = torch.empty((nb, N, N), dtype=tdt, device=dev)
    goals = []
    for i, b in enumerate(range(lo, hi)):
        cost[i] = terrain.cost_block(0, 0, N, N, N, N, seed=1000 + b, device=dev).to(tdt)
        goals.append(c3_goal(cost[i], b, N))
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, nb, N, N, edt)
    if world > 1:
        dist.barrier()
    solve = lambda: fim.solve(cost.data_ptr(), T.data_ptr(), goals, stream.cuda_stream)  # noqa: E731
    sec = timed_loop(solve, steps)
    if world > 1:
        tt = torch.tensor([sec], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
        sec = tt.item()
    st = fim.stats()
    f64 = edt == L.EIK_F64
    roof = None if world > 1 else solver_roofline(
        ctx, fim, solve, edt, f"fim2d_persist_kernel<{'double' if f64 else 'float'}, 1>",
        f"pmc_traffic_c3{'' if f64 else '_f32'}.json")
    reach = float(torch.isfinite(T).float().mean())
    fim.close()
    del cost, T
    torch.cuda.empty_cache()
    return {"workload": f"configs[2]: batch {B} x {N}x{N} terrain maps (seeds 1000..{1000 + B - 1}), one goal each"
                        + (f", sharded {nb} maps per rank over {world} GPUs" if world > 1 else ""),
            "dtype": "f64" if edt == L.EIK_F64 else "f32",
            "value": round(B * N * N / sec / 1e9, 4), "unit": "Gcells/s", "ms_per_step": round(sec * 1e3, 4),
            "steps": steps, "tile_visits_per_solve": st["tile_visits"], "inplace_passes_per_solve": st["inplace_passes"],
            "reached_fraction": round(reach, 4), **({"roofline": roof} if roof else {})}


def bench_c2(ctx, dev, stream, cost, goal, steps, dtype):
    """configs[1] in the other arithmetic type (same raster), with its kernel's event time."""
    f64 = dtype == "f64"
    c = cost.to(torch.float64 if f64 else torch.float32).contiguous()
    T = torch.empty_like(c)
    fim = eikonal.Fim2d(ctx, 1, c.shape[0], c.shape[1], L.EIK_F64 if f64 else L.EIK_F32)
    sec = timed_loop(lambda: fim.solve(c.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream), steps)
    ctx.set_option(L.OPT_TIMING, 1)
    fim.solve(c.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)
    st = fim.stats()
    ctx.set_option(L.OPT_TIMING, 0)
    esz = 8 if f64 else 4
    alg = esz * (st["tile_visits"] * CELLS_PER_VISIT - st["fresh_visits"] * CELLS_T_READ
                 + st["inplace_passes"] * CELLS_PER_PASS)
    fim.close()
    del c, T
    torch.cuda.empty_cache()
    return {"workload": f"configs[1] in {dtype}: the same 4096x4096 raster and goal",
            "dtype": dtype, "value": round(cost.numel() / sec / 1e9, 4), "unit": "Gcells/s",
            "ms_per_step": round(sec * 1e3, 4), "steps": steps,
            "kernel_ms": round(st["sweep_ms"], 4), "alg_bytes_per_launch": int(alg),
            "roofline_frac": round(alg / (st["sweep_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if st["sweep_ms"] else None,
            "tile_visits_per_solve": st["tile_visits"], "inplace_passes_per_solve": st["inplace_passes"]}


def bench_c4(ctx, dev, stream, steps, tdt, edt, N=16384):
    """configs[3] on ONE GPU: the 16384^2 DEM-derived raster (terrain seed 7), goal at the centre,
    solved whole (1 GiB cost + 1 GiB T in HBM).  The N = 4 / 8 driver runs measure the split
    versions; this line is the single-GPU reference point of the same raster size."""
    cost = terrain.cost_block(0, 0, N, N, N, N, seed=7, device=dev).to(tdt).contiguous()
    T = torch.empty_like(cost)
    fim = eikonal.Fim2d(ctx, 1, N, N, edt)
    goal = (N // 2, N // 2)
    solve = lambda: fim.solve(cost.data_ptr(), T.data_ptr(), [goal], stream.cuda_stream)  # noqa: E731
    sec = timed_loop(solve, steps)
    st = fim.stats()
    f64 = edt == L.EIK_F64
    wide = not f64 and (N // 64) * (N // 64) >= WIDE_TILES
    roof = solver_roofline(ctx, fim, solve, edt,
                           f"fim2d_persist_kernel<{'double' if f64 else 'float'}, {4 if wide else 1}>",
                           f"pmc_traffic_c4{'' if f64 else '_f32'}.json", reps=2)
    reach = float(torch.isfinite(T).float().mean())
    fim.close()
    del cost, T
    torch.cuda.empty_cache()
    return {"workload": f"configs[3] at 1 GPU: {N}x{N} DEM-derived raster (seed 7), single goal at the centre, 1x1",
            "dtype": "f64" if edt == L.EIK_F64 else "f32", "value": round(N * N / sec / 1e9, 4), "unit": "Gcells/s", "ms_per_step": round(sec * 1e3, 4),
            "steps": steps, "tile_visits_per_solve": st["tile_visits"], "inplace_passes_per_solve": st["inplace_passes"],
            "reached_fraction": round(reach, 4), "roofline": roof}


def bench_arm(ctx, steps, half=30, m=40, K=16, res=0.05):
    """SURVEY.md §8(f) rank 3, main() step 3 (:1462-1593): the end-effector volume of a 2h x 2h area
    (GetObstMap * TunnelCost, eik_arm_path_f64 also solving FM3D and the 3D path), and K candidate
    fetch poses' volumes solved as ONE batched FM3D (eik_tmap3d_batch_f64) against K single solves."""
    import math
    sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
    import planner
    rng = np.random.default_rng(5)
    n = 2 * half
    yy, xx = np.mgrid[0:n, 0:n] * res
    Z = 0.1 * np.sin(2.1 * xx) * np.cos(0.9 * yy + 0.3) + 0.03 * rng.standard_normal((n, n))
    Z -= Z.min()
    resX = res * (2 * n - 1) / (2 * n)
    sZ = int(round((Z.max() + 0.5) / 0.02))
    obst = (rng.random((n, n)) < 0.1).astype(np.float64)
    p0, p1 = np.array([0.2, 0.35]) * n * resX, np.array([0.6, 0.5]) * n * resX
    t = np.linspace(0, 1, m)[:, None]
    base = np.zeros((m, 3))
    base[:, :2] = p0 + t * (p1 - p0)
    base[:, 2] = 0.25
    heading = np.stack([np.zeros(m), np.zeros(m), np.full(m, math.atan2(*(p1 - p0)[::-1]))], 1)
    fw = np.uint32(np.round([(p1[0] + 0.2) / resX, (p1[1] + 0.15) / resX, (Z.max() * 0.6 + 0.1) / 0.02]))
    iw = np.uint32(np.round([(p0[0] + 0.15) / resX, (p0[1] + 0.1) / resX, 0.45 / 0.02]))
    vol = planner.volume(n, n, sZ, resX, resX, 0.02, 1.0, 2.0, 0.527, 0.2673, 0.1105, fw, iw)
    sec_t = timed_loop(lambda: ctx.arm_tunnel_cost(base, heading, vol), steps)
    out = {}

    # the planner's call: host DEM area -> volume -> early-exit field -> path (no field copies back)
    sec_p = timed_loop(lambda: ctx.arm_path(Z, obst, base, heading, vol, 0.5), steps)
    path, st, cost, _ = ctx.arm_path(Z, obst, base, heading, vol, 0.5, want_fields=True)
    # K candidate fetch poses: the sample node moved around the last base point
    goals = []
    for k in range(K):
        a = 2 * math.pi * k / K
        goals.append([int(fw[0]) + round(4 * math.cos(a)), int(fw[1]) + round(4 * math.sin(a)), int(fw[2])])
    costs = np.repeat(cost[None], K, 0)
    for k, g in enumerate(goals):
        costs[k, g[1], g[0], g[2]] = 1.0  # finite at every candidate node
    sec_b = timed_loop(lambda: ctx.tmap3d_batch(costs, goals), steps)
    # the batch's device solve alone (hipEvents around the persistent launch): the wall time above
    # also holds the pageable copies of 16 volumes each way
    dev_b = []
    for _ in range(max(3, steps)):
        ctx.tmap3d_batch(costs, goals)
        dev_b.append(ctx.stats()["solve_ms"])
    sec_s = timed_loop(lambda: [ctx.tmap3d(costs[k], goals[k]) for k in range(K)], max(1, steps // 2))
    return {"workload": f"configs-adjacent: end-effector volume {n}x{n}x{sZ} ({m} base points), f64",
            "ms_tunnel_cost": round(sec_t * 1e3, 3), "ms_volume_fm3d_path": round(sec_p * 1e3, 3),
            "path_points": int(len(path)), "path_status": int(st),
            f"ms_batch{K}_fm3d": round(sec_b * 1e3, 3), f"ms_batch{K}_fm3d_device": round(float(np.median(dev_b)), 3),
            f"ms_{K}_single_fm3d": round(sec_s * 1e3, 3)}


def c5_volume(c0, dev):
    """configs[4]'s [H][W][5] volume from a 2D raster c0: mode 0 = c0, mode 1 = 1.6 x it and
    impassable above cost 100, mode 2 = 0.8 x it with 1-in-5 impassable 64 x 64 blocks, between two
    +inf padding layers (Coupled_motion_planner.py:355-356)."""
    H, W = c0.shape
    inf = torch.full_like(c0, float("inf"))
    c1 = torch.where(c0 > 100, inf, 1.6 * c0)
    yy = torch.arange(H, device=dev)[:, None] // 64
    xx = torch.arange(W, device=dev)[None, :] // 64
    c2 = torch.where(((yy + 2 * xx) % 5) == 0, inf, 0.8 * c0)
    return torch.stack([inf, c0, c1, c2, inf], dim=-1).contiguous()


def bench_c5_split(ctx, dev, stream, steps, tdt, edt, rank, world, group, shared, N=4096):
    """SURVEY §8(e) "C5: split x-y only, layers stay together" at N > 1: configs[4]'s 4096 x 4096 x 3
    volume (bench_layers' volume of the C2 raster) split into dd.SPLITS[world] blocks, one per rank,
    each solved by the layered solver (eik_fim3dl_*) with ghost strips of 3 values per edge cell, on
    the relaunch schedule (dd.solve: local solve to convergence, pack, RCCL batch_isend_irecv,
    merge, all_reduce of the active count; the shared-GPU rehearsal stages the strips through host
    memory over gloo).  A step = one solve of the whole volume; the time is the max over ranks.
    Checked against the single-domain layered solve (eik_fim3d_solve) of the same volume on every
    rank: masks equal and <= 1e-11 (fp64) / 1e-5 (fp32) relative (dd_field_ok), with every rank's
    tile visits beside the single domain's."""
    px, py = dd.SPLITS[world]
    blk = dd.Block(N, N, px, py, rank)
    if shared:  # the layered kernel holds one workgroup per CU: 3/4 of those, split between the ranks
        ctx.set_option(L.OPT_GRID, max(2, 3 * torch.cuda.get_device_properties(dev).multi_processor_count // (4 * world)))
    vol = c5_volume(terrain.cost_block(0, 0, N, N, N, N, seed=42, device=dev).to(tdt), dev)
    cb = vol[blk.y0:blk.y1, blk.x0:blk.x1].contiguous()
    T = torch.empty_like(cb)
    nl, Lm = 3, 5
    fim = eikonal.Fim3dLayered(ctx, blk.h, blk.w, Lm, 1, nl, edt)
    dsend, drecv, ghost = dd.make_strips(blk, tdt, dev, float("inf"), per_cell=nl)
    loc = dd.GpuLocalLayered(fim, ghost)
    if shared:  # gloo between processes on one GPU: host-staged strips
        hsend, hrecv, _ = dd.make_strips(blk, tdt, "cpu", float("inf"), per_cell=nl)
        drv, send, recv, cdev = dd.HostStaged(loc, dsend, drecv), hsend, hrecv, "cpu"
    else:  # RCCL over xGMI, device strips
        drv, send, recv, cdev = loc, dsend, drecv, None
    lg = blk.local_goal(N // 2, N // 2)
    goal = (lg[0], lg[1], 1)
    rounds, vis, pas = [], [], []
    # the live schedule (round 6: the layered kernel's halo agent, hipIpc strips of nl values per edge
    # cell, the node vote), agreed by every rank, else the relaunch rounds above
    live, live_err, halo, vote = None, None, None, None
    try:
        halo = dd.IpcHalo(ctx, blk, (8 if edt == L.EIK_F64 else 4) * nl, group=group)
        if env_int("LOCAL_WORLD_SIZE", world) == world:
            vote = dd.NodeVote(group=group)
    except Exception as e:
        live_err = repr(e)
    ok = torch.tensor([0 if live_err else 1], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if ok.item() == 1:
        live = dd.LiveGpuLocalLayered(fim, ghost)

    def solve():
        nonlocal live, live_err
        if live is not None:
            try:
                live.start(cb, T, goal, stream.cuda_stream)
                rounds.append(dd.solve_live(live, blk, halo, group=group, vote=vote))
            except Exception as e:  # every rank alike (dd.solve_live's error carry): rounds from here on
                live, live_err = None, repr(e)
        if live is None:
            loc.start(cb, T, goal, stream.cuda_stream)
            rounds.append(dd.solve(drv, blk, send, recv, exchange_every=1, count_device=cdev))
        st = fim.stats()
        vis.append(st["tile_visits"])
        pas.append(st["inplace_passes"])

    solve()  # warmup
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        solve()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    tt = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
    sec = tt.item() / steps
    # the single-domain layered solve of the same volume (every rank its own; no gather)
    Tf = torch.empty_like(vol)
    g3 = np.array([N // 2, N // 2, 1], np.int64)
    ctx._chk(L.lib().eik_fim3d_solve(ctx._h, vol.data_ptr(), Tf.data_ptr(), N, N, Lm, edt, g3, stream.cuda_stream))
    torch.cuda.synchronize()
    sd = ctx.stats()
    ref = Tf[blk.y0:blk.y1, blk.x0:blk.x1, 1:1 + nl]
    Tb = T[:, :, 1:1 + nl]
    fin = torch.isfinite(ref)
    if not torch.equal(fin, torch.isfinite(Tb)):
        err = float("inf")
    elif bool(fin.any()):
        err = float(((Tb[fin].double() - ref[fin].double()).abs() / ref[fin].double().clamp(min=1e-30)).max())
    else:
        err = 0.0
    mine = torch.tensor([err, float(np.mean(vis[1:])), float(np.mean(pas[1:])), float(np.mean(rounds[1:]))],
                        dtype=torch.float64)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine, group=group)
    pr = torch.stack(allr)
    tol = 1e-11 if edt == L.EIK_F64 else 1e-5
    fim.close()
    if halo is not None:
        halo.close()
    if vote is not None:
        vote.close()
    del vol, cb, T, Tf
    torch.cuda.empty_cache()
    sched = ("live schedule: persistent layered launches + halo agents, hipIpc strips (xGMI) + node vote"
             if live is not None else "relaunch schedule (" + ("host-staged gloo rehearsal" if shared else
                                                               "RCCL batch_isend_irecv + all_reduce") + ")")
    return {"workload": f"configs[4] split: {N}x{N}x3 layered costmap (bench_layers' volume, z padded to 5), "
                        f"{px}x{py} x-y blocks over {world} GPUs, layers together; layered solver per block, " + sched,
            "dd_mode": "live" if live is not None else "rounds", **({"dd_live_error": live_err[:200]} if live_err else {}),
            "dtype": "f64" if edt == L.EIK_F64 else "f32", "value": round(N * N * 3 / sec / 1e9, 4),
            "unit": "Gcells/s", "ms_per_step": round(sec * 1e3, 4), "steps": steps,
            "dd_field_ok": bool(float(pr[:, 0].max()) <= tol), "dd_field_max_rel": float(pr[:, 0].max()),
            "dd_rounds_per_solve": round(float(pr[0, 3]), 1),
            "dd_per_rank": {"tile_visits": [round(v, 1) for v in pr[:, 1].tolist()],
                            "inplace_passes": [round(v, 1) for v in pr[:, 2].tolist()],
                            "total_tile_visits": round(float(pr[:, 1].sum()), 1),
                            "visits_vs_single_domain": round(float(pr[:, 1].sum()) / max(sd["tile_visits"], 1), 3)},
            "single_domain_tile_visits": int(sd["tile_visits"])}


def bench_layers(ctx, dev, stream, cost2d, goal, steps, Lz=3):
    """configs[4]: coupled (x, y, locomotion-mode) 4096 x 4096 x 3 costmap, [y][x][z] (FM3D
    layout), unit spacing between layers (FastMarching3D semantics): mode 0 = the C2 raster,
    mode 1 = 1.6 x it and impassable above cost 100, mode 2 = 0.8 x it with 1-in-5 impassable
    64 x 64 blocks.  As the planner builds its FM3D volumes (Coupled_motion_planner.py:355-356)
    the z ends are padded with +inf layers: 5 layers in memory, 3 solved (the layered solver,
    fim2dl.hip).  Solve from (goal, mode 0); then the FM3D path from (256, 256, mode 0).
    Gcells/s counts the 3 real layers."""
    H, W = cost2d.shape
    cost = c5_volume(cost2d, dev)
    T = torch.empty_like(cost)
    Lm = Lz + 2
    g3 = np.array([goal[0], goal[1], 1], np.int64)
    f64 = cost.dtype == torch.float64
    edt = L.EIK_F64 if f64 else L.EIK_F32

    def solve():
        ctx._chk(L.lib().eik_fim3d_solve(ctx._h, cost.data_ptr(), T.data_ptr(), H, W, Lm, edt, g3,
                                         stream.cuda_stream))

    sec = timed_loop(solve, steps)
    # per-launch event time of the layered kernel over the timed solves (one launch per solve)
    ms_l = []
    for _ in range(steps):
        solve()
        ms_l.append(ctx.stats()["solve_ms"])
    st = ctx.stats()
    cap = 30004
    out_d = torch.empty((cap, 3), dtype=torch.float64, device=dev)
    n_d = torch.zeros(1, dtype=torch.int64, device=dev)
    st_d = torch.zeros(1, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    ctx._chk(L.lib().eik_path3d_dev(ctx._h, T.data_ptr(), edt, H, W, Lm, np.array([256.0, 256.0, 1.0]),
                                    np.array([float(goal[0]), float(goal[1]), 1.0]), 0.5, out_d.data_ptr(), cap,
                                    n_d.data_ptr(), st_d.data_ptr(), stream.cuda_stream))
    e1.record(stream)
    torch.cuda.synchronize()
    res = {"workload": f"configs[4]: coupled {H}x{W}x{Lz} layered costmap (x, y, locomotion mode), FM3D semantics, "
                       f"z padded with +inf layers ({Lm} in memory)",
           "reached_fraction": round(float(torch.isfinite(T[:, :, 1:1 + Lz]).float().mean()), 4),
           "dtype": "f64" if f64 else "f32", "solve_ms_device": round(st.get("solve_ms", 0.0), 4),
           "value": round(H * W * Lz / sec / 1e9, 4), "unit": "Gcells/s", "ms_per_step": round(sec * 1e3, 4),
           "steps": steps, "launches_per_solve": st.get("iterations"), "tile_visits_per_solve": st.get("tile_visits"),
           "path_ms_device": round(e0.elapsed_time(e1), 3), "path_points": int(n_d.item()),
           "path_status": int(st_d.item())}
    # roofline of fim2dl_persist_kernel<R, 3> (algorithmic bytes: sizeof(R) x 3 layers per cell of cost
    # read, T read and T write per full visit + halo, T write + halo per in-place pass)
    ms_k = float(np.mean(ms_l))
    ach = st["bytes_alg"] / (ms_k * 1e-3) / 1e9 if ms_k > 0 else None
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_c5{'_f64' if f64 else ''}.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("bytes_per_launch")
        except Exception:
            traffic = None
    res["roofline"] = {"bound": "hbm", "kernel": f"fim2dl_persist_kernel<{'double' if f64 else 'float'}, {Lz}>",
                       "achieved": round(ach, 2) if ach else None,
                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                       "traffic": traffic, "alg_bytes_per_launch": round(st["bytes_alg"]),
                       "avg_launch_us": round(ms_k * 1e3, 2), "inplace_passes_per_solve": st.get("inplace_passes")}
    del cost, T
    torch.cuda.empty_cache()
    return res


def bench_costmap(ctx, dev, stream, steps, goal, N=4096, res=0.05):
    """SURVEY.md §8(f) rank 1, the solver's input producer: the planner's cost raster built from
    the 4096^2 DEM on the GPU (eik_costmap_dev: normals, slope obstacles, two hole fillings, five
    disk morphologies, EDT ramp, 50 x 50 blur), f64 as the reference; then DEM -> path on the
    device (cost map + f64 -> f32 + solve + path kernel)."""
    Z = terrain.dem_block(0, 0, N, N, seed=42, device=dev).double().contiguous()
    cost = torch.empty_like(Z)
    obst = torch.empty(Z.shape, dtype=torch.uint8, device=dev)

    def build():
        ctx._chk(L.lib().eik_costmap_dev(ctx._h, Z.data_ptr(), N, N, res, res * N, None, cost.data_ptr(),
                                         obst.data_ptr(), stream.cuda_stream))

    sec = timed_loop(build, steps)
    fim = eikonal.Fim2d(ctx, 1, N, N, L.EIK_F32)
    cap = 30004
    out_d = torch.empty((cap, 2), dtype=torch.float64, device=dev)
    n_d = torch.zeros(1, dtype=torch.int64, device=dev)
    st_d = torch.zeros(1, dtype=torch.int32, device=dev)
    c32 = torch.empty(Z.shape, dtype=torch.float32, device=dev)
    T = torch.empty_like(c32)
    g = [int(goal[0]), int(goal[1])]

    def dem_to_path():
        build()
        c32.copy_(cost)
        fim.solve(c32.data_ptr(), T.data_ptr(), [tuple(g)], stream.cuda_stream)
        ctx._chk(L.lib().eik_path2d_dev(ctx._h, T.data_ptr(), L.EIK_F32, N, N, np.array([256.0, 256.0]),
                                        np.array([float(g[0]), float(g[1])]), 0.5, out_d.data_ptr(), cap,
                                        n_d.data_ptr(), st_d.data_ptr(), stream.cuda_stream))

    sec2 = timed_loop(dem_to_path, steps)
    obst_frac = float(obst.float().mean())
    fim.close()
    # main()'s whole step 1 (:1097-1258) through one ABI call from the host
    # DEM -- cost raster, both fronts in fp64 as the reference, device join, two path kernels, host
    # assembly (pageable H2D of the DEM included)
    sys.path.insert(0, os.path.join(ROOT, "planning-motion_planning_amd"))
    import planner
    Zh = Z.cpu().numpy()
    q = planner.query(res * (g[0] + 1), res * (g[1] + 1), res * (256 + 1), res * (256 + 1), 0.0, res, res * N)
    rp = {}

    def step1():
        rp["r"] = ctx.rover_path(Zh, q)

    sec3 = timed_loop(step1, max(2, steps // 2))
    default_join = [int(v) for v in rp["r"][2]]
    # the same step with the reference's own band and LIFO ties (EIK_OPT_EXACT_BAND, bidir_exact.hip)
    ctx.set_option(L.OPT_EXACT_BAND, 1)
    try:
        sec4 = timed_loop(step1, max(2, steps // 2))
        xi = ctx.exact_info()
    finally:
        ctx.set_option(L.OPT_EXACT_BAND, 0)
    exact = {"ms": round(sec4 * 1e3, 3), "replay_ms": round(xi["ms"], 3), "passes": xi["passes"],
             "sweeps": xi["sweeps"], "tie_launches": xi["tie_launches"], "node_join": [int(v) for v in rp["r"][2]],
             "join_equals_default": [int(v) for v in rp["r"][2]] == default_join}
    return {"workload": f"cost raster of the planner (Coupled_motion_planner.py:1101-1216) from a {N}x{N} DEM "
                        f"(terrain seed 42, res {res} m), f64",
            "value": round(N * N / sec / 1e9, 4), "unit": "Gcells/s", "ms_per_step": round(sec * 1e3, 3),
            "steps": steps, "obstacle_fraction": round(obst_frac, 4),
            "ms_dem_to_path_device": round(sec2 * 1e3, 3), "path_points": int(n_d.item()),
            "path_status": int(st_d.item()),
            "planner_step1": {"workload": "Coupled_motion_planner.py:1097-1258 via eik_rover_path_f64: host DEM -> "
                                          "cost raster -> biComputeTmap (2 x fp64 fronts) -> 2 GDM paths -> roverPath",
                              "ms": round(sec3 * 1e3, 3), "waypoints": int(len(rp["r"][0])),
                              "node_join": default_join, "exact_band": exact}}


def host_cpu():
    """The host's CPU model, its logical CPU count and the CPUs this process may use (the GPU box
    shows the whole machine's CPUs; OMP_NUM_THREADS there is this job's share)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count()
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(avail, share) if share > 0 else avail
    return {"model": model, "nproc": nproc, "affinity": avail, "threads_used": threads}


def cpu_baseline(cost, goal, dev, B=128, N=1024):
    """The reference's algorithm on the host cores (oracle/eikonal_oracle.c: the bit-exact heap-FMM
    restatement of FastMarching.computeTmap), bounded samples:
    * value: ONE full-field solve of the C2 raster (fp64), 1 thread -- the reference runs one
      Python process, one core;
    * C1 (configs[0]): the 256^2 uniform-cost map, goal at the centre, 1 thread;
    * C3_job_cores: the 128 x 1024^2 batch with one map per thread over this job's share of the
      host's cores (threads_used, the box's OMP_NUM_THREADS; host.affinity says how many CPUs the
      job could see).  BASELINE.md asks for "all host cores": the GPU box leases a share of a
      many-core host, so the label states the share actually used."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    c = cost.double().cpu().numpy()
    hc = host_cpu()
    O.set_strict(False)
    try:
        t0 = time.perf_counter()
        O.fmm2d(c, goal)
        el = time.perf_counter() - t0
        # C1: configs[0] itself
        u = np.ones((256, 256))
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or time.perf_counter() - t0 < 0.5:
            O.fmm2d(u, (128, 128))
            reps += 1
        c1 = (time.perf_counter() - t0) / reps
        # C3 over the host cores: the bench's maps and goals
        costs = np.empty((B, N, N))
        goals = []
        for b in range(B):
            cb = terrain.cost_block(0, 0, N, N, N, N, seed=1000 + b, device=dev).double()
            goals.append(c3_goal(cb, b, N))
            costs[b] = cb.cpu().numpy()
        t0 = time.perf_counter()
        O.fmm2d_batch(costs, np.array(goals, np.int64), nthreads=hc["threads_used"])
        c3 = time.perf_counter() - t0
        del costs
    finally:
        O.set_strict(True)
    return {"value": round(c.size / el / 1e9, 6), "unit": "Gcells/s", "cores": 1, "kind": "port",
            "sample": f"one full-field solve of the same {c.shape[0]}x{c.shape[1]} raster in fp64 "
                      f"({el:.2f} s, oracle/eikonal_oracle.c heap FMM)",
            "seconds": round(el, 3), "host": hc,
            "C1": {"workload": "configs[0]: 256x256 uniform cost, goal at the centre, heap FMM, 1 thread",
                   "ms": round(c1 * 1e3, 3), "value": round(256 * 256 / c1 / 1e9, 6), "unit": "Gcells/s"},
            "C3_job_cores": {"workload": f"configs[2]: {B} x {N}x{N} terrain maps (the bench's seeds and goals), "
                                        f"one map per thread on this job's {hc['threads_used']} of "
                                        f"{hc['affinity']} visible CPUs, heap FMM fp64",
                             "cores": hc["threads_used"], "seconds": round(c3, 3),
                             "value": round(B * N * N / c3 / 1e9, 6), "unit": "Gcells/s"}}


def bench_c1(ctx, N=256, reps=20):
    """configs[0] (the reference's CPU plumbing case) through the drop-in's host entry point:
    256^2 uniform cost, goal at the centre, fp64, host array in -> host field out."""
    u = np.ones((N, N))
    ctx.tmap2d(u, (N // 2, N // 2))
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.tmap2d(u, (N // 2, N // 2))
    sec = (time.perf_counter() - t0) / reps
    return {"workload": "configs[0]: 256x256 uniform cost, goal at the centre, fp64, eik_tmap2d_f64 host -> host",
            "ms": round(sec * 1e3, 4), "value": round(N * N / sec / 1e9, 4), "unit": "Gcells/s"}


if __name__ == "__main__":
    main()
