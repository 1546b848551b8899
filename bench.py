"""bench.py -- BASELINE.json metric: fwd+bwd iters/s and HBM GB/s at 2M Gaussians, 1920x1080.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(N > 1: launched by torch.distributed.run, one rank per GPU, RCCL backend.)

The headline metric needs the rasterizer forward + backward, whose kernels are not built
("Decisions in force"), so `value` is null -- never estimated.  What the repo
does build on this path is measured for real, at the configuration the metric is quoted
on (config 3: 2M Gaussians, one 1920x1080 view, synthetic D2 inputs resident in HBM):

  step      = the binning stage of one view: inclusive scan of the 2M tiles_touched,
              stable radix sort of the K ~ 8M (tile|depth, id) pairs over bits
              [0, 32 + getHigherMsb(8160)) = [0, 45) and the tile ranges, as one
              hidegs_sort_tile_pairs call (rasterizer_impl.cu:321-371).
              W warm-up steps, then K timed steps between HIP events on the launch stream,
              barrier + synchronize on both sides, max over ranks.
  roofline  = the dominant kernel of the step (the most time per step): 24 algorithmic
              bytes per pair per launch for a sort pass (key 8 + value 4, read and written once), averaged
              over its launches with per-launch HIP events (hidegs_kernel_timing), against
              8 TB/s; traffic from the committed rocprofv3 PMC summary when present.
  distCUDA2 = simple_knn._C.distCUDA2 on the 2M D2 centres (once-per-scene initialiser).
  config5_scale = the same binning step and distCUDA2 at config 5's size (10M Gaussians, 4K frame).
  exchange  = the view-DP exchange of 2M x 59 fp32 leaf gradients + stats over RCCL
              (a one-rank group at N = 1), HIP-event timed.
  exchange_and_step = the exchange followed by the masked step, in sequence and overlapped bucket
              by bucket (ViewDPExchange.exchange_and_step); at N = 1 neither exchanges anything.
  masked Adam = the fused row-masked optimizer step (hidegs_amd.optim.Adam, the OurAdam
              drop-in) over the six HiDeGS parameter groups at 2M Gaussians (59 fp32 each), 90%
              of rows visible; 28 algorithmic bytes per updated value; beside it the reference's
              own op sequence (OurAdam.py:249-337 restated as torch ops) on the same GPU.
  cpu_baseline = the oracle's stable sort (numpy, one core) on the same 8M pairs; beside the
              distCUDA2 and masked Adam lines, the oracle's brute force on a sample of queries and
              its masked Adam step.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

N_GAUSSIANS = 2_000_000
W_PX, H_PX = 1920, 1080
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
ROOT = os.path.dirname(os.path.abspath(__file__))
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "latest_kernels.json")  # tools/prof_summary.py output


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001
        pass
    return platform.processor() or "unknown"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--knn-steps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exchange", action="store_true")
    ap.add_argument("--no-adam", action="store_true")
    ap.add_argument("--no-config5", action="store_true")
    args = ap.parse_args()

    # The contract is ONE JSON line on stdout; RCCL prints a version banner there at init, so the
    # process's fd 1 goes to stderr for the run and the result line is written to the saved fd.
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)

    import numpy as np
    import torch
    import torch.distributed as dist

    import simple_knn
    from hidegs_amd import _lib, primitives, synthetic
    from hidegs_amd.view_dp import GradArena, ViewDPExchange

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if not dist.is_initialized():
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ["MASTER_PORT"] = str(free_port())
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        else:
            dist.init_process_group("nccl", device_id=dev)

    def max_over_ranks(x: float) -> float:
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        dist.barrier()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        dist.barrier()
        wall = time.perf_counter() - t0
        return max_over_ranks(e0.elapsed_time(e1) / steps), max_over_ranks(wall * 1e3 / steps)

    # ---- the step: binning of one view (rank r renders its own view: seed r) -------------
    wl = synthetic.binning_workload(N_GAUSSIANS, W_PX, H_PX, seed=rank, device=dev)
    K, T = wl.num_pairs, wl.num_tiles
    end_bit = 32 + primitives.higher_msb(T)
    offsets = torch.empty_like(wl.tiles_touched)

    def step():
        primitives.inclusive_scan_u32(wl.tiles_touched, out=offsets)
        primitives.sort_tile_pairs(wl.keys, wl.values, T)  # SortPairs + identifyTileRanges in one call

    ms_step, wall_ms_step = timed(step, args.steps, args.warmup)

    # per-kernel durations of the same step, live, with per-launch HIP events
    kt_steps = max(10, min(args.steps, 50))
    # algorithmic bytes per launch (SURVEY §8(d) D4 per-pair figures: a sort pass reads and writes
    # key 8 + value 4; a histogram or range pass reads the 8-byte keys; the scan reads and writes u32)
    alg = {"scan_reduce": 4 * N_GAUSSIANS, "scan_small": 0, "scan_downsweep": 8 * N_GAUSSIANS,
           "radix_hist_u64": 8 * K, "radix_digit_scan": 0, "radix_scatter_u64": 24 * K,
           "segment_ranges": 0,  # ranges from the digit counts: a few partial tiles, not the keys
           "segment_sort": 24 * K, "identify_ranges": 8 * K,
           "big_segments": 0}  # the hot-tile queue: no tile over 24576 pairs here, so it only checks and exits
    with _lib.kernel_timer() as kt:
        for _ in range(kt_steps):
            step()
        torch.cuda.synchronize()
        kern = {}
        for nm, nbytes in alg.items():
            ms, n = kt.get(nm)
            if n == 0:
                continue
            avg_us = ms * 1e3 / n
            kern[nm] = {"avg_us": round(avg_us, 2), "launches_per_step": n // kt_steps,
                        "us_per_step": round(ms * 1e3 / kt_steps, 2),
                        "GBps": round(nbytes / (avg_us * 1e-6) / 1e9, 1) if nbytes else None}
    dom = max((k for k in kern if alg[k]), key=lambda k: kern[k]["us_per_step"])
    dom_us = kern[dom]["avg_us"]
    dom_bytes = alg[dom]
    achieved = dom_bytes / (dom_us * 1e-6) / 1e9
    traffic = None
    rocprof_name = {"radix_scatter_u64": "radix_scatter_kernel", "segment_sort": "segment_sort_kernel",
                    "radix_hist_u64": "radix_hist_kernel"}.get(dom, dom + "_kernel")
    # launch grid (threads) the rocprof summary keys the kernel by: one workgroup per tile (T) or per
    # 4096-pair tile of the sort (the scatter runs 512-thread workgroups, the others 256)
    ntiles_sort = (K + 4095) // 4096
    grid = {"segment_sort": T * 256, "radix_scatter_u64": ntiles_sort * 512}.get(dom, ntiles_sort * 256)
    if os.path.exists(TRAFFIC_FILE):
        with open(TRAFFIC_FILE) as f:
            traffic = json.load(f).get(f"{rocprof_name}@{grid}", {}).get("hbm_bytes_per_launch")
    sort_us = sum(kern[k]["us_per_step"] for k in kern if k.startswith(("radix_", "segment_")))

    line = {
        "metric": "fwd+bwd iters/sec & HBM GB/s at 2M Gaussians, 1920x1080",
        "value": None,
        "unit": "iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64/u32 (binning), f32 (distCUDA2, exchange)",
        "data": "synthetic (SURVEY §8(d) D2, seeded per rank)",
        "config": {"workload": "config 3: 2M Gaussians, 1920x1080, one view per rank -- binning stage, "
                               "distCUDA2 and the view-DP exchange measured; rasterizer fwd/bwd not built",
                   "n_gaussians": N_GAUSSIANS, "width": W_PX, "height": H_PX, "tiles": T, "pairs_K": K,
                   "sort_bits": [0, end_bit], "parallelism": f"view-dp{world}"},
        "status": "headline UNMEASURED: the rasterizer forward/backward kernels are not built "
                  "(DESIGN.md, 'Decisions in force'); value stays null",
        "binning_step": {"ms_per_step": round(ms_step, 4), "wall_ms_per_step": round(wall_ms_step, 4),
                         "pairs_per_s_all_ranks": K * world / (ms_step * 1e-3),
                         "views_per_s_all_ranks": world / (ms_step * 1e-3),
                         "sort_us": round(sort_us, 2), "kernels": kern},
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_us": dom_us},
        "cpu_baseline": None,
    }

    # ---- distCUDA2 at 2M ---------------------------------------------------------------------
    pts = synthetic.frustum_points(N_GAUSSIANS, seed=rank).to(dev)
    knn_ms, _ = timed(lambda: simple_knn._C.distCUDA2(pts), args.knn_steps, 1)
    with _lib.kernel_timer() as kt:
        simple_knn._C.distCUDA2(pts)
        torch.cuda.synchronize()
        kk = {nm: round(kt.get(nm)[0] * 1e3, 1) for nm in ("bounds", "morton", "radix_scatter_u64", "gather",
                                                             "leaf_box", "knn_leaf", "knn_hard")}
    line["distCUDA2"] = {"points": N_GAUSSIANS, "ms": round(knn_ms, 3),
                         "points_per_s_all_ranks": N_GAUSSIANS * world / (knn_ms * 1e-3), "kernels_us": kk,
                         "algorithmic_bytes": 16 * N_GAUSSIANS,
                         "hbm_frac": round(16 * N_GAUSSIANS / (knn_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5)}

    # ---- config 5's scale: 10M Gaussians, 3840x2160 frame ------------------------------------
    if not args.no_config5:
        wl5 = synthetic.binning_workload(10_000_000, 3840, 2160, seed=rank, device=dev)
        off5 = torch.empty_like(wl5.tiles_touched)

        def step5():
            primitives.inclusive_scan_u32(wl5.tiles_touched, out=off5)
            primitives.sort_tile_pairs(wl5.keys, wl5.values, wl5.num_tiles)

        ms5, _ = timed(step5, 20, 3)
        pts5 = synthetic.frustum_points(10_000_000, seed=rank).to(dev)
        knn5_ms, _ = timed(lambda: simple_knn._C.distCUDA2(pts5), 3, 1)
        line["config5_scale"] = {"workload": "10M Gaussians, 3840x2160 (32400 tiles): binning step and distCUDA2",
                                 "binning_ms_per_step": round(ms5, 4), "pairs_K": wl5.num_pairs,
                                 "sort_bits": [0, 32 + primitives.higher_msb(wl5.num_tiles)],
                                 "pairs_per_s_all_ranks": wl5.num_pairs * world / (ms5 * 1e-3),
                                 "distCUDA2_ms": round(knn5_ms, 3)}
        del wl5, off5, pts5

    # ---- view-DP exchange at 2M ---------------------------------------------------------------
    if not args.no_exchange:
        g = torch.Generator(device=dev).manual_seed(rank)
        visible = torch.rand(N_GAUSSIANS, device=dev, generator=g) < 0.9
        arena = GradArena(N_GAUSSIANS, device=dev)
        arena.flat.normal_(generator=g)
        norm = torch.rand(N_GAUSSIANS, 1, device=dev, generator=g)
        radii = torch.rand(N_GAUSSIANS, device=dev, generator=g)
        ex = ViewDPExchange()
        ex_ms, _ = timed(lambda: ex.exchange(arena, visible, max_stats=[norm, radii]), 20, 3)
        line["exchange"] = {"ms_per_step": round(ex_ms, 3), "world": world, "grad_bytes_per_rank": ex.last.reduced_bytes,
                            "algbw_GBps": ex.last.reduced_bytes / (ex_ms * 1e-3) / 1e9,
                            "collectives_per_step": ex.last.collectives, "compacted": ex.last.compacted,
                            "union_rows": ex.last.union_rows}

    # ---- masked Adam at 2M ---------------------------------------------------------------------
    if not args.no_adam:
        from hidegs_amd.optim import Adam
        widths = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
        lrs = {"xyz": 0.00016 * 4.2, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005,
               "rotation": 0.001}
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        prm = {k: torch.nn.Parameter(torch.randn(N_GAUSSIANS, w, device=dev, generator=g)) for k, w in widths.items()}
        for p in prm.values():
            p.grad = torch.randn(p.shape, device=dev, generator=g)
        vis = torch.rand(N_GAUSSIANS, device=dev, generator=g) < 0.9
        opt = Adam([{"params": [prm[k]], "lr": lrs[k], "name": k} for k in widths], lr=0.0, eps=1e-15)
        ad_ms, _ = timed(lambda: opt.step(vis), 20, 3)
        nvis = int(vis.sum())
        ad_bytes = 28 * 59 * nvis + N_GAUSSIANS
        with _lib.kernel_timer() as kt:
            opt.step(vis)
            torch.cuda.synchronize()
            k_ms, k_n = kt.get("masked_adam")
        # the reference's op sequence on the same GPU (gather, 8 elementwise ops, scatter per parameter)
        st = {k: (torch.zeros_like(p), torch.zeros_like(p)) for k, p in prm.items()}

        def ref_step():
            with torch.no_grad():
                for k, parami in prm.items():
                    m_all, v_all = st[k]
                    grad, exp_avg, exp_avg_sq, param = parami.grad[vis], m_all[vis], v_all[vis], parami[vis]
                    exp_avg.mul_(0.9).add_(grad, alpha=1 - 0.9)
                    exp_avg_sq.mul_(0.999).addcmul_(grad, grad, value=1 - 0.999)
                    denom = (exp_avg_sq.sqrt() / 0.5).add_(1e-15)
                    param.addcdiv_(exp_avg, denom, value=-lrs[k])
                    m_all[vis] = exp_avg
                    v_all[vis] = exp_avg_sq
                    parami[vis] = param
        ref_ms, _ = timed(ref_step, 5, 1)
        line["masked_adam"] = {"gaussians": N_GAUSSIANS, "visible_rows": nvis, "ms": round(ad_ms, 4),
                               "kernel_us_total": round(k_ms * 1e3, 1), "launches": k_n,
                               "algorithmic_bytes": ad_bytes, "GBps": round(ad_bytes / (ad_ms * 1e-3) / 1e9, 1),
                               "hbm_frac": round(ad_bytes / (ad_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                               "reference_torch_ops_ms": round(ref_ms, 3),
                               "speedup_vs_reference_ops": round(ref_ms / ad_ms, 2)}
        # the exchange and the step after it, in sequence and overlapped bucket by bucket
        if not args.no_exchange:
            arena = GradArena(N_GAUSSIANS, device=dev)
            for k, p in prm.items():
                arena[k].copy_(p.grad)
            arena.attach(prm)
            ex = ViewDPExchange()
            norm = torch.rand(N_GAUSSIANS, 1, device=dev, generator=g)

            def seq_step():
                res = ex.exchange(arena, vis, max_stats=[norm])
                opt.step(res.union)

            seq_ms, _ = timed(seq_step, 10, 2)
            fused_ms, _ = timed(lambda: ex.exchange_and_step(arena, vis, opt, prm, max_stats=[norm]), 10, 2)
            line["exchange_and_step"] = {"world": world, "sequential_ms": round(seq_ms, 3),
                                         "overlapped_ms": round(fused_ms, 3),
                                         "collectives": ex.last.collectives, "union_rows": ex.last.union_rows}
            del arena
        del prm, opt, st

    # ---- CPU baseline (rank 0, N = 1): the oracle's stable sort on the same pairs -------------
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import binning
        keys = wl.keys.cpu().numpy().view(np.uint64)
        vals = wl.values.cpu().numpy().view(np.uint32)
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or (time.perf_counter() - t0 < 10.0 and reps < 20):
            binning.stable_sort_pairs(keys, vals, 0, end_bit)
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        line["cpu_baseline"] = {"value": K / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
                                "sample": f"stable sort of the same {K} (key, value) pairs over bits [0,{end_bit}) "
                                          f"(numpy argsort kind=stable + gather, oracle/binning.py), {reps} reps",
                                "cpu": cpu_model(), "gpu_speedup_sort": round(dt * 1e3 / (sort_us * 1e-3), 1)}
        import oracle
        omp = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        # distCUDA2: the oracle's brute force (OpenMP) for a sample of the 2M D2 queries, each
        # against all 2M points
        if "distCUDA2" in line:
            cpu_pts = synthetic.frustum_points(N_GAUSSIANS, seed=rank).numpy()
            nq = 256
            idx = np.random.default_rng(0).choice(N_GAUSSIANS, nq, replace=False)
            t0 = time.perf_counter()
            oracle.knn_mean3_subset(cpu_pts, idx)
            dq = time.perf_counter() - t0
            line["distCUDA2"]["cpu_baseline"] = {
                "value": nq / dq, "unit": "queries/s", "cores": omp, "kind": "port",
                "sample": f"{nq} of the {N_GAUSSIANS} D2 queries, each brute-forced against all points "
                          "(oracle/knn_ref.c, OpenMP)",
                "gpu_queries_per_s": line["distCUDA2"]["points_per_s_all_ranks"]}
            del cpu_pts
        # masked Adam: the oracle's restatement (oracle/adam_ref.c, one core) of one step over the
        # same six 2M-row parameter groups, 90% of rows relevant
        if "masked_adam" in line:
            rng = np.random.default_rng(1)
            rel = rng.random(N_GAUSSIANS) < 0.9
            t_total = 0.0
            for w in (3, 3, 45, 1, 3, 4):
                pa = rng.standard_normal((N_GAUSSIANS, w), dtype=np.float32)
                ga = rng.standard_normal((N_GAUSSIANS, w), dtype=np.float32)
                ma, va = np.zeros_like(pa), np.zeros_like(pa)
                t0 = time.perf_counter()
                oracle.masked_adam(pa, ga, ma, va, rel, 1e-3, 0.9, 0.999, 1e-15, 0.0, 1)
                t_total += time.perf_counter() - t0
            line["masked_adam"]["cpu_baseline"] = {
                "value": 1e3 * t_total, "unit": "ms per step", "cores": 1, "kind": "port",
                "sample": f"one full step, {N_GAUSSIANS} Gaussians x 59 floats, 90% of rows relevant"}

    dist.destroy_process_group()
    sys.stdout.flush()
    if rank == 0:
        os.write(result_fd, (json.dumps(line) + "\n").encode())


if __name__ == "__main__":
    main()
