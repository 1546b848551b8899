"""bench.py -- BASELINE.json metric: fwd+bwd iters/s and HBM GB/s at 2M Gaussians, 1920x1080.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(N > 1: launched by torch.distributed.run, one rank per GPU, RCCL backend.)

State ("Denials in force"): the rasterizer forward/backward is not built,
so the metric is UNMEASURED and `value` is null -- nothing is estimated or faked.
What does exist is measured for real:
  * N > 1: the view-DP exchange step (hidegs_amd.view_dp) at the metric's size, 2M
    Gaussians x 59 fp32 leaf-gradient values (472 MB) plus the densification statistics
    and the visibility union, K timed steps after W warm-up steps, barrier +
    synchronize on both sides, max over ranks.  Reported under "exchange".
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import time

N_GAUSSIANS = 2_000_000
W_PX, H_PX = 1920, 1080


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    line = {
        "metric": "fwd+bwd iters/sec & HBM GB/s at 2M Gaussians, 1920x1080",
        "value": None,
        "unit": "iters/s",
        "n_gpus": args.gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": "config 3: 2M Gaussians, 1920x1080, fwd+bwd", "n_gaussians": N_GAUSSIANS,
                   "width": W_PX, "height": H_PX, "parallelism": f"view-dp{max(world, 1)}"},
        "status": "UNMEASURED: the rasterizer forward/backward is not built (DESIGN.md, 'Denials in force')",
        "roofline": None,
        "cpu_baseline": None,
    }

    if world > 1:
        import torch.distributed as dist
        from hidegs_amd.view_dp import LEAF_WIDTHS, ViewDPExchange
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        g = torch.Generator(device=dev).manual_seed(rank)
        visible = torch.ones(N_GAUSSIANS, dtype=torch.bool, device=dev)  # synthetic D2 views see ~all Gaussians
        grads = {k: torch.randn(N_GAUSSIANS, w, device=dev, generator=g) for k, w in LEAF_WIDTHS.items()}
        gmax = torch.rand(N_GAUSSIANS, device=dev, generator=g)
        rmax = torch.rand(N_GAUSSIANS, device=dev, generator=g)
        denom = torch.ones(N_GAUSSIANS, device=dev)
        ex = ViewDPExchange()

        def step():
            ex.exchange(grads, visible, max_stats=[gmax, rmax], sum_stats=[denom])

        for _ in range(args.warmup):
            step()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], device=dev)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        ms = float(dt) * 1e3 / max(args.steps, 1)
        payload = ex.last.reduced_bytes
        line["exchange"] = {"ms_per_step": ms, "grad_bytes_per_rank": payload,
                            "algbw_GBps": payload / (ms * 1e-3) / 1e9, "collectives_per_step": ex.last.collectives,
                            "union_rows": ex.last.union_rows}
        dist.destroy_process_group()

    if rank == 0:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
