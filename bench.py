"""bench.py -- BASELINE.json metric: fwd+bwd iters/s and HBM GB/s at 2M Gaussians, 1920x1080.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 without a torch.distributed environment: this process starts
  `python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child (before touching
  any GPU), relays rank 0's JSON line and exits with the child's status.  Under the driver's
  own torch.distributed.run launch the ranks are already there.  --backend gloo runs the
  multi-rank plumbing on CPU (the exchange leg only; tests/test_bench.py).

The headline metric needs the rasterizer forward + backward, whose kernels were refused
("Decisions in force"), so `value` is null -- never estimated.  What the repo builds
on this path is measured for real, at the configuration the metric is quoted on (config 3:
2M Gaussians, one 1920x1080 view per rank, synthetic D2 scene resident in HBM):

  step      = the binning stage of the rank's view: inclusive scan of the 2M tiles_touched
              and one hidegs_sort_tile_pairs call -- the stable radix sort of the K ~ 8.6M
              (tile | depth, id) pairs over [0, 32 + getHigherMsb(8160)) = [0, 45) plus the
              tile ranges (rasterizer_impl.cu:321-371).  Pairs from D2's own screen-space
              footprints (synthetic.d2_binning_workload).  W warm-up steps, then K timed steps
              between HIP events on the launch stream, barrier + synchronize on both sides,
              max over ranks.
  roofline  = the dominant kernel of the step: 24 algorithmic bytes per pair per sort-pass
              launch (key 8 + value 4, read and written once), averaged over its launches with
              per-launch HIP events (hidegs_kernel_timing), against 8 TB/s; traffic from the
              committed rocprofv3 PMC summary (profiles/latest_kernels.json), with the commit and
              source hash it was taken at (profiles/latest_kernels.meta.json).
  binning_skewed = the same step on a view whose Gaussians crowd into hot tiles (15% of them in
              a small disc: ~70 tiles over 8192 pairs take the partition queue).
  distCUDA2 = simple_knn._C.distCUDA2 on the 2M D2 centres, with its issue-rate roofline (VALU
              wave-instructions per second from the committed PMC summary, against the chip's).
  config2_scale / config5_scale = the binning step and distCUDA2 at config 2's size (100k Gaussians,
              1080p) and config 5's (10M Gaussians, 4K frame).  binning_skewed and the config scales
              are single-GPU sub-metrics: measured at N = 1 only.
  exchange  = the view-DP exchange of 2M x 59 fp32 leaf gradients + stats over RCCL (no
              collective at N = 1), HIP-event timed; algbw and ring busbw.  exchange_bf16: the same
              with the bf16 wire (all-to-all + fp32 sums + all-gather; view_dp.py, transport="bf16").
  exchange_and_step = the exchange followed by the masked step, sequential and overlapped.
  dp_step   = the rank's binning step + exchange_and_step, per wire format: the built part of one
              view-DP training step (steps/s over all ranks; no rasterizer), for the scaling runs.  At
              N = 1 the group issues no collective, so it is binning + masked Adam only (the keys say so:
              binning_adam_steps_per_s); every exchange sub-line carries its collective count and
              "rasterizer": false.
  fail fast = init_process_group(timeout=--pg-timeout): RCCL's watchdog ends a rank whose collective
              never completes; gloo exchange waits are bounded on the host (view_dp.py).
  masked Adam = the fused row-masked optimizer step at 2M Gaussians (59 fp32 each), 90% visible.
  cpu_baseline = on rank 0 at N = 1, every CPU leg on the same `cores` threads (cpu_share(): the
              CPUs the process may run on, lowered to a cgroup quota, else to the harness's declared
              share; the evidence is in the line): the oracle's OpenMP stable radix sort of the same
              pairs (headline), its kNN brute force on sampled queries, its masked Adam step.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import math
import platform
import socket
import subprocess
import sys
import time

N_GAUSSIANS = 2_000_000
W_PX, H_PX = 1920, 1080
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 fp32 VALU instruction per SIMD per 2 cycles at 2.4 GHz
VALU_PEAK_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 2
ROOT = os.path.dirname(os.path.abspath(__file__))
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "latest_kernels.json")  # tools/prof_summary.py output
KNN_PMC_FILE = os.path.join(ROOT, "profiles", "latest_knn_pmc.json")   # tools/pmc_knn_valu.sh output
TRAFFIC_META = os.path.join(ROOT, "profiles", "latest_kernels.meta.json")  # where that summary was taken
SKEW_CLUSTER = (0.15, 0.1)
SCOUTS = 128  # HIDEGS_SCOUTS (primitives.hip): segment_sort_kernel launches num_tiles + SCOUTS workgroups
# the bench's kernel names (hidegs_kernel_timing) -> rocprofv3 kernel names
ROCPROF_NAME = {"radix_scatter_u64": "radix_scatter_kernel", "segment_sort": "segment_sort_kernel",
                "radix_hist_u64": "radix_hist_kernel", "scan_downsweep": "scan_downsweep_kernel",
                "scan_reduce": "scan_reduce_kernel"}
# the binning sort's kernels (every launch of hidegs_sort_tile_pairs)
SORT_KERNELS = ("radix_hist_u64", "radix_digit_scan", "radix_scatter_u64", "segment_sort", "big_segments", "piece_sort")


def sources_sha256() -> str:
    """One hash over the library's kernel sources and the ABI header: identifies the code a committed
    profile was taken on (tools/profile_note.py records it beside the profile)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "hidegs_amd", "csrc")
    for f in sorted(os.listdir(csrc)) + ["../../include/hidegs.h"]:
        p = os.path.join(csrc, f)
        if os.path.isfile(p) and p.endswith((".hip", ".h", ".cpp")):
            h.update(os.path.basename(p).encode())
            with open(p, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def traffic_entry(dom: str, K: int, T: int, table: dict):
    """(key, entry) of the committed rocprofv3 summary for the bench's dominant kernel: the entry of
    the same kernel and grid (workgroups x 256 or x 512 threads), else that kernel's entry with the
    most launches, else (None, None)."""
    name = ROCPROF_NAME.get(dom, dom + "_kernel")
    ntiles = (K + 4095) // 4096
    grid = {"segment_sort": (T + SCOUTS) * 256, "radix_scatter_u64": ntiles * 512}.get(dom, ntiles * 256)
    key = f"{name}@{grid}"
    if key in table:
        return key, table[key]
    same = [(k, v) for k, v in table.items() if k.split("@")[0] == name]
    if same:
        return max(same, key=lambda kv: kv[1].get("launches", 0))
    return None, None


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


def _cgroup_cpu_quota():
    """(CPUs allowed by the cgroup CPU quota, the raw setting), or (None, setting) when unlimited or
    unreadable: cgroup v2 cpu.max ("max 100000" / "1600000 100000"), else v1 cfs quota / period."""
    paths = []
    try:
        for line in open("/proc/self/cgroup"):
            _, ctrl, path = line.rstrip("\n").split(":", 2)
            if ctrl == "":
                paths.append(("v2", os.path.join("/sys/fs/cgroup", path.lstrip("/"), "cpu.max")))
                paths.append(("v2", "/sys/fs/cgroup/cpu.max"))
            elif "cpu" in ctrl.split(","):
                for root in ("/sys/fs/cgroup/cpu,cpuacct", "/sys/fs/cgroup/cpu"):
                    paths.append(("v1", os.path.join(root, path.lstrip("/"))))
                    paths.append(("v1", root))
    except OSError:
        pass
    for kind, p in paths:
        try:
            if kind == "v2":
                raw = open(p).read().strip()
                q, per = raw.split()
                return (None if q == "max" else -(-int(q) // int(per))), f"{p}: {raw}"
            q = int(open(os.path.join(p, "cpu.cfs_quota_us")).read())
            per = int(open(os.path.join(p, "cpu.cfs_period_us")).read())
            raw = f"{p}: cfs_quota_us {q} / cfs_period_us {per}"
            return (None if q <= 0 else -(-q // per)), raw
        except (OSError, ValueError):
            continue
    return None, "no cgroup cpu quota file readable"


def cpu_share() -> dict:
    """The CPU legs' thread count and its evidence (BASELINE.md §4 asks for os.cpu_count()):
    * the CPUs this process may run on (sched_getaffinity) -- the allowed count;
    * lowered to the cgroup CPU quota when one is set;
    * with neither lower than os.cpu_count(), lowered to OMP_NUM_THREADS when the harness declares a
      smaller per-GPU share there (the GPU box sets 16 and asks worker pools to stay within it)."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    quota, quota_raw = _cgroup_cpu_quota()
    env = os.environ.get("OMP_NUM_THREADS", "")
    omp = int(env) if env.isdigit() and int(env) > 0 else None
    cores, source = allowed, "sched_getaffinity"
    if quota is not None and quota < cores:
        cores, source = quota, "cgroup cpu quota"
    elif quota is None and omp is not None and omp < cores:
        cores, source = omp, ("OMP_NUM_THREADS: the harness's declared per-GPU CPU share (no cgroup quota and "
                              "no narrower affinity visible)")
    return {"cores": cores, "cores_source": source, "sched_getaffinity": allowed, "cgroup_cpu_quota": quota,
            "cgroup_cpu_setting": quota_raw, "omp_num_threads": omp, "host_cpu_count": os.cpu_count()}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--knn-steps", type=int, default=5)
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: CPU ranks, the exchange leg only (plumbing tests)")
    ap.add_argument("--n-gaussians", type=int, default=N_GAUSSIANS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exchange", action="store_true")
    ap.add_argument("--no-adam", action="store_true")
    ap.add_argument("--no-config5", action="store_true", help="skip the config 2 and config 5 scale sub-metrics")
    ap.add_argument("--no-skewed", action="store_true")
    ap.add_argument("--pg-timeout", type=float, default=300.0,
                    help="seconds: the process group's timeout (RCCL watchdog: a collective that never completes "
                         "ends the process) and the exchange's bounded host waits (gloo)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """Start N ranks as a child torch.distributed.run (nothing here has touched a GPU) and relay
    rank 0's JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    for ln in lines[-1:]:
        print(ln, flush=True)
    if proc.returncode == 0 and not lines:
        print("bench.py: the ranks printed no result line", file=sys.stderr)
        return 1
    return proc.returncode


def main() -> None:
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))

    # The contract is ONE JSON line on stdout; RCCL prints a version banner there at init, so the
    # process's fd 1 goes to stderr for the run and the result line is written to the saved fd.
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    gpu = args.backend == "nccl"
    if gpu:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ["MASTER_PORT"] = str(free_port())
        kw = {"device_id": dev} if gpu else {}
        # fail fast: a rank that stalls or dies ends the run within the timeout instead of hanging
        # it -- the RCCL process group's watchdog ends a rank whose collective is older than this; gloo
        # operations time out after it
        dist.init_process_group(args.backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.pg_timeout), **kw)

    from hidegs_amd import synthetic
    from hidegs_amd.view_dp import GradArena, ViewDPExchange

    N = args.n_gaussians

    def max_over_ranks(x: float) -> float:
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)

    def timed(fn, steps, warmup):
        """(device ms per step from events on the current stream, wall ms per step), max over ranks."""
        for _ in range(warmup):
            fn()
        dist.barrier()
        if gpu:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        if gpu:
            e0.record()
        for _ in range(steps):
            fn()
        if gpu:
            e1.record()
            torch.cuda.synchronize()
        dist.barrier()
        wall = (time.perf_counter() - t0) * 1e3 / steps
        dev_ms = e0.elapsed_time(e1) / steps if gpu else wall
        return max_over_ranks(dev_ms), max_over_ranks(wall)

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
        "dtype": "u64/u32 (binning), f32 (distCUDA2, exchange, masked Adam)",
        "data": "synthetic (SURVEY §8(d) D2 scene, seeded per rank)",
        "config": {"workload": "config 3: 2M Gaussians, 1920x1080, one view per rank -- binning stage, "
                               "distCUDA2, the view-DP exchange and the masked step measured; rasterizer "
                               "fwd/bwd refused (not built)",
                   "n_gaussians": N, "width": W_PX, "height": H_PX, "parallelism": f"view-dp{world}",
                   "backend": "rccl" if gpu else "gloo"},
        "status": "headline UNMEASURED: the rasterizer forward/backward kernels were refused "
                  "(DESIGN.md, 'Decisions in force'); value stays null",
        "roofline": None,
        "cpu_baseline": None,
        "fail_fast": {"process_group_timeout_s": args.pg_timeout, "exchange_host_wait_timeout_s": args.pg_timeout,
                      "rccl": "the watchdog ends a rank whose collective is older than the process group "
                              "timeout; the exchange's waits are stream waits (no host block)",
                      "gloo": "every exchange wait bounded on the host, RuntimeError naming the collective"},
    }
    cam = synthetic.d2_camera(W_PX, H_PX)
    scene = synthetic.d2_scene(N, cam, seed=rank)

    ctx = {}
    if gpu:
        _gpu_legs(args, line, ctx, world, rank, dev, cam, scene, timed, np, torch)
    if not args.no_exchange:
        _exchange_legs(args, line, ctx, world, rank, dev, N, timed, gpu, torch, GradArena, ViewDPExchange)
    if gpu and rank == 0 and world == 1 and not args.no_cpu_baseline:
        _cpu_baselines(line, ctx, N, cam, np)

    dist.destroy_process_group()
    sys.stdout.flush()
    if rank == 0:
        os.write(result_fd, (json.dumps(line) + "\n").encode())


def _gpu_legs(args, line, ctx, world, rank, dev, cam, scene, timed, np, torch):
    import simple_knn
    from hidegs_amd import _lib, primitives, synthetic

    N = scene.n
    # ---- the step: binning of one view (rank r renders its own view: seed r) -------------------
    wl = synthetic.d2_binning_workload(scene, cam, device=dev)
    K, T = wl.num_pairs, wl.num_tiles
    end_bit = 32 + primitives.higher_msb(T)
    offsets = torch.empty_like(wl.tiles_touched)
    V = int((wl.tiles_touched > 0).sum())
    Px = cam.width * cam.height
    line["config"].update({"tiles": T, "pairs_K": K, "visible_V": V, "pixels_Px": Px,
                           "sort_bits": [0, end_bit],
                           # the fwd+bwd iteration's algorithmic bytes at this view (the
                           # headline's denominator were the rasterizer built); the binning sort's share
                           # of it is the 24 B/pair sort term
                           "B_iter_bytes": 288 * N + 542 * V + 164 * K + 112 * Px + 24 * T})

    def make_step(w):
        off = torch.empty_like(w.tiles_touched)

        def step():
            primitives.inclusive_scan_u32(w.tiles_touched, out=off)
            primitives.sort_tile_pairs(w.keys, w.values, w.num_tiles)  # SortPairs + identifyTileRanges
        return step

    step = make_step(wl)
    ms_step, wall_ms_step = timed(step, args.steps, args.warmup)
    qerr = primitives.queue_error()

    # per-kernel durations of the same step, live, with per-launch HIP events on the launch stream
    kt_steps = max(10, min(args.steps, 50))
    # algorithmic bytes per launch (SURVEY §8(d) D4 per-pair figures: a sort pass reads and writes
    # key 8 + value 4; a histogram pass reads the 8-byte keys; the scan reads and writes u32)
    alg = {"scan_reduce": 4 * N, "scan_small": 0, "scan_downsweep": 8 * N,
           "radix_hist_u64": 8 * K, "radix_digit_scan": 0, "radix_scatter_u64": 24 * K,
           "segment_sort": 24 * K, "big_segments": 0, "piece_sort": 0}

    def kernel_table(fn, nsteps):
        with _lib.kernel_timer() as kt:
            for _ in range(nsteps):
                fn()
            torch.cuda.synchronize()
            kern = {}
            for nm, nbytes in alg.items():
                ms, n = kt.get(nm)
                if n == 0:
                    continue
                avg_us = ms * 1e3 / n
                kern[nm] = {"avg_us": round(avg_us, 2), "launches_per_step": n // nsteps,
                            "us_per_step": round(ms * 1e3 / nsteps, 2),
                            "GBps": round(nbytes / (avg_us * 1e-6) / 1e9, 1) if nbytes else None}
        return kern

    kern = kernel_table(step, kt_steps)
    dom = max((k for k in kern if alg[k]), key=lambda k: kern[k]["us_per_step"])
    dom_us = kern[dom]["avg_us"]
    dom_bytes = alg[dom]
    achieved = dom_bytes / (dom_us * 1e-6) / 1e9
    traffic, traffic_key, meta = None, None, {}
    if os.path.exists(TRAFFIC_FILE):
        with open(TRAFFIC_FILE) as f:
            traffic_key, ent = traffic_entry(dom, K, T, json.load(f))
        traffic = (ent or {}).get("hbm_bytes_per_launch")
    if os.path.exists(TRAFFIC_META):
        with open(TRAFFIC_META) as f:
            meta = json.load(f)
    sort_us = sum(kern[k]["us_per_step"] for k in kern if k in SORT_KERNELS)
    line["binning_step"] = {"ms_per_step": round(ms_step, 4), "wall_ms_per_step": round(wall_ms_step, 4),
                            "timed_region": "inclusive scan of tiles_touched + hidegs_sort_tile_pairs (sort + "
                                            "tile ranges); no key emission, no rasterizer",
                            "pairs_per_s_all_ranks": K * world / (ms_step * 1e-3),
                            "binning_steps_per_s_all_ranks": world / (ms_step * 1e-3),
                            "sort_us": round(sort_us, 2), "queue_error": qerr, "kernels": kern}
    line["roofline"] = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                        "traffic": None if traffic is None else round(traffic),
                        # traffic is NOT measured in this run: it is the committed PMC summary's, taken at
                        # traffic_profile_commit on the kernel sources hashed there (same_source: this run's
                        # sources hash the same)
                        "traffic_profile": traffic_key, "traffic_profile_commit": meta.get("commit"),
                        "traffic_profile_same_source": (meta.get("sources_sha256") == sources_sha256()
                                                        if meta.get("sources_sha256") else None),
                        "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_us": dom_us}
    line["ms_per_step_binning"] = round(ms_step, 4)

    # ---- the same step on a skewed view (hot tiles through the partition queue) ----------------
    if not args.no_skewed and world == 1:  # single-GPU sub-metric (N > 1 ranks skip its CPU-side scene)
        sk_scene = synthetic.d2_scene(N, cam, seed=1000 + rank, cluster=SKEW_CLUSTER)
        wls = synthetic.d2_binning_workload(sk_scene, cam, device=dev)
        counts = torch.bincount((wls.keys >> 32).long(), minlength=wls.num_tiles)
        sk_step = make_step(wls)
        ms_sk, _ = timed(sk_step, max(20, args.steps // 4), 3)
        qerr_sk = primitives.queue_error()
        ksk = kernel_table(sk_step, 10)
        line["binning_skewed"] = {"workload": f"D2 with {SKEW_CLUSTER[0]:.0%} of the Gaussians in a disc of NDC "
                                              f"radius {SKEW_CLUSTER[1]}",
                                  "pairs_K": wls.num_pairs, "max_tile_pairs": int(counts.max()),
                                  "tiles_over_8192": int((counts > 8192).sum()),
                                  "tiles_over_2048": int((counts > 2048).sum()),
                                  "ms_per_step": round(ms_sk, 4), "queue_error": qerr_sk,
                                  "kernels_us_per_step": {k: v["us_per_step"] for k, v in ksk.items()}}
        del sk_scene, wls, counts

    # ---- distCUDA2 at 2M -------------------------------------------------------------------------
    pts = scene.means3D.to(dev)
    knn_ms, _ = timed(lambda: simple_knn._C.distCUDA2(pts), args.knn_steps, 1)
    with _lib.kernel_timer() as kt:
        simple_knn._C.distCUDA2(pts)
        torch.cuda.synchronize()
        kk = {nm: round(kt.get(nm)[0] * 1e3, 1) for nm in ("bounds", "morton", "radix_scatter_u64", "gather",
                                                             "leaf_box", "knn_leaf", "knn_hard")}
    # bound by the search's dependent evaluation chain (VALU issue), not HBM: 16 B/point in ~1 ms is
    # 0.4% of the HBM peak, so no HBM fraction is reported for it -- the issue roofline below is the bound
    kd = {"points": N, "ms": round(knn_ms, 3), "points_per_s_all_ranks": N * world / (knn_ms * 1e-3),
          "kernels_us": kk, "algorithmic_bytes": 16 * N, "bound": "valu-issue (search latency), not HBM"}
    if os.path.exists(KNN_PMC_FILE):
        with open(KNN_PMC_FILE) as f:
            pmc = json.load(f)
        leaf = pmc.get("knn_leaf_kernel")
        if leaf and leaf.get("SQ_INSTS_VALU") and kk.get("knn_leaf"):
            rate = leaf["SQ_INSTS_VALU"] / (kk["knn_leaf"] * 1e-6)
            kd["issue_roofline"] = {"kernel": "knn_leaf", "bound": "valu-issue",
                                    "valu_wave_instr_per_launch": leaf["SQ_INSTS_VALU"],
                                    "achieved_wave_instr_per_s": rate, "peak_wave_instr_per_s": VALU_PEAK_WAVE_INSTR_PER_S,
                                    "frac": round(rate / VALU_PEAK_WAVE_INSTR_PER_S, 4), "pmc_source": KNN_PMC_FILE[len(ROOT) + 1:]}
    line["distCUDA2"] = kd

    # ---- config 2's scale: 100k Gaussians, 1920x1080 ------------------------------------------------
    if not args.no_config5 and world == 1:  # single-GPU sub-metric, like config 5's below
        sc2 = synthetic.d2_scene(100_000, cam, seed=rank)
        wl2 = synthetic.d2_binning_workload(sc2, cam, device=dev)
        ms2, _ = timed(make_step(wl2), 50, 5)
        pts2 = sc2.means3D.to(dev)
        knn2_ms, _ = timed(lambda: simple_knn._C.distCUDA2(pts2), 10, 2)
        line["config2_scale"] = {"workload": "100k D2 Gaussians, 1920x1080 (8160 tiles): binning step and distCUDA2",
                                 "binning_ms_per_step": round(ms2, 4), "pairs_K": wl2.num_pairs,
                                 "distCUDA2_ms": round(knn2_ms, 3), "queue_error": primitives.queue_error()}
        del sc2, wl2, pts2

    # ---- config 5's scale: 10M Gaussians, 3840x2160 frame ----------------------------------------
    if not args.no_config5 and world == 1:  # single-GPU sub-metric (a 10M scene per rank is CPU time)
        cam5 = synthetic.d2_camera(3840, 2160)
        sc5 = synthetic.d2_scene(10_000_000, cam5, seed=rank)
        wl5 = synthetic.d2_binning_workload(sc5, cam5, device=dev)
        step5 = make_step(wl5)
        ms5, _ = timed(step5, 20, 3)
        pts5 = sc5.means3D.to(dev)
        knn5_ms, _ = timed(lambda: simple_knn._C.distCUDA2(pts5), 3, 1)
        line["config5_scale"] = {"workload": "10M D2 Gaussians, 3840x2160 (32400 tiles): binning step and distCUDA2",
                                 "binning_ms_per_step": round(ms5, 4), "pairs_K": wl5.num_pairs,
                                 "sort_bits": [0, 32 + primitives.higher_msb(wl5.num_tiles)],
                                 "pairs_per_s_all_ranks": wl5.num_pairs * world / (ms5 * 1e-3),
                                 "distCUDA2_ms": round(knn5_ms, 3), "queue_error": primitives.queue_error()}
        del sc5, wl5, pts5

    # ---- masked Adam at 2M ------------------------------------------------------------------------
    if not args.no_adam:
        from hidegs_amd.optim import Adam
        widths = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
        lrs = {"xyz": 0.00016 * 4.2, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005,
               "rotation": 0.001}
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        prm = {k: torch.nn.Parameter(torch.randn(N, w, device=dev, generator=g)) for k, w in widths.items()}
        for p in prm.values():
            p.grad = torch.randn(p.shape, device=dev, generator=g)
        vis = torch.rand(N, device=dev, generator=g) < 0.9
        opt = Adam([{"params": [prm[k]], "lr": lrs[k], "name": k} for k, w in widths.items()], lr=0.0, eps=1e-15)
        ad_ms, _ = timed(lambda: opt.step(vis), 20, 3)
        nvis = int(vis.sum())
        ad_bytes = 28 * 59 * nvis + N
        with _lib.kernel_timer() as kt:
            opt.step(vis)
            torch.cuda.synchronize()
            k_ms, k_n = kt.get("masked_adam")
        st = {k: (torch.zeros_like(p), torch.zeros_like(p)) for k, p in prm.items()}
        ref_t = [0]

        def ref_step():
            """OurAdam's masked, non-capturable path as torch ops on the same GPU (scene/OurAdam.py:266-337):
            gather the relevant rows, the two moment updates, bias_correction1/2 from the step count (host
            floats, as step_t.item()), denom = sqrt(v) / bias_correction2_sqrt + eps, addcdiv_ with
            -lr / bias_correction1, scatter the rows back."""
            ref_t[0] += 1
            bc1, bc2 = 1 - 0.9 ** ref_t[0], 1 - 0.999 ** ref_t[0]
            bc2_sqrt = math.sqrt(bc2)
            with torch.no_grad():
                for k, parami in prm.items():
                    m_all, v_all = st[k]
                    grad, exp_avg, exp_avg_sq, param = parami.grad[vis], m_all[vis], v_all[vis], parami[vis]
                    exp_avg.mul_(0.9).add_(grad, alpha=1 - 0.9)
                    exp_avg_sq.mul_(0.999).addcmul_(grad, grad.conj(), value=1 - 0.999)
                    denom = (exp_avg_sq.sqrt() / bc2_sqrt).add_(1e-15)
                    param.addcdiv_(exp_avg, denom, value=-(lrs[k] / bc1))
                    m_all[vis] = exp_avg
                    v_all[vis] = exp_avg_sq
                    parami[vis] = param
        ref_ms, _ = timed(ref_step, 5, 1)
        line["masked_adam"] = {"gaussians": N, "visible_rows": nvis, "ms": round(ad_ms, 4),
                               "kernel_us_total": round(k_ms * 1e3, 1), "launches": k_n,
                               "algorithmic_bytes": ad_bytes, "GBps": round(ad_bytes / (ad_ms * 1e-3) / 1e9, 1),
                               "hbm_frac": round(ad_bytes / (ad_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                               "reference_torch_ops_ms": round(ref_ms, 3),
                               "reference_torch_ops": "scene/OurAdam.py:266-337 masked path as torch ops on this "
                                                      "GPU, bias-corrected step_size and bias_correction2_sqrt",
                               "speedup_vs_reference_ops": round(ref_ms / ad_ms, 2)}
        ctx["adam_state"] = (prm, opt, vis, g)
    ctx["binning_pairs"] = (wl, end_bit, sort_us)
    ctx["binning_step"] = step


def _exchange_legs(args, line, ctx, world, rank, dev, N, timed, gpu, torch, GradArena, ViewDPExchange):
    import torch.distributed as dist
    g = torch.Generator(device=dev).manual_seed(rank)
    visible = torch.rand(N, device=dev, generator=g) < 0.9
    arena = GradArena(N, device=dev)
    arena.flat.normal_(generator=g)
    norm = torch.rand(N, 1, device=dev, generator=g)
    radii = torch.rand(N, device=dev, generator=g)
    reps = 20 if gpu else 3
    def replicas_identical(ex) -> bool:
        """One exchange of fresh per-rank gradients, then every rank's reduced arena compared bit for bit
        through 1024 int64 chunk sums of its int32 view (all-gathered: 8 KB per rank)."""
        arena.flat.normal_(generator=g)
        ex.exchange(arena, visible, max_stats=[norm, radii])
        flat = arena.flat.view(torch.int32)
        pad = (-flat.numel()) % 1024
        sums = torch.nn.functional.pad(flat, (0, pad)).view(1024, -1).to(torch.int64).sum(1)
        got = [torch.empty_like(sums) for _ in range(world)]
        dist.all_gather(got, sums)
        return all(torch.equal(x, got[0]) for x in got)

    for transport in ("fp32", "bf16"):
        ex = ViewDPExchange(transport=transport, timeout=args.pg_timeout)
        same = replicas_identical(ex)
        ex_ms, ex_wall = timed(lambda: ex.exchange(arena, visible, max_stats=[norm, radii]), reps, 2)
        nbytes = ex.last.reduced_bytes
        algbw = nbytes / (ex_ms * 1e-3) / 1e9 if nbytes else None
        line["exchange" if transport == "fp32" else "exchange_bf16"] = {
            "ms_per_step": round(ex_ms, 3), "wall_ms_per_step": round(ex_wall, 3), "world": world,
            "transport": transport,
            "timing": "HIP events on the compute stream (it waits for every RCCL bucket)" if gpu
            else "wall clock (gloo, CPU)",
            "grad_bytes_per_rank": nbytes, "wire_bytes_per_rank": ex.last.wire_bytes,
            "algbw_GBps": algbw,  # fp32 gradient bytes made consistent per second
            "busbw_GBps": None if algbw is None else algbw * 2 * (world - 1) / world,
            "collectives_per_step": ex.last.collectives, "compacted": ex.last.compacted,
            "union_rows": ex.last.union_rows, "replicas_bit_identical": same, "rasterizer": False,
            "timed_region": ("one-rank group: no collective, the visibility union only (the sum over one rank is "
                             "its input)" if ex.last.collectives == 0 else
                             f"{ex.last.collectives} collectives: visibility all-gather, gradient buckets, MAX")}
        if world == 1 and gpu:
            # the N-rank path forced on the one-rank group: every collective the multi-GPU run issues,
            # real RCCL calls (over one rank a copy), so the machinery's own cost is on the record
            exf = ViewDPExchange(transport=transport, force_collectives=True, timeout=args.pg_timeout)
            f_ms, _ = timed(lambda: exf.exchange(arena, visible, max_stats=[norm, radii]), reps, 2)
            line["exchange" if transport == "fp32" else "exchange_bf16"]["forced_one_rank_rccl"] = {
                "ms_per_step": round(f_ms, 3), "collectives_per_step": exf.last.collectives,
                "wire_bytes": exf.last.wire_bytes, "compacted": exf.last.compacted,
                "union_rows": exf.last.union_rows}
    st = ctx.get("adam_state")
    if st is not None:
        prm, opt, vis, g2 = st
        arena2 = GradArena(N, device=dev)
        for k, p in prm.items():
            arena2[k].copy_(p.grad)
        arena2.attach(prm)
        ex2 = ViewDPExchange(timeout=args.pg_timeout)
        norm2 = torch.rand(N, 1, device=dev, generator=g2)

        def seq_step():
            res = ex2.exchange(arena2, vis, max_stats=[norm2], params=prm)
            opt.step(res.union)

        seq_ms, _ = timed(seq_step, 10, 2)
        fused_ms, _ = timed(lambda: ex2.exchange_and_step(arena2, vis, opt, prm, max_stats=[norm2]), 10, 2)
        ex3 = ViewDPExchange(transport="bf16", timeout=args.pg_timeout)
        bf16_ms, _ = timed(lambda: ex3.exchange_and_step(arena2, vis, opt, prm, max_stats=[norm2]), 10, 2)
        line["exchange_and_step"] = {"world": world, "sequential_ms": round(seq_ms, 3),
                                     "overlapped_ms": round(fused_ms, 3), "overlapped_bf16_ms": round(bf16_ms, 3),
                                     "collectives": ex2.last.collectives, "union_rows": ex2.last.union_rows,
                                     "rasterizer": False,
                                     "timed_region": ("masked Adam step only (one-rank group: no collective)"
                                                      if ex2.last.collectives == 0 else
                                                      "view-DP exchange + masked Adam step")}
        bin_step = ctx.get("binning_step")
        if bin_step is not None:
            # what this build runs of one view-DP training step, the rasterizer aside: the rank's view's
            # binning, the exchange and the masked optimizer step (overlapped), per wire format
            dp = {"world": world, "rasterizer": False,
                  "includes": ("binning step + masked Adam; one-rank group: no collective, no rasterizer fwd/bwd "
                               "(refused)") if world == 1 else
                              "binning step + view-DP exchange + masked Adam (overlapped); no rasterizer fwd/bwd "
                              "(refused)"}
            for tag, exn in (("fp32", ex2), ("bf16", ex3)):
                ms, _ = timed(lambda: (bin_step(), exn.exchange_and_step(arena2, vis, opt, prm, max_stats=[norm2])),
                              10, 2)
                dp[f"{tag}_ms_per_step"] = round(ms, 3)
                dp[f"{tag}_collectives"] = exn.last.collectives
                rate = "binning_adam_steps_per_s" if world == 1 else "binning_exchange_adam_steps_per_s_all_ranks"
                dp[f"{tag}_{rate}"] = round(world / (ms * 1e-3), 1)
            line["dp_step"] = dp


def _cpu_baselines(line, ctx, N, cam, np):
    import oracle
    from hidegs_amd import synthetic
    share = cpu_share()
    threads = oracle.set_threads(share["cores"])
    info = {"cpu": cpu_model(), **share, "cores": threads}
    wl, end_bit, sort_us = ctx["binning_pairs"]
    keys = wl.keys.cpu().numpy().view(np.uint64)
    vals = wl.values.cpu().numpy().view(np.uint32)
    K = keys.size
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or (time.perf_counter() - t0 < 10.0 and reps < 30):
        oracle.sort_pairs_omp(keys, vals, 0, end_bit, threads)
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    line["cpu_baseline"] = {"value": K / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
                            "sample": f"stable sort of the same {K} (key, value) pairs over bits [0,{end_bit}) "
                                      f"(oracle/sort_ref.c, OpenMP radix sort on {threads} threads), {reps} reps",
                            **info, "gpu_speedup_sort": round(dt * 1e3 / (sort_us * 1e-3), 1)}
    # distCUDA2: the oracle's brute force for a sample of the 2M D2 queries, each against all points
    if "distCUDA2" in line:
        cpu_pts = synthetic.d2_scene(N, cam, seed=0).means3D.numpy()
        nq = 64 * threads
        idx = np.random.default_rng(0).choice(N, nq, replace=False)
        t0 = time.perf_counter()
        oracle.knn_mean3_subset(cpu_pts, idx)
        dq = time.perf_counter() - t0
        line["distCUDA2"]["cpu_baseline"] = {
            "value": nq / dq, "unit": "queries/s", "cores": threads, "kind": "port",
            "algorithm": "brute force over all points (the definition the oracle pins), NOT the reference's box "
                         "search (SK/simple_knn.cu:148-184): the GPU/CPU ratio is not like for like",
            "sample": f"{nq} of the {N} D2 queries, each brute-forced against all points (oracle/knn_ref.c, OpenMP)",
            "gpu_queries_per_s": line["distCUDA2"]["points_per_s_all_ranks"]}
        del cpu_pts
    # masked Adam: the oracle's restatement (oracle/adam_ref.c, OpenMP over rows), one full step
    if "masked_adam" in line:
        rng = np.random.default_rng(1)
        rel = rng.random(N) < 0.9
        t_total = 0.0
        for w in (3, 3, 45, 1, 3, 4):
            pa = rng.standard_normal((N, w), dtype=np.float32)
            ga = rng.standard_normal((N, w), dtype=np.float32)
            ma, va = np.zeros_like(pa), np.zeros_like(pa)
            t0 = time.perf_counter()
            oracle.masked_adam(pa, ga, ma, va, rel, 1e-3, 0.9, 0.999, 1e-15, 0.0, 1)
            t_total += time.perf_counter() - t0
        line["masked_adam"]["cpu_baseline"] = {
            "value": 1e3 * t_total, "unit": "ms per step", "cores": threads, "kind": "port",
            "sample": f"one full step, {N} Gaussians x 59 floats, 90% of rows relevant (oracle/adam_ref.c, OpenMP)"}


if __name__ == "__main__":
    main()
