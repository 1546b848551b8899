"""Randomised stress of hidegs_sort_tile_pairs' hot-tile paths (scouts, partition queue, WIDE jobs,
deferred pieces): many random skewed views and injected hot tiles, each result compared with torch's
stable sort of the same keys on the GPU (equal keys keep input order), the queue's error word clear.

With --with-exchange a second host thread runs the view-DP exchange with its overlapped masked Adam
step (every RCCL call forced on a one-rank group, 1M Gaussians) on its own stream the whole time, as
config 4's ranks do beside their binning (randomised).

usage: python tools/queue_stress.py [SECONDS] [SEED] [--with-exchange]
       (prints one line per case, FAIL lines on mismatch)"""
import os
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import primitives, synthetic  # noqa: E402


def case_keys(g, cam, i):
    kind = i % 3
    if kind == 0:  # a D2 view with a disc of Gaussians
        n = int(torch.randint(200_000, 2_000_001, (1,), generator=g))
        frac = float(torch.rand(1, generator=g)) * 0.9
        rad = 0.005 + float(torch.rand(1, generator=g)) * 0.2
        wl = synthetic.d2_binning_workload(synthetic.d2_scene(n, cam, seed=int(torch.randint(0, 1 << 30, (1,), generator=g)),
                                                              cluster=(frac, rad)), cam, device="cuda")
        return wl.keys, wl.values, wl.num_tiles, f"D2 n={n} cluster=({frac:.2f},{rad:.3f})"
    T = 8160
    k = int(torch.randint(100_000, 6_000_001, (1,), generator=g))
    tiles = torch.randint(0, T, (k,), generator=g)
    if kind == 1:  # hot tiles of random sizes injected into uniform keys
        nhot = int(torch.randint(1, 65, (1,), generator=g))
        hot = torch.randint(0, T, (nhot,), generator=g)
        share = float(torch.rand(1, generator=g))
        pick = torch.rand(k, generator=g) < share
        tiles[pick] = hot[torch.randint(0, nhot, (int(pick.sum()),), generator=g)]
        desc = f"inject k={k} hot={nhot} share={share:.2f}"
    else:  # few distinct depths (ties everywhere) and a narrow or wide depth range
        desc = f"ties k={k}"
    lo, hi = sorted((0.2 + 99.8 * torch.rand(2, generator=g)).tolist())
    depth = lo + (hi - lo) * torch.rand(k, generator=g)
    if kind == 2:
        depth = torch.round(depth * 4) / 4
        tiles[: k // 2] = int(torch.randint(0, T, (1,), generator=g))
    keys = (tiles.to(torch.int64) << 32) | depth.view(torch.int32).to(torch.int64)
    vals = torch.arange(k, dtype=torch.int32)
    return keys.cuda(), vals.cuda(), T, desc + f" depth=[{lo:.1f},{hi:.1f}]"


def start_exchange_load():
    """A thread looping forced-RCCL exchange_and_step on its own stream; returns (stop event, thread,
    counter, errors)."""
    import torch.distributed as dist

    from hidegs_amd.optim import Adam
    from hidegs_amd.view_dp import LEAF_WIDTHS, GradArena, ViewDPExchange
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    n = 1_000_000
    g = torch.Generator(device="cuda").manual_seed(3)
    visible = torch.rand(n, device="cuda", generator=g) < 0.9
    params = {k: torch.nn.Parameter(torch.randn(n, w, device="cuda", generator=g)) for k, w in LEAF_WIDTHS.items()}
    arena = GradArena(n, device="cuda")
    arena.attach(params)
    arena.flat.normal_(generator=g)
    opt = Adam(list(params.values()), lr=1e-4, eps=1e-15)
    ex = ViewDPExchange(bucket_bytes=16 << 20, compact_below=0.0, force_collectives=True, timeout=120)
    stop, count, errors = threading.Event(), [0], []
    stream = torch.cuda.Stream()

    def loop():
        try:
            with torch.cuda.stream(stream):
                while not stop.is_set():
                    ex.exchange_and_step(arena, visible, opt, params)
                    count[0] += 1
            stream.synchronize()
        except Exception as e:  # noqa: BLE001 -- reported by main
            errors.append(e)

    th = threading.Thread(target=loop)
    th.start()
    return stop, th, count, errors


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    budget = float(args[0]) if args else 120.0
    g = torch.Generator().manual_seed(int(args[1]) if len(args) > 1 else 1)
    load = start_exchange_load() if "--with-exchange" in sys.argv else None
    cam = synthetic.d2_camera(1920, 1080)
    t0, i, fails = time.time(), 0, 0
    primitives.queue_error()
    while time.time() - t0 < budget:
        keys, vals, T, desc = case_keys(g, cam, i)
        _, perm = torch.sort(keys, stable=True)
        ko, vo, _ = primitives.sort_tile_pairs(keys, vals, T)
        ok = bool(torch.equal(ko, keys[perm]) and torch.equal(vo, vals[perm]))
        qerr = primitives.queue_error()
        if not ok or qerr:
            fails += 1
        print(f"{'ok  ' if ok and not qerr else 'FAIL'} case {i}: {desc} qerr {qerr}", flush=True)
        i += 1
        del keys, vals, ko, vo, perm
    if load is not None:
        stop, th, count, errors = load
        stop.set()
        th.join(120)
        if errors or th.is_alive():
            fails += 1
        print(f"exchange_and_step beside the sorts: {count[0]} steps, errors {errors}", flush=True)
        import torch.distributed as dist
        dist.destroy_process_group()
    print(f"{i} cases, {fails} failures", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
