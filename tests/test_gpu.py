"""GPU-box checks of the native library as a whole: it is the code that runs (mapped in the
process, gfx950 kernels launched), it fails loudly where nothing is built, and the view-DP
exchange runs over RCCL on device tensors."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_library_loaded_in_gpu_process(built_lib):
    import simple_knn
    simple_knn._C.distCUDA2(torch.rand(100, 3, device="cuda"))
    torch.cuda.synchronize()
    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert "libhidegs.so" in maps


def test_rasterizer_raises_instead_of_falling_back(built_lib):
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    d = "cuda"
    e = torch.empty(0, device=d)
    s = GaussianRasterizationSettings(64, 64, 0.5, 0.5, torch.zeros(3, device=d), 1.0, torch.eye(4, device=d),
                                      torch.eye(4, device=d), 3, torch.zeros(3, device=d), False, False, e.int(),
                                      e.int(), e.float(), e.int(), True, True)
    P = 16
    with pytest.raises(RuntimeError, match="unsupported"):
        GaussianRasterizer(s)(torch.rand(P, 3, device=d), torch.zeros(P, 3, device=d), torch.rand(P, 1, device=d),
                              shs=torch.zeros(P, 16, 3, device=d), scales=torch.ones(P, 3, device=d),
                              rotations=torch.ones(P, 4, device=d), all_map=torch.zeros(P, 5, device=d))


def test_view_dp_exchange_over_rccl_single_rank():
    import torch.distributed as dist
    from hidegs_amd.view_dp import LEAF_WIDTHS, ViewDPExchange
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 100_000
        g = torch.Generator(device="cuda").manual_seed(0)
        visible = torch.rand(n, device="cuda", generator=g) < 0.5
        grads = {k: torch.randn(n, w, device="cuda", generator=g) * visible[:, None] for k, w in LEAF_WIDTHS.items()}
        ref = {k: v.clone() for k, v in grads.items()}
        gmax = torch.rand(n, device="cuda", generator=g)
        res = ViewDPExchange(bucket_bytes=1 << 20, compact_below=1.0).exchange(grads, visible,
                                                                                max_stats=[gmax.clone()])
        torch.cuda.synchronize()
        assert torch.equal(res.union, visible)
        assert torch.equal(res.view_count.squeeze(1), visible.float())
        for k in grads:
            assert torch.equal(grads[k], ref[k])
    finally:
        dist.destroy_process_group()


def test_exchange_and_step_over_rccl_single_rank_equals_step():
    """exchange_and_step on a one-rank RCCL group: no collective, and the masked step on the union
    equals optimizer.step(visible) bit for bit."""
    import torch.distributed as dist
    from hidegs_amd.optim import Adam
    from hidegs_amd.view_dp import LEAF_WIDTHS, GradArena, ViewDPExchange
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 50_001
        g = torch.Generator(device="cuda").manual_seed(3)
        visible = torch.rand(n, device="cuda", generator=g) < 0.8
        init = {k: torch.randn(n, w, device="cuda", generator=g) for k, w in LEAF_WIDTHS.items()}
        grads = {k: torch.randn(n, w, device="cuda", generator=g) for k, w in LEAF_WIDTHS.items()}
        pa = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
        pb = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
        arena = GradArena(n, device="cuda")
        arena.attach(pb)
        for k in LEAF_WIDTHS:
            pa[k].grad = grads[k].clone()
            arena[k].copy_(grads[k])
        Adam(list(pa.values()), lr=0.01, eps=1e-15).step(visible)
        ex = ViewDPExchange(compact_below=0.0)
        res = ex.exchange_and_step(arena, visible, Adam(list(pb.values()), lr=0.01, eps=1e-15), pb)
        torch.cuda.synchronize()
        assert ex.last.collectives == 0 and torch.equal(res.union, visible)
        for k in LEAF_WIDTHS:
            assert torch.equal(pa[k].detach(), pb[k].detach()), k
    finally:
        dist.destroy_process_group()


def _one_rank_nccl():
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    return dist


@pytest.mark.parametrize("transport", ["fp32", "bf16"])
@pytest.mark.parametrize("compact_below", [0.0, 1.0])
def test_view_dp_collectives_on_rccl_forced_single_rank(transport, compact_below):
    """Every RCCL call of the N-rank exchange on real hardware: a one-rank group with the N-rank path
    forced (visibility all-gather, bucketed async all-reduce or bf16 all-to-all + all-gather, compacted
    or dense, the MAX all-reduce).  Over one rank the sum is the input (bf16 wire: rounded to bf16)."""
    from hidegs_amd.view_dp import LEAF_WIDTHS, ViewDPExchange
    dist = _one_rank_nccl()
    try:
        n = 100_003
        g = torch.Generator(device="cuda").manual_seed(11)
        visible = torch.rand(n, device="cuda", generator=g) < 0.4
        grads = {k: torch.randn(n, w, device="cuda", generator=g) * visible[:, None] for k, w in LEAF_WIDTHS.items()}
        ref = {k: (v.to(torch.bfloat16).float() if transport == "bf16" else v.clone()) for k, v in grads.items()}
        gmax = torch.rand(n, device="cuda", generator=g)
        gm = gmax.clone()
        ex = ViewDPExchange(bucket_bytes=1 << 20, compact_below=compact_below, transport=transport,
                            force_collectives=True)
        res = ex.exchange(grads, visible, max_stats=[gm])
        torch.cuda.synchronize()
        assert ex.last.collectives >= 3 and ex.last.compacted == (compact_below == 1.0)
        assert torch.equal(res.union, visible)
        assert torch.equal(res.view_count.squeeze(1), visible.float())
        assert torch.equal(gm, gmax)
        for k in grads:
            assert torch.equal(grads[k], ref[k]), k
    finally:
        dist.destroy_process_group()


def test_hot_tile_queue_beside_an_rccl_exchange_on_another_stream():
    """Config 4's concurrency: the binning sort of a skewed view -- hot tiles, so the
    partition queue's cross-workgroup hand-offs run -- on one stream and host thread, while the view-DP
    exchange with its overlapped masked Adam step (every RCCL call forced on a one-rank group) runs on
    another stream from the main thread, several iterations each, started together.  Every sort is
    bit-identical to oracle/binning.py, the queue's error word stays clear, the next call on the sort's
    stream does not raise HIDEGS_E_ASYNC, and the exchange still equals Adam.step on the union."""
    import threading

    import numpy as np

    from hidegs_amd import primitives, synthetic
    from hidegs_amd.optim import Adam
    from hidegs_amd.view_dp import LEAF_WIDTHS, GradArena, ViewDPExchange
    from oracle import binning

    iters = 6
    cam = synthetic.d2_camera(1920, 1080)
    wl = synthetic.d2_binning_workload(synthetic.d2_scene(2_000_000, cam, seed=1000, cluster=(0.15, 0.1)), cam)
    T = wl.num_tiles
    ek, ev = binning.stable_sort_pairs(wl.keys.numpy().view(np.uint64), wl.values.numpy().view(np.uint32), 0,
                                       32 + primitives.higher_msb(T))
    er = binning.tile_ranges(ek, T)
    ek_d, ev_d = torch.from_numpy(ek.view(np.int64)).cuda(), torch.from_numpy(ev.view(np.int32)).cuda()
    er_d = torch.from_numpy(er.view(np.int32)).cuda().view(T, 2)
    keys, vals = wl.keys.cuda(), wl.values.cuda()
    primitives.queue_error(clear=True)

    dist = _one_rank_nccl()
    try:
        n = 1_000_000
        g = torch.Generator(device="cuda").manual_seed(21)
        visible = torch.rand(n, device="cuda", generator=g) < 0.9
        init = {k: torch.randn(n, w, device="cuda", generator=g) for k, w in LEAF_WIDTHS.items()}
        grads = {k: torch.randn(n, w, device="cuda", generator=g) for k, w in LEAF_WIDTHS.items()}
        pa = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
        pb = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
        opt_a = Adam(list(pa.values()), lr=0.01, eps=1e-15)
        opt_b = Adam(list(pb.values()), lr=0.01, eps=1e-15)
        arena = GradArena(n, device="cuda")
        arena.attach(pb)
        for k in LEAF_WIDTHS:
            pa[k].grad = grads[k].clone()
        for _ in range(iters):
            opt_a.step(visible)
        ex = ViewDPExchange(bucket_bytes=16 << 20, compact_below=0.0, force_collectives=True)
        sort_stream, dp_stream = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        start = threading.Barrier(2)
        results, errors = [], []

        def sorter():
            try:
                with torch.cuda.stream(sort_stream):
                    start.wait()
                    for _ in range(iters):
                        results.append(primitives.sort_tile_pairs(keys, vals, T))
            except Exception as e:  # noqa: BLE001 -- re-raised on the main thread
                errors.append(e)

        th = threading.Thread(target=sorter)
        th.start()
        with torch.cuda.stream(dp_stream):
            start.wait()
            for _ in range(iters):
                for k in LEAF_WIDTHS:
                    arena[k].copy_(grads[k])
                ex.exchange_and_step(arena, visible, opt_b, pb)
        th.join(120)
        assert not th.is_alive() and not errors, errors
        torch.cuda.synchronize()
        assert len(results) == iters
        for it, (ko, vo, r) in enumerate(results):
            assert torch.equal(ko, ek_d) and torch.equal(vo, ev_d) and torch.equal(r, er_d), f"sort {it} differs"
        assert primitives.queue_error() == 0
        with torch.cuda.stream(sort_stream):  # raises RuntimeError on a pending HIDEGS_E_ASYNC
            ko, vo, _ = primitives.sort_tile_pairs(keys, vals, T)
        torch.cuda.synchronize()
        assert torch.equal(vo, ev_d)
        assert ex.last.collectives > len(LEAF_WIDTHS)
        for k in LEAF_WIDTHS:
            assert torch.equal(pa[k].detach(), pb[k].detach()), k
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("transport,blocking", [("fp32", False), ("bf16", False), ("fp32", True)])
def test_exchange_and_step_on_rccl_forced_single_rank(transport, blocking):
    """The overlapped path on hardware (every bucket's collective issued, then per bucket its wait
    and that bucket's rows' masked Adam step): equals Adam.step(visible) on the summed gradients.
    blocking=True: every RCCL wait bounded on the host (view_dp.py "Failure detection"), same result."""
    from hidegs_amd.optim import Adam
    from hidegs_amd.view_dp import LEAF_WIDTHS, GradArena, ViewDPExchange
    dist = _one_rank_nccl()
    try:
        n = 50_001
        g = torch.Generator(device="cuda").manual_seed(12)
        visible = torch.rand(n, device="cuda", generator=g) < 0.8
        init = {k: torch.randn(n, w, device="cuda", generator=g) for k, w in LEAF_WIDTHS.items()}
        grads = {k: torch.randn(n, w, device="cuda", generator=g) for k, w in LEAF_WIDTHS.items()}
        pa = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
        pb = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
        arena = GradArena(n, device="cuda")
        arena.attach(pb)
        for k in LEAF_WIDTHS:
            pa[k].grad = grads[k].to(torch.bfloat16).float() if transport == "bf16" else grads[k].clone()
            arena[k].copy_(grads[k])
        Adam(list(pa.values()), lr=0.01, eps=1e-15).step(visible)
        ex = ViewDPExchange(bucket_bytes=256 << 10, compact_below=0.0, transport=transport, force_collectives=True,
                            timeout=60, blocking=blocking)
        res = ex.exchange_and_step(arena, visible, Adam(list(pb.values()), lr=0.01, eps=1e-15), pb)
        torch.cuda.synchronize()
        assert ex.last.collectives > len(LEAF_WIDTHS) and torch.equal(res.union, visible)
        for k in LEAF_WIDTHS:
            assert torch.equal(pa[k].detach(), pb[k].detach()), k
    finally:
        dist.destroy_process_group()
