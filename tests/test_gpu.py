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
