"""View-data-parallel exchange over gloo, world sizes 2 and 3, on CPU.

Each rank builds synthetic per-view gradients with its own visibility mask (rows a view
does not see are zero, as the rasterizer's backward produces them), runs one exchange
step and checks the result against the sum / max / OR computed locally from every
rank's regenerated inputs.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hidegs_amd.view_dp import LEAF_WIDTHS, ViewDPExchange, pack_mask, unpack_mask, view_index

N = 1000


def rank_inputs(rank, n=N):
    g = torch.Generator().manual_seed(1234 + rank)
    visible = torch.rand(n, generator=g) < (0.3 + 0.1 * rank)
    grads = {}
    for name, w in LEAF_WIDTHS.items():
        t = torch.randn(n, w, generator=g)
        t[~visible] = 0.0
        grads[name] = t
    grad_norm_max = torch.rand(n, generator=g) * visible
    max_radii = (torch.rand(n, generator=g) * 10).floor() * visible
    denom = visible.float()
    return visible, grads, grad_norm_max, max_radii, denom


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank, world, port, compact, bucket_bytes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        visible, grads, gmax, rmax, denom = rank_inputs(rank)
        ex = ViewDPExchange(bucket_bytes=bucket_bytes, compact=compact)
        union = ex.exchange(grads, visible, max_stats=[gmax, rmax], sum_stats=[denom])
        # expected values from every rank's regenerated inputs
        all_in = [rank_inputs(r) for r in range(world)]
        exp_union = torch.zeros(N, dtype=torch.bool)
        for v, *_ in all_in:
            exp_union |= v
        err = 0.0
        for name in LEAF_WIDTHS:
            exp = sum(a[1][name] for a in all_in)
            err = max(err, float((grads[name] - exp).abs().max()))
        ok = (torch.equal(union, exp_union)
              and err < 1e-5
              and torch.equal(gmax, torch.stack([a[2] for a in all_in]).max(0).values)
              and torch.equal(rmax, torch.stack([a[3] for a in all_in]).max(0).values)
              and torch.equal(denom, sum(a[4] for a in all_in)))
        if rank == 0:
            q.put((ok, err, ex.last.union_rows, ex.last.collectives, int(exp_union.sum())))
    finally:
        dist.destroy_process_group()


def run(world, compact, bucket_bytes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, compact, bucket_bytes, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return q.get(timeout=10)


@pytest.mark.parametrize("world,compact,bucket_bytes", [(2, True, 64 << 20), (2, False, 64 << 20),
                                                        (2, True, 4096), (3, True, 1000)])
def test_exchange_matches_local_reduction(world, compact, bucket_bytes):
    ok, err, union_rows, collectives, exp_rows = run(world, compact, bucket_bytes)
    assert ok, f"max grad error {err}"
    assert union_rows == (exp_rows if compact else N)
    if bucket_bytes < 4 * 59 * N:  # small buckets -> more than one SUM collective
        assert collectives > 1 + 2 + 1 + 1


def test_pack_roundtrip():
    g = torch.Generator().manual_seed(0)
    for n in (0, 1, 7, 8, 9, 1000, 1023):
        m = torch.rand(n, generator=g) < 0.5
        assert torch.equal(unpack_mask(pack_mask(m), n), m)


def test_view_index_partition():
    world = 8
    seen = [view_index(s, r, world) for s in range(5) for r in range(world)]
    assert sorted(seen) == list(range(5 * world))


def test_exchange_rejects_bad_inputs():
    ex = ViewDPExchange()
    with pytest.raises(ValueError):
        ex.sum_gradients([torch.zeros(3, 2), torch.zeros(4, 2)])
    with pytest.raises(ValueError):
        ex.sum_gradients([torch.zeros(3, 2, dtype=torch.float64)])
    with pytest.raises(ValueError):
        ex.sum_gradients([torch.zeros(2, 3).t()])
    with pytest.raises(ValueError):
        ViewDPExchange(bucket_bytes=2)
