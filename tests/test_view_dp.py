"""View-data-parallel exchange over gloo, world sizes 2, 3, 4 and 8, on CPU.

Each rank builds synthetic per-view gradients with its own visibility mask (rows a view
does not see are zero, as the rasterizer's backward produces them), runs the exchange for
several steps starting from non-zero replicated densification state, and checks the
replicas against the reference's sequential semantics: processing the world's views one
after another with add_densification_stats (scene/gaussian_model.py:763-765):
    accum = max(accum, norm_v) on rows view v sees;  denom += 1 on those rows.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hidegs_amd.view_dp import (LEAF_WIDTHS, GradArena, ViewDPExchange, pack_mask, unpack_mask, view_index)

N = 1000
STEPS = 3


def rank_inputs(rank, step, n=N, pattern="rate"):
    """pattern "rate": rank r sees a random 30 + 10r % of the rows (the union nearly all rows at world >= 4);
    "window": rank r sees 90% of the rows in [r n/16, r n/16 + n/4) -- divergent views whose union over 8
    ranks is 11/16 of the rows, so the exchange compacts at world 8."""
    g = torch.Generator().manual_seed(1234 + 97 * rank + 7919 * step)
    if pattern == "window":
        rows = torch.arange(n)
        lo = rank * n // 16
        visible = (rows >= lo) & (rows < lo + n // 4) & (torch.rand(n, generator=g) < 0.9)
    else:
        visible = torch.rand(n, generator=g) < (0.3 + 0.1 * rank)
    grads = {}
    for name, w in LEAF_WIDTHS.items():
        t = torch.randn(n, w, generator=g)
        t[~visible] = 0.0
        grads[name] = t
    norm = torch.rand(n, 1, generator=g) * visible[:, None]
    radii = (torch.rand(n, generator=g) * 10).floor() * visible
    return visible, grads, norm, radii


def initial_state(n=N):
    g = torch.Generator().manual_seed(5)
    return torch.rand(n, 1, generator=g), (torch.rand(n, 1, generator=g) * 4).floor(), torch.rand(n, generator=g) * 3


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank, world, port, compact_below, bucket_bytes, use_arena, q, pattern="rate"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = ViewDPExchange(bucket_bytes=bucket_bytes, compact_below=compact_below, debug=True)
        accum, denom, max_radii = initial_state()
        e_accum, e_denom, e_radii = initial_state()
        ok, err, info = True, 0.0, None
        for step in range(STEPS):
            visible, grads, norm, radii = rank_inputs(rank, step, pattern=pattern)
            if use_arena:
                arena = GradArena(N)
                for k, v in grads.items():
                    arena[k].copy_(v)
                res = ex.exchange(arena, visible, max_stats=[norm, radii])
                reduced = {k: arena[k] for k in LEAF_WIDTHS}
            else:
                res = ex.exchange(grads, visible, max_stats=[norm, radii])
                reduced = grads
            # replicated-state update, as the train loop applies it after the exchange
            accum = torch.maximum(accum, norm)
            denom += res.view_count
            max_radii = torch.maximum(max_radii, radii)
            # expected: the world's views applied one after another (reference semantics)
            all_in = [rank_inputs(r, step, pattern=pattern) for r in range(world)]
            exp_union = torch.zeros(N, dtype=torch.bool)
            for v, g, nv, rv in all_in:
                exp_union |= v
                e_accum[v] = torch.maximum(nv[v], e_accum[v])
                e_denom[v] += 1
                e_radii[v] = torch.maximum(e_radii[v], rv[v])
            for name in LEAF_WIDTHS:
                exp = sum(a[1][name] for a in all_in)
                err = max(err, float((reduced[name] - exp).abs().max()))
            ok = ok and torch.equal(res.union, exp_union) and torch.equal(accum, e_accum) \
                and torch.equal(denom, e_denom) and torch.equal(max_radii, e_radii)
            # replicas bit-identical: every rank's reduced gradients and replicated state
            mine = torch.cat([reduced[k].reshape(-1) for k in LEAF_WIDTHS] + [accum.reshape(-1), denom.reshape(-1)])
            got = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(got, mine)
            ok = ok and all(torch.equal(x.view(torch.int32), got[0].view(torch.int32)) for x in got)
            info = (ex.last.union_rows, ex.last.collectives, ex.last.compacted, int(exp_union.sum()))
        if rank == 0:
            q.put((ok and err < 1e-5, err, info))
    finally:
        dist.destroy_process_group()


def run(world, compact_below, bucket_bytes, use_arena, pattern="rate"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, compact_below, bucket_bytes, use_arena, q, pattern))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return q.get(timeout=10)


@pytest.mark.parametrize("world,compact_below,bucket_bytes,use_arena,pattern,compacts", [
    (2, 1.0, 64 << 20, True, "rate", True),    # compacted (union < 100% of rows)
    (2, 0.0, 64 << 20, True, "rate", False),   # dense, in place on the arena
    (2, 0.0, 64 << 20, False, "rate", False),  # dense, separate tensors
    (2, 1.0, 4096, False, "rate", True),       # compacted, many buckets
    (3, 1.0, 1000, True, "rate", True),
    # world 8 (the driver's scaling node): divergent windows, union 11/16 < the default 0.75 -> compacted
    (8, 0.75, 4096, True, "window", True),
    (8, 0.0, 4096, True, "window", False),     # the same views, dense
    (8, 0.75, 64 << 20, True, "rate", False),  # union ~ all rows: the default stays dense
])
def test_multistep_exchange_matches_sequential_reference(world, compact_below, bucket_bytes, use_arena, pattern,
                                                         compacts):
    ok, err, (union_rows, collectives, compacted, exp_rows) = run(world, compact_below, bucket_bytes, use_arena,
                                                                  pattern)
    assert ok, f"max grad error {err} (or replicas differ)"
    assert union_rows == exp_rows
    assert compacted == compacts
    # one all-gather (masks) + SUM buckets + ONE fused MAX
    nbytes = 4 * 59 * (exp_rows if compacted else N)
    assert collectives == 1 + -(-nbytes // bucket_bytes) + 1


def test_pack_roundtrip():
    g = torch.Generator().manual_seed(0)
    for n in (0, 1, 7, 8, 9, 1000, 1023):
        m = torch.rand(n, generator=g) < 0.5
        assert torch.equal(unpack_mask(pack_mask(m), n), m)


def test_view_index_partition():
    world = 8
    seen = [view_index(s, r, world) for s in range(5) for r in range(world)]
    assert sorted(seen) == list(range(5 * world))


def test_arena_views_are_param_grads():
    arena = GradArena(10)
    p = torch.nn.Parameter(torch.zeros(10, 15, 3))
    q = torch.nn.Parameter(torch.zeros(10, 3))
    arena.attach({"f_rest": p, "xyz": q})
    (p.sum() * 2 + q.sum()).backward()
    assert p.grad.data_ptr() == arena["f_rest"].data_ptr()
    assert float(arena["f_rest"].sum()) == 2 * 450 and float(arena["xyz"].sum()) == 30
    assert arena.flat.numel() == 10 * 59


def test_exchange_rejects_bad_inputs():
    ex = ViewDPExchange()
    with pytest.raises(ValueError):
        ex.sum_gradients([torch.zeros(3, 2), torch.zeros(4, 2)])
    with pytest.raises(ValueError):
        ex.sum_gradients([torch.zeros(3, 2, dtype=torch.float64)])
    with pytest.raises(ValueError):
        ex.sum_gradients([torch.zeros(2, 3).t()])
    with pytest.raises(ValueError, match="union must be a bool mask"):
        ex.sum_gradients([torch.zeros(4, 2)], union=torch.ones(3, dtype=torch.bool))
    with pytest.raises(ValueError, match="union must be a bool mask"):
        ex.sum_gradients([torch.zeros(4, 2)], union=torch.ones(4))
    with pytest.raises(ValueError):
        ViewDPExchange(bucket_bytes=2)
    with pytest.raises(ValueError):
        ViewDPExchange(compact_below=1.5)


def test_debug_mode_catches_rows_outside_union():
    ex = ViewDPExchange(debug=True, compact_below=1.0)
    g = torch.zeros(6, 2)
    g[5] = 1.0
    union = torch.tensor([True, True, False, False, False, False])
    with pytest.raises(RuntimeError, match="outside the visibility union"):
        ex.sum_gradients([g], union=union)


class RecordingPlan:
    """Stands in for hidegs_amd.optim.AdamStepPlan on CPU: records which rows were stepped and what
    the arena held for them at that moment."""

    def __init__(self, arena, names):
        self.arena, self.names = arena, names
        self.calls, self.snap = [], {}

    def run(self):
        self.calls.append(("all", 0, 0))

    def run_rows(self, p, r0, r1):
        name = self.names[id(p)]
        self.calls.append((name, r0, r1))
        self.snap[(name, r0, r1)] = self.arena[name][r0:r1].clone()

    def run_except(self, params):
        self.rest_skipped = {self.names[id(p)] for p in params}


class RecordingOptimizer:
    def __init__(self, plan):
        self.plan, self.relevant = plan, None

    def begin_step(self, relevant):
        self.relevant = relevant.clone()
        return self.plan


def worker_step(rank, world, port, compact_below, bucket_bytes, q, transport="fp32"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        visible, grads, norm, _ = rank_inputs(rank, 0)
        arena = GradArena(N)
        params = {k: torch.nn.Parameter(torch.zeros(N, w)) for k, w in LEAF_WIDTHS.items()}
        arena.attach(params)
        for k, v in grads.items():
            arena[k].copy_(v)
        plan = RecordingPlan(arena, {id(p): k for k, p in params.items()})
        opt = RecordingOptimizer(plan)
        ex = ViewDPExchange(bucket_bytes=bucket_bytes, compact_below=compact_below, transport=transport)
        res = ex.exchange_and_step(arena, visible, opt, params, max_stats=[norm])
        all_in = [rank_inputs(r, 0) for r in range(world)]
        if transport == "bf16" and world > 1:
            exp = {k: bf16_sum([a[1][k] for a in all_in]) for k in LEAF_WIDTHS}
        else:
            exp = {k: sum(a[1][k] for a in all_in) for k in LEAF_WIDTHS}
        exp_union = torch.zeros(N, dtype=torch.bool)
        for a in all_in:
            exp_union |= a[0]
        ok = torch.equal(res.union, exp_union) and torch.equal(opt.relevant, exp_union)
        ok = ok and all(torch.allclose(arena[k], exp[k], atol=1e-5) for k in LEAF_WIDTHS)
        if plan.calls == [("all", 0, 0)]:
            mode = "whole"
        else:
            mode = "rows"
            # every row of every field stepped exactly once, in order, after its bucket was reduced
            for k in LEAF_WIDTHS:
                spans = [(r0, r1) for (name, r0, r1) in plan.calls if name == k]
                ok = ok and spans[0][0] == 0 and spans[-1][1] == N
                ok = ok and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            ok = ok and [c[0] for c in plan.calls] == sorted((c[0] for c in plan.calls),
                                                             key=list(LEAF_WIDTHS).index)
            for (name, r0, r1), got in plan.snap.items():
                ok = ok and torch.allclose(got, exp[name][r0:r1], atol=1e-5)
            # the plan's other parameters are stepped whole, the arena fields are skipped there
            ok = ok and getattr(plan, "rest_skipped", None) == set(LEAF_WIDTHS)
        if rank == 0:
            q.put((ok, mode, ex.last.collectives))
    finally:
        dist.destroy_process_group()


def run_step(world, compact_below, bucket_bytes, transport="fp32"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker_step, args=(r, world, port, compact_below, bucket_bytes, q, transport))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return q.get(timeout=10)


@pytest.mark.parametrize("world,compact_below,bucket_bytes,mode,transport", [
    (2, 0.0, 4096, "rows", "fp32"),       # dense: per-bucket steps overlapped with the later buckets' reduces
    (3, 0.0, 1 << 20, "rows", "fp32"),
    (2, 1.0, 4096, "whole", "fp32"),      # compacted: reduce, then one step
    (1, 0.0, 4096, "whole", "fp32"),      # one rank: no collective at all
    (2, 0.0, 4096, "rows", "bf16"),       # bf16 wire: all-to-all + all-gather per bucket, pipelined
    (3, 0.0, 1 << 20, "rows", "bf16"),
    (3, 1.0, 4096, "whole", "bf16"),
    (8, 0.0, 4096, "rows", "fp32"),       # world 8: per-bucket overlap at the driver's scaling width
    (8, 0.0, 4096, "rows", "bf16"),
])
def test_exchange_and_step_steps_each_row_once_after_its_reduction(world, compact_below, bucket_bytes, mode, transport):
    ok, got_mode, collectives = run_step(world, compact_below, bucket_bytes, transport)
    assert ok and got_mode == mode
    if world == 1:
        assert collectives == 0


def bf16_sum(parts):
    """The bf16 transport's definition: every rank's values rounded to bf16 (nearest even), added in
    fp32 in rank order, the sum rounded to bf16 once (returned as fp32)."""
    acc = parts[0].to(torch.bfloat16).to(torch.float32)
    for x in parts[1:]:
        acc = acc + x.to(torch.bfloat16).to(torch.float32)
    return acc.to(torch.bfloat16).to(torch.float32)


def worker_bf16(rank, world, port, compact_below, bucket_bytes, q, pattern="rate"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = ViewDPExchange(bucket_bytes=bucket_bytes, compact_below=compact_below, transport="bf16")
        ok, rel = True, 0.0
        for step in range(2):
            visible, grads, norm, _ = rank_inputs(rank, step, pattern=pattern)
            arena = GradArena(N)
            for k, v in grads.items():
                arena[k].copy_(v)
            ex.exchange(arena, visible, max_stats=[norm])
            all_in = [rank_inputs(r, step, pattern=pattern) for r in range(world)]
            for k in LEAF_WIDTHS:
                parts = [a[1][k] for a in all_in]
                ok = ok and torch.equal(arena[k], bf16_sum(parts))  # the definition, bit for bit
                exact = sum(p.double() for p in parts)
                scale = sum(p.double().abs() for p in parts)
                rel = max(rel, float(((arena[k].double() - exact).abs() / scale.clamp(min=1e-30)).max()))
            # replicas identical: every rank's summed arena, bit for bit
            got = [torch.empty_like(arena.flat) for _ in range(world)]
            dist.all_gather(got, arena.flat)
            ok = ok and all(torch.equal(g.view(torch.int32), got[0].view(torch.int32)) for g in got)
        if rank == 0:
            q.put((ok, rel, ex.last.wire_bytes, ex.last.reduced_bytes, ex.last.compacted))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,compact_below,bucket_bytes,pattern", [
    (2, 0.0, 64 << 20, "rate"), (3, 0.0, 4096, "rate"), (3, 1.0, 1000, "rate"), (4, 0.0, 10000, "rate"),
    (8, 0.75, 4096, "window"),  # world 8, divergent views: compacted, [world][chunk] wire layout at 8 ranks
    (8, 0.0, 10000, "window")])
def test_bf16_transport_is_its_definition_and_identical_on_every_rank(world, compact_below, bucket_bytes, pattern):
    """transport="bf16": half the wire bytes, the sum formed in fp32 by the chunk's owner; the result
    equals bf16(sum_r bf16(g_r)) exactly and is the same on every rank; within 2^-7 of the exact sum
    relative to sum_r |g_r| (two bf16 roundings of relative 2^-9 each, plus fp32 adds)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker_bf16, args=(r, world, port, compact_below, bucket_bytes, q, pattern))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    ok, rel, wire, reduced, compacted = q.get(timeout=10)
    assert ok, "bf16 exchange differs from its definition or between ranks"
    assert rel <= 2.0 ** -7, rel
    assert wire * 2 == reduced and compacted == (compact_below > 0.0)


EX_TIMEOUT, PG_TIMEOUT = 1.5, 5.0


def worker_fail(rank, world, port, scenario, q):
    """The last rank stops taking part at some point of the exchange (stall: sleeps; crash: exits 3); every
    other rank must raise RuntimeError naming the collective it waited on, within the exchange's timeout."""
    import datetime
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=PG_TIMEOUT))
    try:
        transport = "bf16" if scenario == "stall_bf16" else "fp32"
        ex = ViewDPExchange(bucket_bytes=4096, compact_below=0.0, transport=transport, timeout=EX_TIMEOUT)
        visible, grads, norm, _ = rank_inputs(rank, 0)
        arena = GradArena(N)
        for k, v in grads.items():
            arena[k].copy_(v)
        if rank == world - 1:
            if scenario != "stall_visibility":
                union, _ = ex.gather_visibility(visible)
            if scenario == "stall_max":
                ex.sum_gradients(arena, union)
            if scenario == "crash_buckets":
                os._exit(3)
            time.sleep(600)  # stalled: the launcher (here the test) ends it once the others have failed
            return
        t0 = time.perf_counter()
        try:
            ex.exchange(arena, visible, max_stats=[norm])
        except RuntimeError as e:
            q.put((rank, str(e), time.perf_counter() - t0))
            raise
        q.put((rank, "no error", time.perf_counter() - t0))
    finally:
        if rank != world - 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world,scenario,what", [
    (2, "stall_visibility", "visibility all-gather"),
    (2, "stall_buckets", "gradient bucket 1 of "),
    (2, "stall_bf16", "bf16 all-to-all"),
    (2, "stall_max", "MAX all-reduce"),
    (2, "crash_buckets", "gradient bucket 1 of "),
    (8, "stall_buckets", "gradient bucket "),  # the driver's scaling width: seven ranks wait on the eighth
])
def test_a_rank_that_stops_participating_fails_the_others_fast(world, scenario, what):
    """SURVEY §5 "DP: fail fast" (VERDICT r05 item 2): gloo, the last rank stalls or dies mid-exchange.
    Every other rank raises RuntimeError naming the collective within the exchange timeout plus a small
    margin, and every child exits non-zero instead of hanging (the waiting ranks after at most the process
    group's timeout; the stalled rank is ended by its launcher, as torch.distributed.run ends the others
    when one fails)."""
    import time
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker_fail, args=(r, world, port, scenario, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=60) for _ in range(world - 1)]
        t_err = time.perf_counter()
        for p in procs[:-1]:
            p.join(PG_TIMEOUT + 30)
        exit_after = time.perf_counter() - t_err
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
            p.join(10)
    assert sorted(r for r, _, _ in got) == list(range(world - 1))
    for rank, msg, elapsed in got:
        print(f"{scenario} world {world} rank {rank}: raised after {elapsed:.2f} s: {msg[:160]}")
        assert what in msg and "did not complete" in msg and f"rank {rank} of {world}" in msg, msg
        if scenario.startswith("stall"):
            assert f"waited at most {EX_TIMEOUT:g} s" in msg and "timed out" in msg, msg
        assert elapsed < EX_TIMEOUT + 3.0, f"rank {rank} raised after {elapsed:.1f} s"
    print(f"{scenario} world {world}: the waiting ranks exited {exit_after:.1f} s after the errors")
    assert all(p.exitcode not in (0, None) for p in procs), [p.exitcode for p in procs]
    assert exit_after < PG_TIMEOUT + 15, f"the waiting ranks took {exit_after:.1f} s to exit after the error"


def test_timeout_is_checked():
    with pytest.raises(ValueError, match="timeout"):
        ViewDPExchange(timeout=0)
    assert ViewDPExchange(timeout=None).timeout is None


def test_transport_is_checked():
    with pytest.raises(ValueError, match="transport"):
        ViewDPExchange(transport="fp16")


def test_detached_grad_is_refused():
    """zero_grad(set_to_none=True) or a reassigned .grad breaks the parameter/arena link: the
    exchange must raise instead of summing stale arena rows."""
    arena = GradArena(8)
    params = {k: torch.nn.Parameter(torch.zeros(8, w)) for k, w in LEAF_WIDTHS.items()}
    arena.attach(params)
    arena.check_attached(params)
    opt = torch.optim.SGD(list(params.values()), lr=0.1)
    opt.zero_grad(set_to_none=True)
    with pytest.raises(RuntimeError, match="not the gradient arena's view"):
        arena.check_attached(params)
    arena.attach(params)
    params["xyz"].grad = torch.zeros(8, 3)
    with pytest.raises(RuntimeError, match="xyz.grad"):
        ViewDPExchange().exchange(arena, torch.ones(8, dtype=torch.bool), params=params)
