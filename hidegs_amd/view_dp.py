"""View-data-parallel exchange for multi-GPU HiDeGS training.

The reference is single-process; this is a new capability.  Every rank
holds a full replica of the Gaussian parameters and renders its own camera view
(`view_index(step, rank, world)`); after the backward pass one exchange step makes the
replicas agree again, with the result the reference would reach by processing the
world's views one after another:

    leaf gradients (xyz, f_dc, f_rest, opacity, scaling, rotation)   SUM
    per-step densification maxima (|dL/dmeans2D| norm, radii)        MAX, one collective
    per-Gaussian count of views that saw it (the denom increment)    from the masks
    visibility                                                       OR

`add_densification_stats` keeps a running max of the view-space gradient norm and
counts views in `denom` (scene/gaussian_model.py:763-765).  Both accumulators are
replicated, so only this step's contributions are exchanged: the MAX of the per-step
norms and the number of ranks whose view saw each Gaussian.  Summing the accumulators
themselves would count the replicated history `world` times per step.

Leaf gradients live in one flat fp32 arena (`GradArena`), field-major, so each
parameter's `.grad` is a contiguous view that autograd accumulates into in place and the
dense exchange is an in-place all-reduce of the arena with no copies.  When few rows are
visible anywhere (union fraction below `compact_below`) only those rows are packed and
reduced; rows outside the union are zero on every rank (the rasterizer's backward writes
zero rows for Gaussians it did not render), so the packed sum equals the dense one.
Buckets of `bucket_bytes` (default 64 MiB) are all issued before any is waited on: a ring
over xGMI is bound per link (~153 GB/s) and pays a fixed cost per collective.

Backend: whatever process group is current -- "nccl" (RCCL on ROCm) on the GPU, "gloo" in
the CPU tests.  Bitwise OR is formed from an all-gather of packed masks (RCCL has no
bitwise reduction), which also yields the per-Gaussian view count.  A one-rank group has
nothing to exchange and issues no collective.

Transport (`transport=`): "fp32" (default) all-reduces the fp32 gradients as they are.  "bf16" halves
the bytes on the wire with the sum still formed in fp32: each bucket is rounded to bf16 (nearest-even)
and split into `world` chunks; one all-to-all hands chunk c of every rank to rank c, which adds them in
fp32 in rank order (0, 1, ...) and rounds the sum to bf16 once; one all-gather returns every chunk's
sum to every rank.  The result is each element's bf16(sum_r bf16(g_r)) -- within ~2^-8 relative of the
fp32 sum per input plus one output rounding, identical on every rank (each chunk is summed by exactly
one rank, in a fixed order), so the replicas stay bit-identical.  It is a semantic change (SURVEY §8(e)
E2 item 3: "bf16 transport, behind a parity flag"); the default stays fp32, and stays so until an N > 1
measurement shows the halved xGMI bytes save more than the wire's local cost (pack, sum, unpack and
twice the collectives: +0.73 ms per 472 MB step on the forced one-rank RCCL path, BENCH_r04).
Memory: a bf16 bucket in flight holds a send, a receive and a gathered buffer of 2 B per element each
(and its rank's chunk sum); at most `BF16_IN_FLIGHT` buckets are started ahead of the one being
finished, so the extra memory is bounded by (BF16_IN_FLIGHT + 1) x 6 B x bucket elements (~480 MB at
the default 64 MiB buckets) whatever the arena's size, instead of ~6 B per arena element.

`exchange_and_step` fuses the exchange with the masked optimizer step that follows it: each
dense bucket's rows are updated as soon as that bucket's all-reduce lands, while the later
buckets are still reducing (SURVEY §8(e) E2's overlap; the backward that would also overlap it is
not built here).

Failure detection ("DP: fail fast on RCCL error").  Every collective is issued
asynchronously and waited on through one helper, so no wait is unbounded and a rank that stops
participating (stalled, crashed) turns into a RuntimeError naming the collective -- visibility
all-gather, bucket i of k (fp32 all-reduce, bf16 all-to-all or all-gather) or the MAX all-reduce --
on the ranks still waiting:
* host tensors (gloo): each wait is bounded by `timeout` (seconds, default 300) and raises when it
  expires.  The process group's own timeout (`init_process_group(timeout=...)`) still bounds the
  abandoned operation, so a process exiting after the error takes up to that long to tear down.
* device tensors (RCCL): a wait only makes the compute stream wait on the collective's stream --
  the host never blocks, which is what lets the bucket pipeline overlap.  A collective that never
  completes is caught by the process group's watchdog after the process group's timeout, which ends
  the process (TORCH_NCCL_ASYNC_ERROR_HANDLING, on by default in torch 2.10): pass an
  explicit `timeout` to init_process_group (bench.py does).  `blocking=True` bounds the host wait by
  `timeout` on device tensors too and raises the same RuntimeError, at the price of a host wait per
  collective (the bucket overlap then depends on the host keeping ahead).
"""
from __future__ import annotations

import datetime
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Union

import torch
import torch.distributed as dist

from . import wire

LEAF_WIDTHS = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
"""Per-Gaussian fp32 widths of the HiDeGS leaf parameters (59 floats = 236 B; SURVEY §8(e) E1)."""

_BITS = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8)


def view_index(step: int, rank: int, world_size: int) -> int:
    """Camera view rendered by `rank` at `step` (E1: rank r renders view world*step + r)."""
    return world_size * step + rank


def pack_mask(mask: torch.Tensor) -> torch.Tensor:
    """bool (N,) -> uint8 (ceil(N/8),), bit i of byte j = mask[8j + i]."""
    n = mask.numel()
    pad = (-n) % 8
    m = mask.reshape(-1).to(torch.uint8)
    if pad:
        m = torch.cat([m, m.new_zeros(pad)])
    return (m.view(-1, 8) * _BITS.to(m.device)).sum(dim=1, dtype=torch.uint8)


def unpack_mask(bits: torch.Tensor, n: int) -> torch.Tensor:
    """Inverse of pack_mask (also accepts a (R, B) stack, giving (R, n))."""
    b = bits.unsqueeze(-1) & _BITS.to(bits.device)
    return (b != 0).reshape(*bits.shape[:-1], -1)[..., :n]


class GradArena:
    """One flat fp32 buffer holding every leaf gradient, field-major ([field][row][col]).

    `views[name]` is a contiguous (n, width) view; `attach` makes it the `.grad` of a
    parameter (autograd then accumulates into it in place, shape-matched via view_as).

    The link is the parameter's `.grad` object itself: `optimizer.zero_grad(set_to_none=True)`
    (the 3DGS default), re-creating the parameters (densification) or assigning `.grad` detaches
    it, and autograd then writes a fresh tensor the arena never sees.  Call `zero_()` instead of
    zero_grad, and `attach` again after the parameters change; the exchange checks the link
    (`check_attached`) and raises when it is broken.
    """

    def __init__(self, n: int, widths: Dict[str, int] = None, device=None, dtype=torch.float32):
        self.n = int(n)
        self.widths = dict(widths or LEAF_WIDTHS)
        self.row_width = sum(self.widths.values())
        self.flat = torch.zeros(self.n * self.row_width, dtype=dtype, device=device)
        self.views: Dict[str, torch.Tensor] = {}
        off = 0
        for name, w in self.widths.items():
            self.views[name] = self.flat[off:off + self.n * w].view(self.n, w)
            off += self.n * w

    def attach(self, params: Dict[str, torch.Tensor]) -> None:
        for name, p in params.items():
            v = self.views[name]
            if p.numel() != v.numel():
                raise ValueError(f"{name}: parameter has {p.numel()} values, arena slot {v.numel()}")
            p.grad = v.view_as(p)

    def check_attached(self, params: Dict[str, torch.Tensor]) -> None:
        """Raise if some params[name].grad is not this arena's view (the gradient would be summed
        from stale arena rows while the optimizer stepped the local one: replicas drift apart)."""
        for name, p in params.items():
            if name not in self.views:
                continue
            g = p.grad
            v = self.views[name]
            if g is None or g.data_ptr() != v.data_ptr() or g.numel() != v.numel():
                raise RuntimeError(f"view-DP: {name}.grad is not the gradient arena's view (zero_grad(set_to_none="
                                   "True), re-created parameters or a reassigned .grad detach it); call "
                                   "arena.attach(params) again and clear gradients with arena.zero_()")

    def zero_(self) -> None:
        self.flat.zero_()

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.views[name]


@dataclass
class ExchangeStats:
    union_rows: int = 0     # rows visible to some rank (-1: not counted, a one-rank group)
    reduced_bytes: int = 0  # fp32 gradient bytes summed over ranks (per rank)
    wire_bytes: int = 0     # bytes this rank handed to the collectives for them (bf16: half)
    collectives: int = 0
    compacted: bool = False


TRANSPORTS = ("fp32", "bf16")
BF16_IN_FLIGHT = 4  # bf16 buckets started ahead of the one being finished (bounds the wire buffers' memory)


class _Bucket:
    """One gradient bucket's SUM over the group, in three steps so that several buckets can be in
    flight: start() issues the first collective, mid() the second (bf16 only: the fp32 sum of this
    rank's chunk between the two), finish() waits and leaves the summed values in `view` (fp32)."""

    def __init__(self, view: torch.Tensor, group, transport: str, world: int, rank: int, wait=None,
                 label: str = "bucket"):
        self.view, self.group, self.transport, self.world, self.rank = view, group, transport, world, rank
        self.work = None
        self.label = label
        self._wait = wait or (lambda work, what: work.wait())

    def start(self) -> int:
        if self.transport == "fp32":
            self.work = dist.all_reduce(self.view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            return 1
        n, w = self.view.numel(), self.world
        self.chunk = -(-n // (8 * w)) * 8  # 16-byte aligned chunks, one per rank
        flat = self.view.reshape(-1)
        if flat.is_cuda:  # one pass: round to nearest even, zero padding (csrc/wire.hip)
            send = wire.bf16_pack(flat, torch.empty(self.chunk * w, dtype=torch.bfloat16, device=flat.device))
        else:  # gloo ranks on the CPU: the definition as torch ops
            send = torch.zeros(self.chunk * w, dtype=torch.bfloat16)
            send[:n].copy_(flat)  # round to nearest even
        self.recv = torch.empty_like(send)
        # bf16 moved as bytes: the collective only moves them (gloo has no 16-bit all-to-all)
        self.work = dist.all_to_all_single(self.recv.view(torch.uint8), send.view(torch.uint8), group=self.group,
                                           async_op=True)
        self.send = send
        return 1

    def mid(self) -> int:
        if self.transport == "fp32":
            return 0
        self._wait(self.work, f"{self.label}: bf16 all-to-all")
        parts = self.recv.view(self.world, self.chunk)
        if parts.is_cuda:  # one pass over the w rows (csrc/wire.hip), the same bits as below
            mine = wire.bf16_sum_ranks(parts)
        else:
            acc = parts[0].to(torch.float32)
            for r in range(1, self.world):  # fp32, rank order: the same sum on whichever rank owns the chunk
                acc += parts[r].to(torch.float32)
            mine = acc.to(torch.bfloat16)
        self.gathered = torch.empty_like(self.send)
        self.send = self.recv = None  # the all-to-all is complete and `mine` is formed: free them now
        self.work = dist.all_gather_into_tensor(self.gathered.view(torch.uint8), mine.view(torch.uint8),
                                                group=self.group, async_op=True)
        self.mine = mine  # kept alive until the all-gather is waited on
        return 1

    def finish(self) -> None:
        self._wait(self.work, f"{self.label}: " + ("fp32 SUM all-reduce" if self.transport == "fp32"
                                                   else "bf16 all-gather"))
        if self.transport == "bf16":
            flat = self.view.reshape(-1)  # a view: the bucket is a contiguous slice
            if flat.is_cuda:
                wire.bf16_unpack(self.gathered, flat)
            else:
                flat.copy_(self.gathered[:self.view.numel()])
            self.gathered = self.mine = None

    @property
    def wire_bytes(self) -> int:
        return self.view.numel() * (4 if self.transport == "fp32" else 2)


@dataclass
class ExchangeResult:
    union: torch.Tensor       # bool (N,): visible in some rank's view (the masked Adam's rows)
    view_count: torch.Tensor  # float32 (N, 1): how many ranks' views saw each Gaussian (denom increment)


class ViewDPExchange:
    """One exchange step per training iteration of view-data-parallel rendering."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None, bucket_bytes: int = 64 << 20,
                 compact_below: float = 0.75, debug: bool = False, transport: str = "fp32",
                 force_collectives: bool = False, timeout: Optional[float] = 300.0, blocking: bool = False):
        if bucket_bytes < 4:
            raise ValueError("bucket_bytes must hold at least one fp32 value")
        if not 0.0 <= compact_below <= 1.0:
            raise ValueError("compact_below is a fraction of rows in [0, 1]")
        if transport not in TRANSPORTS:
            raise ValueError(f"transport must be one of {TRANSPORTS}")
        if timeout is not None and not timeout > 0:
            raise ValueError("timeout is a positive number of seconds (or None: the process group's own)")
        self.timeout = None if timeout is None else float(timeout)
        self.blocking = bool(blocking)
        self.transport = transport
        self.group = group
        self.bucket_bytes = int(bucket_bytes)
        self.compact_below = float(compact_below)
        self.debug = debug
        # tests and hardware checks: a one-rank group takes the N-rank path (its collectives are real
        # RCCL calls, so the 1-GPU box exercises every one the 8-GPU bench issues)
        self.force_collectives = bool(force_collectives)
        self.last = ExchangeStats()

    def _solo(self) -> bool:
        """One rank and nothing forced: every sum is its input, no collective is issued."""
        return dist.get_world_size(self.group) == 1 and not self.force_collectives

    def _wait(self, work, what: str, cuda: bool) -> None:
        """Wait for one collective: bounded on the host (gloo, or blocking=True) or a stream wait (RCCL,
        bounded by the process group's watchdog); a timeout or a failed peer raises RuntimeError naming it."""
        bounded = self.timeout is not None and (not cuda or self.blocking)
        try:
            done = work.wait(datetime.timedelta(seconds=self.timeout)) if bounded else work.wait()
        except Exception as e:  # noqa: BLE001 -- re-raised with the collective named
            raise RuntimeError(self._failure(what, bounded, e)) from e
        if done is False:
            raise RuntimeError(self._failure(what, bounded, None))

    def _failure(self, what: str, bounded: bool, err) -> str:
        rank, world = dist.get_rank(self.group), dist.get_world_size(self.group)
        limit = f" (waited at most {self.timeout:g} s)" if bounded else ""
        cause = f": {type(err).__name__}: {err}" if err is not None else ""
        return (f"view-DP exchange: {what} did not complete on rank {rank} of {world}{limit}{cause}; another rank "
                "stopped participating or failed -- the replicas can no longer agree, end this process")

    # ---- visibility -------------------------------------------------------------
    def gather_visibility(self, visible: torch.Tensor):
        """(union bool (N,), view_count float32 (N,1)) over every rank's mask; one all-gather."""
        if visible.dtype != torch.bool or visible.dim() != 1:
            raise ValueError("visible must be a 1-D bool mask")
        world = dist.get_world_size(self.group)
        if self._solo():  # one view: nothing to exchange
            return visible.clone(), visible.to(torch.float32).unsqueeze(1)
        cuda = visible.is_cuda
        bits = wire.mask_pack(visible.contiguous()) if cuda else pack_mask(visible)
        flat = bits.new_empty((world * bits.numel(),))
        self._wait(dist.all_gather_into_tensor(flat, bits, group=self.group, async_op=True),
                   "visibility all-gather", cuda)
        self.last.collectives += 1
        if cuda:  # one pass (csrc/wire.hip), the same result as the torch definition below
            return wire.mask_union_count(flat.view(world, bits.numel()), visible.numel())
        per_rank = unpack_mask(flat.view(world, bits.numel()), visible.numel())
        count = per_rank.sum(0, dtype=torch.int32)
        return count > 0, count.to(torch.float32).unsqueeze(1)

    # ---- leaf gradients -----------------------------------------------------------
    def _bucket(self, view: torch.Tensor, label: str = "bucket") -> _Bucket:
        cuda = view.is_cuda
        return _Bucket(view, self.group, self.transport, dist.get_world_size(self.group), dist.get_rank(self.group),
                       wait=lambda work, what: self._wait(work, what, cuda), label=label)

    @staticmethod
    def _label_buckets(buckets: List[_Bucket], what: str) -> List[_Bucket]:
        for i, b in enumerate(buckets):
            nb = b.view.numel() * 4
            size = f"{nb / 2**20:.1f} MiB" if nb >= 1 << 20 else f"{nb / 2**10:.1f} KiB"
            b.label = f"{what} bucket {i + 1} of {len(buckets)} ({size} fp32)"
        return buckets

    def _run_buckets(self, buckets: List[_Bucket], after=None) -> None:
        """fp32: every bucket's all-reduce issued at once (in place: no extra memory).  bf16: the first
        collective of up to BF16_IN_FLIGHT buckets ahead of the one being finished.  Then per bucket in
        order: its second collective (bf16) issued one bucket ahead, its wait, and `after(i)` (e.g. that
        bucket's rows' optimizer update) while the later buckets are still on the wire."""
        ahead = len(buckets) if self.transport == "fp32" else max(2, BF16_IN_FLIGHT)
        started = 0

        def start_until(k):
            nonlocal started
            while started < min(k, len(buckets)):
                b = buckets[started]
                self.last.collectives += b.start()
                self.last.wire_bytes += b.wire_bytes
                self.last.reduced_bytes += b.view.numel() * 4
                started += 1

        start_until(ahead)
        if buckets:
            self.last.collectives += buckets[0].mid()
        for i, b in enumerate(buckets):
            start_until(i + 1 + ahead)
            if i + 1 < len(buckets):
                self.last.collectives += buckets[i + 1].mid()
            b.finish()
            if after is not None:
                after(i)

    def _all_reduce_buckets(self, flat: torch.Tensor, what: str = "gradient") -> None:
        if self._solo():  # the sum over one rank is the tensor itself
            return
        per = max(1, self.bucket_bytes // flat.element_size())
        self._run_buckets(self._label_buckets([self._bucket(flat[s:s + per]) for s in range(0, flat.numel(), per)],
                                              what))

    def sum_gradients(self, grads: Union[GradArena, Iterable[torch.Tensor]],
                      union: Optional[torch.Tensor] = None) -> None:
        """In-place SUM over ranks of per-Gaussian gradients (each (N, ...), same N).

        `union` (bool (N,), identical on every rank, rows visible to some rank) allows the
        compacted exchange; every row outside it must be zero on every rank.
        """
        if isinstance(grads, GradArena):
            tensors, n = list(grads.views.values()), grads.n
            arena = grads.flat
        else:
            tensors = [g for g in grads if g is not None]
            if not tensors:
                return
            n, arena = tensors[0].size(0), None
        for g in tensors:
            if g.size(0) != n:
                raise ValueError("all gradients must have the same number of rows")
            if g.dtype != torch.float32:
                raise ValueError("gradients are exchanged in fp32")
            if not g.is_contiguous():
                raise ValueError("gradients must be contiguous (results are written back in place)")
        if union is not None:
            if union.dtype != torch.bool or union.dim() != 1 or union.numel() != n:
                raise ValueError(f"union must be a bool mask of the {n} gradient rows "
                                 "(fullP rows: scatter hierarchy render_indices/parent_indices into it)")
        if self.debug and union is not None and n:
            outside = ~union
            for g in tensors:
                if bool(g.reshape(n, -1)[outside].ne(0).any()):
                    raise RuntimeError("view-DP: a gradient row outside the visibility union is non-zero; "
                                       "the compacted exchange would desynchronise the replicas")
        if self._solo():  # one rank: the sum is the input, in place already
            self.last.union_rows = -1  # not counted: no host synchronisation on the one-rank path
            return
        rows = None
        if union is not None and n:
            nu = int(union.sum())
            self.last.union_rows = nu
            if nu < self.compact_below * n:
                rows = union.nonzero().flatten()
        else:
            self.last.union_rows = n
        if rows is None:
            self.last.compacted = False
            if arena is not None:
                self._all_reduce_buckets(arena)
            else:
                flat = torch.cat([g.reshape(-1) for g in tensors])
                self._all_reduce_buckets(flat)
                off = 0
                for g in tensors:
                    g.view(-1).copy_(flat[off:off + g.numel()])
                    off += g.numel()
            return
        self.last.compacted = True
        if rows.numel() == 0:
            return
        widths = [g[0].numel() for g in tensors]
        packed = torch.empty(rows.numel() * sum(widths), dtype=torch.float32, device=tensors[0].device)
        off = 0
        for g, w in zip(tensors, widths):
            torch.index_select(g.reshape(n, w), 0, rows, out=packed[off:off + rows.numel() * w].view(-1, w))
            off += rows.numel() * w
        self._all_reduce_buckets(packed, "compacted gradient")
        off = 0
        for g, w in zip(tensors, widths):
            g.reshape(n, w).index_copy_(0, rows, packed[off:off + rows.numel() * w].view(-1, w))
            off += rows.numel() * w

    # ---- statistics ---------------------------------------------------------------
    def max_stats(self, stats: List[torch.Tensor]) -> None:
        """In-place MAX over ranks of per-step maxima, all in ONE collective."""
        stats = [s for s in stats if s is not None]
        if not stats or self._solo():
            return
        flat = torch.cat([s.reshape(-1).to(torch.float32) for s in stats])
        self._wait(dist.all_reduce(flat, op=dist.ReduceOp.MAX, group=self.group, async_op=True),
                   "MAX all-reduce of the per-step maxima", flat.is_cuda)
        self.last.collectives += 1
        off = 0
        for s in stats:
            s.view(-1).copy_(flat[off:off + s.numel()].to(s.dtype))
            off += s.numel()

    # ---- the whole exchange step ----------------------------------------------------
    def exchange(self, grads: Union[GradArena, Dict[str, torch.Tensor]], visible: torch.Tensor,
                 max_stats: Optional[List[torch.Tensor]] = None,
                 params: Optional[Dict[str, torch.Tensor]] = None) -> ExchangeResult:
        """Run one exchange step.

        grads      GradArena or {name: (N, w) grad}; summed in place.
        params     with a GradArena: the parameters attached to it; their `.grad` must still be
                   the arena's views (checked: RuntimeError otherwise).
        visible    this rank's visibility filter (radii > 0), bool (N,).
        max_stats  this step's per-Gaussian maxima (e.g. the view-space gradient norm of
                   visible rows, radii), reduced in place by MAX.
        Returns the union mask and the per-Gaussian view count; the caller then applies the
        reference's update to its replicated accumulators:
            xyz_gradient_accum = max(xyz_gradient_accum, norm)   # on union rows
            denom += view_count
        """
        if params is not None and isinstance(grads, GradArena):
            grads.check_attached(params)
        self.last = ExchangeStats()
        union, count = self.gather_visibility(visible)
        g = grads if isinstance(grads, GradArena) else grads.values()
        self.sum_gradients(g, union)
        self.max_stats(max_stats or [])
        return ExchangeResult(union, count)

    def exchange_and_step(self, arena: GradArena, visible: torch.Tensor, optimizer, params: Dict[str, torch.Tensor],
                          max_stats: Optional[List[torch.Tensor]] = None) -> ExchangeResult:
        """`exchange` followed by the masked optimizer step on the union, with the two overlapped.

        optimizer  has `begin_step(relevant) -> plan` with `plan.run()` and `plan.run_rows(p, r0, r1)`
                   (hidegs_amd.optim.Adam); it is stepped with relevant = the union mask.
        params     {field name: parameter} whose `.grad` are the arena's views (GradArena.attach).

        Dense exchange: every bucket is a row range of one field; all buckets' all-reduces are issued
        first, then, bucket by bucket, the compute stream waits for that bucket's reduction and
        updates its rows -- so the update of bucket b runs while buckets b+1... are still on the
        wire, and only the last bucket's update is exposed.  The field order ends with the narrow
        fields, so that last bucket is small.  The compacted exchange (few union rows) and a
        one-rank group step once after the exchange.  The result is bit-identical to `exchange`
        then `optimizer.step(union)`: the update is row-local and every row is updated once.
        """
        if not isinstance(arena, GradArena):
            raise TypeError("exchange_and_step works on a GradArena")
        missing = [k for k in arena.widths if k not in params]
        if missing:
            raise KeyError(f"no parameter for arena fields {missing}")
        arena.check_attached(params)
        self.last = ExchangeStats()
        union, count = self.gather_visibility(visible)
        n = arena.n
        solo = self._solo()
        nu = int(union.sum()) if n and not solo else 0  # (no host synchronisation on one rank)
        if solo or n == 0 or nu < self.compact_below * n:
            self.sum_gradients(arena, union)
            optimizer.begin_step(union).run()  # counters advance only once the gradients are summed
        else:
            self.last.union_rows = nu
            spans, buckets = [], []
            for name, w in arena.widths.items():
                rows = max(4, (self.bucket_bytes // (4 * w)) // 4 * 4)  # 4-row multiples keep 16-byte alignment
                view = arena.views[name]
                for r0 in range(0, n, rows):
                    r1 = min(n, r0 + rows)
                    spans.append((name, r0, r1))
                    buckets.append(self._bucket(view[r0:r1]))
            for (name, r0, r1), b in zip(spans, self._label_buckets(buckets, "gradient")):
                b.label += f" = {name} rows {r0}..{r1}"
            plans = []

            def step_rows(i):
                # the step counters advance once every first collective has been issued
                if not plans:
                    plans.append(optimizer.begin_step(union))
                name, r0, r1 = spans[i]
                plans[0].run_rows(params[name], r0, r1)  # later buckets keep reducing meanwhile

            self._run_buckets(buckets, after=step_rows)
            plan = plans[0] if plans else optimizer.begin_step(union)
            # parameters the plan steps that are not arena fields (their gradients were not exchanged
            # here): stepped whole, as optimizer.step(union) would
            plan.run_except([params[k] for k in arena.widths])
        self.max_stats(max_stats or [])
        return ExchangeResult(union, count)
