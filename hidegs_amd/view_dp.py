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

`exchange_and_step` fuses the exchange with the masked optimizer step that follows it: each
dense bucket's rows are updated as soon as that bucket's all-reduce lands, while the later
buckets are still reducing (SURVEY §8(e) E2's overlap; the backward that would also overlap it is
not built here).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Union

import torch
import torch.distributed as dist

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
    union_rows: int = 0
    reduced_bytes: int = 0
    collectives: int = 0
    compacted: bool = False


@dataclass
class ExchangeResult:
    union: torch.Tensor       # bool (N,): visible in some rank's view (the masked Adam's rows)
    view_count: torch.Tensor  # float32 (N, 1): how many ranks' views saw each Gaussian (denom increment)


class ViewDPExchange:
    """One exchange step per training iteration of view-data-parallel rendering."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None, bucket_bytes: int = 64 << 20,
                 compact_below: float = 0.75, debug: bool = False):
        if bucket_bytes < 4:
            raise ValueError("bucket_bytes must hold at least one fp32 value")
        if not 0.0 <= compact_below <= 1.0:
            raise ValueError("compact_below is a fraction of rows in [0, 1]")
        self.group = group
        self.bucket_bytes = int(bucket_bytes)
        self.compact_below = float(compact_below)
        self.debug = debug
        self.last = ExchangeStats()

    # ---- visibility -------------------------------------------------------------
    def gather_visibility(self, visible: torch.Tensor):
        """(union bool (N,), view_count float32 (N,1)) over every rank's mask; one all-gather."""
        if visible.dtype != torch.bool or visible.dim() != 1:
            raise ValueError("visible must be a 1-D bool mask")
        world = dist.get_world_size(self.group)
        if world == 1:  # one view: nothing to exchange
            return visible.clone(), visible.to(torch.float32).unsqueeze(1)
        bits = pack_mask(visible)
        flat = bits.new_empty((world * bits.numel(),))
        dist.all_gather_into_tensor(flat, bits, group=self.group)
        self.last.collectives += 1
        per_rank = unpack_mask(flat.view(world, bits.numel()), visible.numel())
        count = per_rank.sum(0, dtype=torch.int32)
        return count > 0, count.to(torch.float32).unsqueeze(1)

    # ---- leaf gradients -----------------------------------------------------------
    def _all_reduce_buckets(self, flat: torch.Tensor) -> None:
        if dist.get_world_size(self.group) == 1:  # the sum over one rank is the tensor itself
            return
        per = max(1, self.bucket_bytes // flat.element_size())
        works = [dist.all_reduce(flat[s:s + per], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                 for s in range(0, flat.numel(), per)]
        for w in works:
            w.wait()
        self.last.collectives += len(works)
        self.last.reduced_bytes += flat.numel() * flat.element_size()

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
        rows = None
        if union is not None and n:
            nu = int(union.sum())
            self.last.union_rows = nu
            if nu < self.compact_below * n:
                rows = union.nonzero().flatten()
            if self.debug:
                outside = ~union
                for g in tensors:
                    if bool(g.reshape(n, -1)[outside].ne(0).any()):
                        raise RuntimeError("view-DP: a gradient row outside the visibility union is non-zero; "
                                           "the compacted exchange would desynchronise the replicas")
        else:
            self.last.union_rows = n
        if dist.get_world_size(self.group) == 1:  # one rank: the sum is the input, in place already
            return
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
        self._all_reduce_buckets(packed)
        off = 0
        for g, w in zip(tensors, widths):
            g.reshape(n, w).index_copy_(0, rows, packed[off:off + rows.numel() * w].view(-1, w))
            off += rows.numel() * w

    # ---- statistics ---------------------------------------------------------------
    def max_stats(self, stats: List[torch.Tensor]) -> None:
        """In-place MAX over ranks of per-step maxima, all in ONE collective."""
        stats = [s for s in stats if s is not None]
        if not stats or dist.get_world_size(self.group) == 1:
            return
        flat = torch.cat([s.reshape(-1).to(torch.float32) for s in stats])
        dist.all_reduce(flat, op=dist.ReduceOp.MAX, group=self.group)
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
        world = dist.get_world_size(self.group)
        nu = int(union.sum()) if n else 0
        if world == 1 or n == 0 or nu < self.compact_below * n:
            self.sum_gradients(arena, union)
            optimizer.begin_step(union).run()  # counters advance only once the gradients are summed
        else:
            self.last.union_rows = nu
            works = []
            for name, w in arena.widths.items():
                rows = max(4, (self.bucket_bytes // (4 * w)) // 4 * 4)  # 4-row multiples keep 16-byte alignment
                view = arena.views[name]
                for r0 in range(0, n, rows):
                    r1 = min(n, r0 + rows)
                    works.append((dist.all_reduce(view[r0:r1], op=dist.ReduceOp.SUM, group=self.group,
                                                  async_op=True), name, r0, r1))
            self.last.collectives += len(works)
            self.last.reduced_bytes += arena.flat.numel() * arena.flat.element_size()
            # the step counters advance once every collective has been issued
            plan = optimizer.begin_step(union)
            for work, name, r0, r1 in works:
                work.wait()  # the current stream waits for this bucket; later buckets keep reducing
                plan.run_rows(params[name], r0, r1)
            # parameters the plan steps that are not arena fields (their gradients were not exchanged
            # here): stepped whole, as optimizer.step(union) would
            plan.run_except([params[k] for k in arena.widths])
        self.max_stats(max_stats or [])
        return ExchangeResult(union, count)
