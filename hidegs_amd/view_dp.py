"""View-data-parallel gradient exchange for multi-GPU HiDeGS training.

The reference is single-process; this is a new capability.  Every rank
holds a full replica of the Gaussian parameters and renders its own camera view
(`view_index(step, rank, world)`); after the backward pass one exchange step makes
the replicas agree again:

    leaf gradients (xyz, f_dc, f_rest, opacity, scaling, rotation)  SUM
    densification statistics kept as running maxima                 MAX
      (viewspace-gradient norm, scene/gaussian_model.py:763-765; max_radii2D)
    densification counters (denom)                                   SUM
    visibility masks                                                 OR

Compaction: gradients of Gaussians that no rank saw are zero on every rank (the
rasterizer writes zero rows for invisible Gaussians), so only the union-visible rows
are packed and reduced; the result equals the dense all-reduce exactly.  The union is
formed from 1-bit masks gathered from every rank (N/8 bytes each).  Packed rows are
reduced in flat fp32 buckets of `bucket_bytes` (default 64 MiB), all issued
asynchronously, because a ring over xGMI is per-link bound (~153 GB/s) and pays a
fixed cost per collective: few, large collectives.

Backend: whatever process group is current -- "nccl" (RCCL on ROCm) on the GPU,
"gloo" in the CPU tests.  Bitwise OR is done by gathering packed masks (RCCL has no
bitwise reduction).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist

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
    """Inverse of pack_mask."""
    b = bits.reshape(-1, 1) & _BITS.to(bits.device)
    return (b != 0).reshape(-1)[:n]


@dataclass
class ExchangeStats:
    union_rows: int = 0
    reduced_bytes: int = 0
    collectives: int = 0


class ViewDPExchange:
    """One exchange step per training iteration of view-data-parallel rendering."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None, bucket_bytes: int = 64 << 20,
                 compact: bool = True):
        if bucket_bytes < 4:
            raise ValueError("bucket_bytes must hold at least one fp32 value")
        self.group = group
        self.bucket_bytes = int(bucket_bytes)
        self.compact = compact
        self.last = ExchangeStats()

    # ---- visibility -------------------------------------------------------------
    def union_visibility(self, visible: torch.Tensor) -> torch.Tensor:
        """OR of the (N,) bool masks of every rank."""
        world = dist.get_world_size(self.group)
        bits = pack_mask(visible)
        flat = bits.new_empty((world * bits.numel(),))
        dist.all_gather_into_tensor(flat, bits, group=self.group)
        out = flat.view(world, bits.numel())
        self.last.collectives += 1
        merged = out[0].clone()
        for r in range(1, world):
            merged |= out[r]
        return unpack_mask(merged, visible.numel())

    # ---- leaf gradients -----------------------------------------------------------
    def _reduce_flat(self, flat: torch.Tensor) -> None:
        per = max(1, self.bucket_bytes // flat.element_size())
        works = []
        for start in range(0, flat.numel(), per):
            works.append(dist.all_reduce(flat[start:start + per], op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))
        for w in works:
            w.wait()
        self.last.collectives += len(works)
        self.last.reduced_bytes += flat.numel() * flat.element_size()

    def sum_gradients(self, grads: Iterable[torch.Tensor], union: Optional[torch.Tensor] = None) -> None:
        """In-place SUM over ranks of per-Gaussian gradients (each (N, ...), same N).

        With `union` (bool (N,), identical on every rank) only those rows are packed and
        reduced; rows outside it must be zero on every rank.
        """
        grads = [g for g in grads if g is not None]
        if not grads:
            return
        n = grads[0].size(0)
        for g in grads:
            if g.size(0) != n:
                raise ValueError("all gradients must have the same number of rows")
            if g.dtype != torch.float32:
                raise ValueError("gradients are exchanged in fp32")
            if not g.is_contiguous():
                raise ValueError("gradients must be contiguous (results are written back in place)")
        rows = None
        if union is not None and self.compact:
            rows = union.nonzero().flatten()
            self.last.union_rows = rows.numel()
            if rows.numel() == 0:
                return
        else:
            self.last.union_rows = n
        widths = [g[0].numel() if n else 0 for g in grads]
        parts = [(g.reshape(n, -1) if rows is None else g.reshape(n, -1).index_select(0, rows)) for g in grads]
        flat = torch.cat([p.reshape(-1) for p in parts])
        self._reduce_flat(flat)
        nr = n if rows is None else rows.numel()
        off = 0
        for g, w in zip(grads, widths):
            block = flat[off:off + nr * w].view(nr, w)
            off += nr * w
            if rows is None:
                g.reshape(n, -1).copy_(block)
            else:
                g.reshape(n, -1).index_copy_(0, rows, block)

    # ---- statistics ---------------------------------------------------------------
    def max_stats(self, stats: Iterable[torch.Tensor]) -> None:
        for s in stats:
            if s is not None:
                dist.all_reduce(s, op=dist.ReduceOp.MAX, group=self.group)
                self.last.collectives += 1

    def sum_stats(self, stats: Iterable[torch.Tensor]) -> None:
        for s in stats:
            if s is not None:
                dist.all_reduce(s, op=dist.ReduceOp.SUM, group=self.group)
                self.last.collectives += 1

    # ---- the whole exchange step ----------------------------------------------------
    def exchange(self, grads: Dict[str, torch.Tensor], visible: torch.Tensor,
                 max_stats: Optional[List[torch.Tensor]] = None,
                 sum_stats: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
        """Run one exchange step; returns the union visibility mask (for the masked Adam)."""
        self.last = ExchangeStats()
        union = self.union_visibility(visible)
        self.sum_gradients(grads.values(), union if self.compact else None)
        self.max_stats(max_stats or [])
        self.sum_stats(sum_stats or [])
        return union


LEAF_WIDTHS = {"xyz": 3, "f_dc": 3, "f_rest": 45, "opacity": 1, "scaling": 3, "rotation": 4}
"""Per-Gaussian fp32 widths of the HiDeGS leaf parameters (59 floats = 236 B; SURVEY §8(e) E1)."""
