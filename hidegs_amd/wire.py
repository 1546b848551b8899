"""bf16 wire format of the view-DP exchange on the GPU (include/hidegs.h: hidegs_bf16_pack /
_sum_ranks / _unpack; hidegs_amd/csrc/wire.hip).  Device tensors only: each call is one HBM pass on
the tensors' device's current stream, bit-identical to the torch definition it replaces in
view_dp._Bucket (the CPU path of that class keeps the torch ops for gloo ranks)."""
from __future__ import annotations

import torch

from . import _lib


def _need(t: torch.Tensor, dtype: torch.dtype, what: str) -> None:
    if t.dtype != dtype or not t.is_contiguous():
        raise RuntimeError(f"{what}: expected a contiguous {dtype} tensor, got {t.dtype}")


def bf16_pack(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst[:n] = src.to(bfloat16) (round to nearest even), dst[n:] = 0; n = src.numel()."""
    _need(src, torch.float32, "bf16_pack")
    _need(dst, torch.bfloat16, "bf16_pack")
    if dst.numel() < src.numel():
        raise RuntimeError("bf16_pack: destination shorter than the source")
    dev = _lib.device_of(src, dst) if src.numel() else _lib.device_of(dst)
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_bf16_pack(_lib.ptr(src), _lib.ptr(dst), src.numel(), dst.numel(),
                                         _lib.stream_handle(dev))
    _lib.check(rc, "bf16_pack")
    return dst


def bf16_sum_ranks(parts: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """parts (world, chunk) bfloat16 -> (chunk,) bfloat16: the fp32 sum of the rows in rank order,
    rounded once (acc = parts[0].float(); acc += parts[r].float() ...; acc.to(bfloat16))."""
    _need(parts, torch.bfloat16, "bf16_sum_ranks")
    if parts.dim() != 2:
        raise RuntimeError("bf16_sum_ranks: parts must be (world, chunk)")
    world, chunk = parts.shape
    if out is None:
        out = torch.empty(chunk, dtype=torch.bfloat16, device=parts.device)
    _need(out, torch.bfloat16, "bf16_sum_ranks")
    if out.numel() != chunk:
        raise RuntimeError("bf16_sum_ranks: out must hold one chunk")
    if chunk == 0:
        return out
    dev = _lib.device_of(parts, out)
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_bf16_sum_ranks(_lib.ptr(parts), int(world), int(chunk), _lib.ptr(out),
                                              _lib.stream_handle(dev))
    _lib.check(rc, "bf16_sum_ranks")
    return out


def bf16_unpack(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst = src.float() (exact), dst.numel() elements from the front of src."""
    _need(src, torch.bfloat16, "bf16_unpack")
    _need(dst, torch.float32, "bf16_unpack")
    if src.numel() < dst.numel():
        raise RuntimeError("bf16_unpack: source shorter than the destination")
    if dst.numel() == 0:
        return dst
    dev = _lib.device_of(src, dst)
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_bf16_unpack(_lib.ptr(src), _lib.ptr(dst), dst.numel(), _lib.stream_handle(dev))
    _lib.check(rc, "bf16_unpack")
    return dst


def mask_pack(mask: torch.Tensor) -> torch.Tensor:
    """bool (N,) -> uint8 (ceil(N/8),), bit i of byte j = mask[8j + i] (view_dp.pack_mask's bits)."""
    if mask.dtype != torch.bool or mask.dim() != 1 or not mask.is_contiguous():
        raise RuntimeError("mask_pack: expected a contiguous 1-D bool mask")
    bits = torch.empty((mask.numel() + 7) // 8, dtype=torch.uint8, device=mask.device)
    if mask.numel() == 0:
        return bits
    dev = _lib.device_of(mask, bits)
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_mask_pack(_lib.ptr(mask), mask.numel(), _lib.ptr(bits), _lib.stream_handle(dev))
    _lib.check(rc, "mask_pack")
    return bits


def mask_union_count(bits: torch.Tensor, n: int):
    """(R, ceil(n/8)) uint8 packed masks -> (union bool (n,), view count float32 (n, 1)), the
    definition unpack_mask(bits, n).sum(0) > 0 and its float count, in one pass."""
    if bits.dtype != torch.uint8 or bits.dim() != 2 or not bits.is_contiguous() or bits.shape[1] != (n + 7) // 8:
        raise RuntimeError("mask_union_count: expected (ranks, ceil(n/8)) contiguous uint8")
    union = torch.empty(n, dtype=torch.bool, device=bits.device)
    count = torch.empty(n, 1, dtype=torch.float32, device=bits.device)
    if n == 0:
        return union, count
    dev = _lib.device_of(bits, union, count)
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_mask_union_count(_lib.ptr(bits), int(bits.shape[0]), int(n), _lib.ptr(union),
                                                _lib.ptr(count), _lib.stream_handle(dev))
    _lib.check(rc, "mask_union_count")
    return union, count
