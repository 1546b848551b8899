"""Torch-facing wrappers of the binning primitives in include/hidegs.h.

These are the stages between preprocess and render in Rasterizer::forward
(rasterizer_impl.cu:321-371): inclusive scan of tiles_touched, the stable radix sort
of (tile|depth key, Gaussian id) pairs over bits [0, 32 + getHigherMsb(tiles)), and
the tile-range split of the sorted keys.  Keys are carried in int64 / int32 tensors
holding the unsigned bit patterns.  Every call runs the gfx950 kernels on PyTorch's
current stream of the tensors' device; there is no CPU fallback.
"""
from __future__ import annotations

from typing import Tuple

import torch

from hidegs_amd import _lib


def _scratch(nbytes: int, device) -> torch.Tensor:
    return torch.empty((max(int(nbytes), 1),), dtype=torch.uint8, device=device)


def higher_msb(n: int) -> int:
    """getHigherMsb (rasterizer_impl.cu:35-50): bits needed to hold n (at least 1)."""
    if not 0 <= int(n) < (1 << 32):
        raise ValueError("getHigherMsb takes a uint32")
    return int(_lib.lib().hidegs_higher_msb(int(n)))


def inclusive_scan_u32(x: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """Inclusive prefix sum of a uint32 bit-pattern tensor (int32 or uint32 dtype), mod 2^32."""
    if x.dtype not in (torch.int32, torch.uint32) or x.dim() != 1:
        raise RuntimeError("inclusive_scan_u32 takes a 1-D int32/uint32 tensor")
    n = x.numel()
    out = torch.empty_like(x) if out is None else out
    if n == 0:
        return out
    dev = _lib.device_of(x, out)
    xi = x.contiguous()
    L = _lib.lib()
    with torch.cuda.device(dev):
        tmp = _scratch(L.hidegs_scan_scratch_bytes(n), dev)
        rc = L.hidegs_inclusive_scan_u32(_lib.ptr(tmp), tmp.numel(), _lib.ptr(xi), _lib.ptr(out), n,
                                         _lib.stream_handle(dev))
        _lib.check(rc, "inclusive_scan_u32")
    return out


def sort_pairs(keys: torch.Tensor, values: torch.Tensor, begin_bit: int = 0,
               end_bit: int = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stable radix sort of (key, value) pairs by key bits [begin_bit, end_bit).

    keys: int64 (u64 bit patterns) or int32 (u32); values: int32 (u32).  Returns new
    (keys_sorted, values_sorted); the inputs are not modified.
    """
    if keys.dim() != 1 or values.dim() != 1 or keys.numel() != values.numel():
        raise RuntimeError("sort_pairs takes 1-D keys and values of equal length")
    if values.dtype not in (torch.int32, torch.uint32):
        raise RuntimeError("values must be 32-bit")
    if keys.dtype in (torch.int64, torch.uint64):
        kbits, fn, sz = 64, "hidegs_sort_pairs_u64", "hidegs_sort_pairs_u64_scratch_bytes"
    elif keys.dtype in (torch.int32, torch.uint32):
        kbits, fn, sz = 32, "hidegs_sort_pairs_u32", "hidegs_sort_pairs_u32_scratch_bytes"
    else:
        raise RuntimeError("keys must be 64- or 32-bit integers")
    end_bit = kbits if end_bit is None else int(end_bit)
    n = keys.numel()
    ko, vo = torch.empty_like(keys), torch.empty_like(values)
    if n == 0:
        return ko, vo
    dev = _lib.device_of(keys, values)
    ki, vi = keys.contiguous(), values.contiguous()
    L = _lib.lib()
    with torch.cuda.device(dev):
        tmp = _scratch(getattr(L, sz)(n), dev)
        rc = getattr(L, fn)(_lib.ptr(tmp), tmp.numel(), _lib.ptr(ki), _lib.ptr(ko), _lib.ptr(vi), _lib.ptr(vo), n,
                            int(begin_bit), end_bit, _lib.stream_handle(dev))
        _lib.check(rc, fn)
    return ko, vo


def sort_tile_pairs(keys: torch.Tensor, values: torch.Tensor,
                    num_tiles: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """The reference's SortPairs + memset + identifyTileRanges (rasterizer_impl.cu:354-371) in one
    call: pairs sorted over [0, 32 + getHigherMsb(num_tiles)) and the (num_tiles, 2) tile ranges.

    keys are (tile << 32 | depth bits) with tile < num_tiles.  The same results as sort_pairs
    followed by identify_tile_ranges; the per-tile ranges the sort computes anyway are the output.
    """
    if keys.dtype not in (torch.int64, torch.uint64) or keys.dim() != 1:
        raise RuntimeError("sort_tile_pairs takes 1-D 64-bit keys")
    if values.dtype not in (torch.int32, torch.uint32) or values.dim() != 1 or values.numel() != keys.numel():
        raise RuntimeError("sort_tile_pairs takes 32-bit values, one per key")
    n = keys.numel()
    dev = _lib.device_of(keys, values) if n else _lib.device_of(keys)
    ko, vo = torch.empty_like(keys), torch.empty_like(values)
    ranges = torch.empty((int(num_tiles), 2), dtype=torch.int32, device=dev)
    ki, vi = keys.contiguous(), values.contiguous()
    L = _lib.lib()
    with torch.cuda.device(dev):
        tmp = _scratch(L.hidegs_sort_pairs_u64_scratch_bytes(n), dev)
        rc = L.hidegs_sort_tile_pairs(_lib.ptr(tmp), tmp.numel(), _lib.ptr(ki), _lib.ptr(ko), _lib.ptr(vi),
                                      _lib.ptr(vo), n, int(num_tiles), _lib.ptr(ranges), _lib.stream_handle(dev))
        _lib.check(rc, "sort_tile_pairs")
    return ko, vo, ranges


def identify_tile_ranges(sorted_keys: torch.Tensor, num_tiles: int) -> torch.Tensor:
    """(num_tiles, 2) int32 [start, end) of each tile (key >> 32) in the sorted list."""
    if sorted_keys.dtype not in (torch.int64, torch.uint64) or sorted_keys.dim() != 1:
        raise RuntimeError("identify_tile_ranges takes 1-D 64-bit keys")
    dev = sorted_keys.device if sorted_keys.numel() else None
    if dev is None or dev.type != "cuda":
        dev = _lib.device_of(sorted_keys)
    ranges = torch.empty((int(num_tiles), 2), dtype=torch.int32, device=dev)
    k = sorted_keys.contiguous()
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_identify_tile_ranges(_lib.ptr(k), k.numel(), _lib.ptr(ranges), int(num_tiles),
                                                    _lib.stream_handle(dev))
        _lib.check(rc, "identify_tile_ranges")
    return ranges


def queue_error(device=None, clear: bool = True) -> int:
    """Sticky error word of the hot-tile partition queue on `device` (hidegs_queue_error): 0, or
    bit 1 (job slots exhausted) / bit 4 (a worker gave up) if some sort since the last clear returned
    pairs that are not fully sorted.  Synchronises the current stream."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    flags = _lib.C.c_uint32(0)
    with torch.cuda.device(dev):
        rc = _lib.lib().hidegs_queue_error(_lib.stream_handle(dev), int(bool(clear)), _lib.C.byref(flags))
    _lib.check(rc, "queue_error")
    return int(flags.value)


def set_debug(enable: bool) -> None:
    """Library-wide debug mode (hidegs_set_debug): synchronising launch checks, and every sort
    verifies the partition queue's error word and raises RuntimeError if it is set."""
    _lib.lib().hidegs_set_debug(int(bool(enable)))
