"""Binning-primitive oracles -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Generic integer definitions of the three primitives between preprocess and render in
Rasterizer::forward, as the reference calls them (no reference code is restated):
  * inclusive scan of uint32, wrapping mod 2^32     (cub::DeviceScan::InclusiveSum,
    rasterizer_impl.cu:321)
  * stable sort of (key, value) pairs by key bits [begin, end)  (cub::DeviceRadixSort::
    SortPairs, rasterizer_impl.cu:357-362; CUB documents the sort as stable)
  * per-tile [start, end) of the sorted keys, tile = key >> 32, with the reference's
    documented n == 1 edge (identifyTileRanges writes the end of the last range only for
    idx > 0, rasterizer_impl.cu:130-141; ranges zeroed first, :364)
"""
from __future__ import annotations

import numpy as np


def inclusive_scan_u32(x: np.ndarray) -> np.ndarray:
    return np.cumsum(x.astype(np.uint64), dtype=np.uint64).astype(np.uint32)


def stable_sort_pairs(keys: np.ndarray, vals: np.ndarray, begin_bit: int, end_bit: int):
    width = end_bit - begin_bit
    k = keys.astype(np.uint64)
    sub = (k >> np.uint64(begin_bit)) & np.uint64((1 << width) - 1) if width < 64 else k
    order = np.argsort(sub, kind="stable")
    return keys[order], vals[order]


def tile_ranges(sorted_keys: np.ndarray, num_tiles: int) -> np.ndarray:
    ranges = np.zeros((num_tiles, 2), dtype=np.int64)
    n = sorted_keys.shape[0]
    if n == 0:
        return ranges.astype(np.uint32)
    tiles = (sorted_keys.astype(np.uint64) >> np.uint64(32)).astype(np.int64)
    starts = np.flatnonzero(np.r_[True, tiles[1:] != tiles[:-1]])
    ends = np.r_[starts[1:], n]
    ranges[tiles[starts], 0] = starts
    ranges[tiles[starts], 1] = ends
    if n == 1:
        ranges[tiles[0], 1] = 0
    return ranges.astype(np.uint32)


def bit_length_at_least_one(n: int) -> int:
    """The value getHigherMsb returns (KATs: 64 -> 7, 8160 -> 13, 32400 -> 15)."""
    return max(1, int(n).bit_length())
