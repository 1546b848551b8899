"""CPU oracle -- TEST INFRASTRUCTURE ONLY.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and only as
the checker or the timed CPU baseline.  The product packages (diff_gaussian_rasterization,
simple_knn, hidegs_amd) never import it.

  knn_mean3 / knn_mean3_subset  -- distCUDA2's value from its definition (knn_ref.c)
  masked_adam                   -- one OurAdam step on one parameter tensor (adam_ref.c)
  stable_sort_pairs / inclusive_scan_u32 / tile_ranges -- generic integer restatements
     of the binning primitives (numpy), see binning.py
  sort_pairs_omp                -- the same stable sort as a multi-threaded C radix sort
                                   (sort_ref.c): the binning step's CPU baseline on all cores
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        dll = C.CDLL(LIB_PATH)
        dll.oracle_knn_mean3.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p]
        dll.oracle_knn_mean3.restype = None
        dll.oracle_knn_mean3_subset.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_longlong, C.c_void_p]
        dll.oracle_knn_mean3_subset.restype = None
        dll.oracle_masked_adam.argtypes = [C.c_void_p] * 5 + [C.c_longlong, C.c_int] + [C.c_double] * 5 + \
            [C.c_longlong]
        dll.oracle_masked_adam.restype = None
        dll.oracle_sort_pairs_u64.argtypes = [C.c_void_p] * 4 + [C.c_longlong, C.c_int, C.c_int, C.c_int]
        dll.oracle_sort_pairs_u64.restype = C.c_int
        dll.oracle_set_threads.argtypes = [C.c_int]
        dll.oracle_set_threads.restype = None
        dll.oracle_max_threads.argtypes = []
        dll.oracle_max_threads.restype = C.c_int
        _lib = dll
    return _lib


def knn_mean3(points: np.ndarray) -> np.ndarray:
    """distCUDA2 value for every point of a (P, 3) float32 array (brute force, OpenMP)."""
    pts = np.ascontiguousarray(points, dtype=np.float32)
    out = np.empty(pts.shape[0], dtype=np.float32)
    if pts.shape[0]:
        lib().oracle_knn_mean3(pts.ctypes.data, pts.shape[0], out.ctypes.data)
    return out


def knn_mean3_subset(points: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """distCUDA2 value for the queries idx only (each against all points)."""
    pts = np.ascontiguousarray(points, dtype=np.float32)
    ii = np.ascontiguousarray(idx, dtype=np.int64)
    out = np.empty(ii.shape[0], dtype=np.float32)
    if ii.shape[0]:
        lib().oracle_knn_mean3_subset(pts.ctypes.data, pts.shape[0], ii.ctypes.data, ii.shape[0], out.ctypes.data)
    return out


def masked_adam(param, grad, exp_avg, exp_avg_sq, relevant, lr, beta1=0.9, beta2=0.999, eps=1e-8,
                weight_decay=0.0, step=1):
    """One OurAdam step on float32 arrays (rows, ...) updated in place; relevant: bool (rows,) or None."""
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (param, grad, exp_avg, exp_avg_sq)]
    for a, orig in zip(arrs, (param, grad, exp_avg, exp_avg_sq)):
        if a is not orig:
            raise ValueError("arrays must be contiguous float32 (updated in place)")
    rows = param.shape[0]
    width = int(np.prod(param.shape[1:])) if param.ndim > 1 else 1
    rel = None if relevant is None else np.ascontiguousarray(relevant, dtype=np.uint8)
    lib().oracle_masked_adam(param.ctypes.data, grad.ctypes.data, exp_avg.ctypes.data, exp_avg_sq.ctypes.data,
                             None if rel is None else rel.ctypes.data, rows, width, lr, beta1, beta2, eps,
                             weight_decay, int(step))


def sort_pairs_omp(keys: np.ndarray, vals: np.ndarray, begin_bit: int, end_bit: int, threads: int = 0):
    """Stable sort of (uint64 key, uint32 value) pairs by key bits [begin_bit, end_bit), OpenMP radix
    sort on `threads` threads (0: OpenMP's default).  Same result as binning.stable_sort_pairs."""
    k = np.ascontiguousarray(keys, dtype=np.uint64)
    v = np.ascontiguousarray(vals, dtype=np.uint32)
    ko, vo = np.empty_like(k), np.empty_like(v)
    if k.shape[0]:
        rc = lib().oracle_sort_pairs_u64(k.ctypes.data, v.ctypes.data, ko.ctypes.data, vo.ctypes.data, k.shape[0],
                                         int(begin_bit), int(end_bit), int(threads))
        if rc != 0:
            raise MemoryError("oracle_sort_pairs_u64: allocation failed")
    return ko, vo


def set_threads(threads: int) -> int:
    """OpenMP thread count of the oracle's later calls; returns the count now in force."""
    lib().oracle_set_threads(int(threads))
    return int(lib().oracle_max_threads())
