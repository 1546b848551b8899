"""Runs tools/probes/tile_part.hip (a one-pass unstable tile partition) on the bench's D2
view (2M Gaussians, 1080p, 8.59M pairs) beside the product's hidegs_sort_tile_pairs, same process, same box.

For each probe mode: the partition is checked (every tile's pairs are exactly its input pairs: the output's
tiles ascend, and the (key, value) multisets agree), then timed per phase with HIP events (median of 20).
The product's per-kernel times come from hidegs_kernel_timing over 20 calls.
usage: python tools/probes/tile_part.py [n_gaussians]
"""
import ctypes as C
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from hidegs_amd import _lib, primitives, synthetic  # noqa: E402

lib = C.CDLL(os.path.join(HERE, "libtile_part.so"))
lib.tp_partition.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_longlong, C.c_int,
                             C.c_void_p, C.c_int, C.c_void_p]
lib.tp_scratch_words.argtypes = [C.c_int, C.c_longlong, C.c_int]
lib.tp_scratch_words.restype = C.c_longlong

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
dev = torch.device("cuda", 0)
cam = synthetic.d2_camera()
wl = synthetic.d2_binning_workload(synthetic.d2_scene(N, cam, seed=0), cam, device=dev)
K, T = wl.num_pairs, wl.num_tiles
print(f"pairs {K}, tiles {T}", flush=True)
stream = torch.cuda.current_stream().cuda_stream


def ev_time(fn, reps=20):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


# the product, per kernel
with _lib.kernel_timer() as kt:
    for _ in range(20):
        primitives.sort_tile_pairs(wl.keys, wl.values, T)
    torch.cuda.synchronize()
    prod = {nm: kt.get(nm) for nm in ("radix_hist_u64", "radix_digit_scan", "radix_scatter_u64", "segment_sort",
                                       "big_segments", "piece_sort")}
part_us = sum(prod[nm][0] * 1e3 / 20 for nm in ("radix_hist_u64", "radix_digit_scan", "radix_scatter_u64"))
print("product per step (us): " + ", ".join(f"{nm} {ms * 1e3 / 20:.1f} ({n // 20}x)" for nm, (ms, n) in prod.items()),
      flush=True)
print(f"product tile grouping (2 LSD passes: hist + digit scan + scatter): {part_us:.1f} us", flush=True)
whole = ev_time(lambda: primitives.sort_tile_pairs(wl.keys, wl.values, T))
print(f"product sort_tile_pairs whole: {whole:.1f} us", flush=True)

ko = torch.empty_like(wl.keys)
vo = torch.empty_like(wl.values)
ref_tiles = torch.sort(wl.keys >> 32).values
ref_pairs = torch.sort(wl.keys).values  # the keys' multiset
for mode, name in ((0, "direct S=16K"), (1, "direct S=32K"), (2, "staged S=8K")):
    scratch = torch.empty(lib.tp_scratch_words(mode, K, T), dtype=torch.int32, device=dev)

    def run(mask=7):
        assert lib.tp_partition(mode, wl.keys.data_ptr(), wl.values.data_ptr(), ko.data_ptr(), vo.data_ptr(), K, T,
                                scratch.data_ptr(), mask, stream) == 0
    ko.fill_(-1)
    run()
    torch.cuda.synchronize()
    tiles = ko >> 32
    ok = bool((tiles[1:] >= tiles[:-1]).all()) and torch.equal(tiles, ref_tiles)
    # pairs preserved: (key, value) as one sortable int64 per pair (value < 2^31 here), compared as multisets
    a = torch.sort((wl.keys & 0xFFFFFFFF) * 2**31 + wl.values.long()).values
    b = torch.sort((ko & 0xFFFFFFFF) * 2**31 + vo.long()).values
    ok = ok and torch.equal(a, b) and torch.equal(torch.sort(ko).values, ref_pairs)
    t_all = ev_time(lambda: run(7))
    t_cnt = ev_time(lambda: run(1))
    # the column scan works in place: every timed scan gets fresh counts first (untimed)
    ts = []
    for _ in range(20):
        run(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(2)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    t_scan = statistics.median(ts)
    run(3)  # consistent prefixes for the scatter-only timing (the scatter does not modify them)
    t_sc = ev_time(lambda: run(4))
    print(f"probe {name}: partition ok={ok}; whole {t_all:.1f} us = count {t_cnt:.1f} + column/tile scans "
          f"{t_scan:.1f} + scatter {t_sc:.1f}; scatter at 24 B/pair = {24 * K / (t_sc * 1e-6) / 1e12:.2f} TB/s",
          flush=True)
