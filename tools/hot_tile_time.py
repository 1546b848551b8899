"""Binning sort time with one hot tile of S pairs among the bench's 8M pairs (the per-tile sort's
partition queue: segment_sort opens the record, big_segments runs it), against the bench workload
without it."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib, primitives, synthetic  # noqa: E402

wl = synthetic.binning_workload(2_000_000, 1920, 1080, seed=0, device="cuda")
T = wl.num_tiles
for hot in [int(a) for a in sys.argv[1:]] or (0, 4096, 20_000, 100_000, 500_000):
    keys = wl.keys.clone()
    if hot:
        idx = torch.randperm(keys.numel(), device="cuda")[:hot]
        keys[idx] = (keys[idx] & 0xFFFFFFFF) | (4000 << 32)  # move `hot` pairs into tile 4000
    for _ in range(3):
        primitives.sort_tile_pairs(keys, wl.values, T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        primitives.sort_tile_pairs(keys, wl.values, T)
    e1.record()
    torch.cuda.synchronize()
    with _lib.kernel_timer() as kt:
        for _ in range(5):
            primitives.sort_tile_pairs(keys, wl.values, T)
        torch.cuda.synchronize()
        ms, n = kt.get("segment_sort")
        qms, qn = kt.get("big_segments")
    print(f"hot tile {hot:7d} pairs: segment_sort {ms * 1e3 / n:8.1f} us  big_segments {qms * 1e3 / max(qn, 1):8.1f} us"
          f"  whole sort {e0.elapsed_time(e1) * 1e3 / 5:8.1f} us", flush=True)
