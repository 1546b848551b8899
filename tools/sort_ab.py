"""sort_tile_pairs time (HIP events, mean of 50 calls after warm-up) on the bench's 1080p workload and
config 5's 4K workload, with the library HIDEGS_LIB points at (A/B builds)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import primitives, synthetic  # noqa: E402

out = []
for n, w, h in ((2_000_000, 1920, 1080), (10_000_000, 3840, 2160)):
    wl = synthetic.binning_workload(n, w, h, seed=0, device="cuda")
    for _ in range(5):
        primitives.sort_tile_pairs(wl.keys, wl.values, wl.num_tiles)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        primitives.sort_tile_pairs(wl.keys, wl.values, wl.num_tiles)
    e1.record()
    torch.cuda.synchronize()
    out.append(f"{w}x{h} {e0.elapsed_time(e1) * 1e3 / 50:.1f}us")
    del wl
print(os.environ.get("HIDEGS_LIB", "default"), " ".join(out), flush=True)
