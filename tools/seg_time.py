"""Per-kernel times of the binning sort (bench workload) with the library HIDEGS_LIB points at."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib, primitives, synthetic  # noqa: E402

big = len(sys.argv) > 1 and sys.argv[1] == "4k"  # config 5's frame: 10M Gaussians at 3840 x 2160
wl = synthetic.binning_workload(10_000_000 if big else 2_000_000, 3840 if big else 1920, 2160 if big else 1080,
                                seed=0, device="cuda")
end = 32 + primitives.higher_msb(wl.num_tiles)
for _ in range(10):
    primitives.sort_pairs(wl.keys, wl.values, 0, end)
torch.cuda.synchronize()
with _lib.kernel_timer() as kt:
    for _ in range(50):
        primitives.sort_pairs(wl.keys, wl.values, 0, end)
    torch.cuda.synchronize()
    out = []
    for nm in ("radix_hist_u64", "radix_digit_scan", "radix_scatter_u64", "segment_ranges", "segment_sort",
               "big_segments"):
        ms, n = kt.get(nm)
        if n:
            out.append(f"{nm} {ms * 1e3 / n:.1f}us")
print(os.environ.get("HIDEGS_LIB", "default"), "4k" if big else "1080p", " ".join(out), flush=True)
