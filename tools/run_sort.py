"""Runs the binning sort of the bench workload a few times (profiling target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import primitives, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
wl = synthetic.binning_workload(2_000_000, device="cuda")
end = 32 + primitives.higher_msb(wl.num_tiles)
for _ in range(reps):
    primitives.sort_tile_pairs(wl.keys, wl.values, wl.num_tiles)
torch.cuda.synchronize()
print("ok", wl.num_pairs)
