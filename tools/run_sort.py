"""Runs the binning sort of the bench workload a few times (profiling target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import primitives, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cam = synthetic.d2_camera(1920, 1080)
wl = synthetic.d2_binning_workload(synthetic.d2_scene(2_000_000, cam, seed=0), cam, device="cuda")  # the bench's view
end = 32 + primitives.higher_msb(wl.num_tiles)
for _ in range(reps):
    primitives.sort_tile_pairs(wl.keys, wl.values, wl.num_tiles)
torch.cuda.synchronize()
print("ok", wl.num_pairs)
