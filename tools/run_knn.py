"""Runs distCUDA2 on the 2M D2 centres a few times (profiling target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import simple_knn  # noqa: E402
from hidegs_amd import synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
pts = synthetic.frustum_points(2_000_000).cuda()
for _ in range(reps):
    simple_knn._C.distCUDA2(pts)
torch.cuda.synchronize()
print("ok")
