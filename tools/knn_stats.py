"""Prints distCUDA2 search statistics (HIDEGS_KNN_STATS=1) and timing for a few distributions."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HIDEGS_KNN_STATS"] = "2"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import simple_knn  # noqa: E402
from hidegs_amd import _lib, synthetic  # noqa: E402

sets = {
    "frustum2M": synthetic.frustum_points(2_000_000),
    "uniform2M": torch.rand(2_000_000, 3),
    "plane2M": torch.cat([torch.rand(2_000_000, 2), torch.zeros(2_000_000, 1)], 1),
}
for name, pts in sets.items():
    p = pts.cuda()
    simple_knn._C.distCUDA2(p)
    torch.cuda.synchronize()
    os.environ["HIDEGS_KNN_STATS"] = "0"
    with _lib.kernel_timer() as kt:
        t = time.perf_counter()
        simple_knn._C.distCUDA2(p)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(name, f"total {dt*1e3:.2f} ms", {k: round(kt.get(k)[0] * 1e3, 1) for k in ("knn_leaf", "knn_hard", "radix_scatter_u64")}, flush=True)
    os.environ["HIDEGS_KNN_STATS"] = "2"
