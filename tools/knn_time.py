"""distCUDA2 per-kernel times (median and min of 10 calls) for three 2M-point distributions, with the
library HIDEGS_LIB points at."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import simple_knn  # noqa: E402
from hidegs_amd import _lib, synthetic  # noqa: E402

sets = {"frustum2M": synthetic.frustum_points(2_000_000), "uniform2M": torch.rand(2_000_000, 3),
        "plane2M": torch.cat([torch.rand(2_000_000, 2), torch.zeros(2_000_000, 1)], 1)}
for name, pts in sets.items():
    p = pts.cuda()
    simple_knn._C.distCUDA2(p)
    torch.cuda.synchronize()
    tot = []
    for _ in range(10):  # the whole call, no per-kernel events
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        simple_knn._C.distCUDA2(p)
        e1.record()
        torch.cuda.synchronize()
        tot.append(e0.elapsed_time(e1) * 1e3)
    per = {k: [] for k in ("knn_leaf", "knn_hard", "radix_scatter_u64", "gather", "leaf_box")}
    for _ in range(10):
        with _lib.kernel_timer() as kt:
            simple_knn._C.distCUDA2(p)
            torch.cuda.synchronize()
            for k in per:
                per[k].append(kt.get(k)[0] * 1e3)
    print(name, f"total med {statistics.median(tot):.1f} us", {k: f"med {statistics.median(v):.1f} min {min(v):.1f}"
                                                                 for k, v in per.items()}, flush=True)
