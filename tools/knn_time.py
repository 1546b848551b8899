import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import simple_knn
from hidegs_amd import synthetic, _lib
sets = {"frustum2M": synthetic.frustum_points(2_000_000), "uniform2M": torch.rand(2_000_000, 3),
        "plane2M": torch.cat([torch.rand(2_000_000, 2), torch.zeros(2_000_000, 1)], 1)}
for name, pts in sets.items():
    p = pts.cuda()
    simple_knn._C.distCUDA2(p); torch.cuda.synchronize()
    with _lib.kernel_timer() as kt:
        for _ in range(3):
            simple_knn._C.distCUDA2(p)
        torch.cuda.synchronize()
        print(name, {k: round(kt.get(k)[0] * 1e3 / 3, 1) for k in ("knn_leaf", "knn_hard", "radix_scatter_u64", "gather", "leaf_box")}, flush=True)
