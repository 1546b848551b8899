"""`simple_knn._C.distCUDA2(points) -> (P,) float32`, backed by hidegs_dist_cuda2 (include/hidegs.h).

Contract of submodules/simple-knn/spatial.cu:15-25: points (P,3) float32 on the GPU, result
(P,) float32 on the same device, the mean squared distance to the 3 nearest other points.
Caller: scene/gaussian_model.py:217 (clamped at 1e-7 there).  Runs the gfx950 kernels in
hidegs_amd/csrc/knn.hip on PyTorch's current stream; there is no CPU fallback.
"""
from __future__ import annotations

import torch

from hidegs_amd import _lib


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    if points.dim() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    if points.dtype != torch.float32:
        raise RuntimeError("points must be float32")
    P = points.size(0)
    dev = _lib.device_of(points) if P else points.device
    means = torch.zeros((P,), dtype=torch.float32, device=points.device)
    if P == 0:
        return means
    pts = points.contiguous()
    with torch.cuda.device(dev):
        scratch = _lib.Scratch(dev)
        rc = _lib.lib().hidegs_dist_cuda2(scratch.callback, None, P, _lib.ptr(pts), _lib.ptr(means),
                                          _lib.stream_handle(dev))
        _lib.check_with(rc, "distCUDA2", scratch)
    return means
