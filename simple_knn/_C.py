"""`simple_knn._C.distCUDA2(points) -> (P,) float32`, backed by hidegs_dist_cuda2 (include/hidegs.h).

Contract of submodules/simple-knn/spatial.cu:15-25: points (P,3) float32 on the GPU, result
(P,) float32 on the same device, the mean squared distance to the 3 nearest other points.
Caller: scene/gaussian_model.py:217 (clamped at 1e-7 there).
"""
from __future__ import annotations

import torch

from hidegs_amd import _lib


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    P = points.size(0)
    means = torch.zeros((P,), dtype=torch.float32, device=points.device)
    if P == 0:
        return means
    pts = points.contiguous()
    scratch = torch.empty((0,), dtype=torch.uint8, device=points.device)

    def alloc(_user, nbytes):
        try:
            scratch.resize_(int(nbytes))
            return scratch.data_ptr() if nbytes else None
        except Exception:
            return None

    cb = _lib.ALLOC_FN(alloc)
    rc = _lib.lib().hidegs_dist_cuda2(cb, None, P, _lib.ptr(pts), _lib.ptr(means), _lib.current_stream_handle())
    _lib.check(rc, "distCUDA2")
    return means
