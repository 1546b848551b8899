"""Seeded synthetic workloads of SURVEY.md §8(d) D2 (generated on the CPU with
torch.Generator().manual_seed(seed), then copied, so oracle and device see the same bits).

  frustum_points(N)   Gaussian centres placed as D2 places them: z ~ U[2, 20],
                      x = u tan(FoVx/2) z, y = v tan(FoVy/2) z, u, v ~ U[-0.95, 0.95],
                      tan(FoVx/2) = tan 30 deg, 1920 x 1080 aspect -- the input of distCUDA2.
  binning_workload()  the binning stage's inputs for one 1920 x 1080 view: per-Gaussian
                      tiles_touched and the Gaussian-major (tile << 32 | depth bits, id)
                      pairs the forward sorts.  Footprints are w x h tiles with w, h
                      uniform in {1, 2, 3} (E[w h] = 4, so K ~ 4N as D2 specifies), placed
                      uniformly on the 120 x 68 tile grid; depth bits are those of z.
                      Synthetic keys of the sorted shape, not a rasterizer's projection.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

TAN_FOVX = math.tan(math.radians(30.0))
BLOCK = 16  # tile edge in pixels (cuda_rasterizer/config.h:17-18)


def frustum_points(n: int, seed: int = 0, width: int = 1920, height: int = 1080) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    z = 2 + 18 * torch.rand(n, generator=g)
    u = (torch.rand(n, generator=g) * 2 - 1) * 0.95
    v = (torch.rand(n, generator=g) * 2 - 1) * 0.95
    tan_y = TAN_FOVX * height / width
    return torch.stack([u * TAN_FOVX * z, v * tan_y * z, z], 1).contiguous()


@dataclass
class BinningWorkload:
    tiles_touched: torch.Tensor  # (N,) int32 (u32 counts)
    keys: torch.Tensor           # (K,) int64 (u64 tile << 32 | depth bits), Gaussian-major
    values: torch.Tensor         # (K,) int32 Gaussian ids
    num_tiles: int
    grid: tuple

    @property
    def num_pairs(self) -> int:
        return int(self.keys.numel())


def binning_workload(n: int, width: int = 1920, height: int = 1080, seed: int = 0,
                     device: str = "cpu") -> BinningWorkload:
    gx, gy = (width + BLOCK - 1) // BLOCK, (height + BLOCK - 1) // BLOCK
    g = torch.Generator().manual_seed(seed)
    w = torch.randint(1, 4, (n,), generator=g)
    h = torch.randint(1, 4, (n,), generator=g)
    x0 = (torch.rand(n, generator=g) * (gx - w + 1).float()).long()
    y0 = (torch.rand(n, generator=g) * (gy - h + 1).float()).long()
    z = 2 + 18 * torch.rand(n, generator=g)
    depth_bits = z.view(torch.int32).long() & 0xFFFFFFFF
    touched = (w * h).int()
    K = int(touched.sum())
    owner = torch.repeat_interleave(torch.arange(n), touched.long())
    start = torch.cumsum(touched.long(), 0) - touched.long()
    j = torch.arange(K) - start[owner]           # index inside the Gaussian's footprint (row-major)
    tx = x0[owner] + j % w[owner]
    ty = y0[owner] + j // w[owner]
    tile = ty * gx + tx
    keys = (tile << 32) | depth_bits[owner]
    return BinningWorkload(touched.to(device), keys.to(device), owner.int().to(device), gx * gy, (gx, gy))
