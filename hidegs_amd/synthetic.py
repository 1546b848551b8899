"""Seeded synthetic workloads of SURVEY.md §8(d) D2 (generated on the CPU with
torch.Generator().manual_seed(seed), then copied, so oracle and device see the same bits).

  frustum_points(N)   Gaussian centres placed as D2 places them: z ~ U[2, 20],
                      x = u tan(FoVx/2) z, y = v tan(FoVy/2) z, u, v ~ U[-0.95, 0.95],
                      tan(FoVx/2) = tan 30 deg, 1920 x 1080 aspect -- the input of distCUDA2.
  d2_camera()         the D2 camera: identity view, the projection of utils/graphics_utils.py:59-85
                      (znear 0.01, zfar 100, centred principal point) composed as scene/cameras.py:127-130
                      does (row-vector convention), campos 0, black background.
  d2_scene(N)         every per-Gaussian input of the rasterizer API at D2's distribution: centres as
                      above, post-activation scales (sigma_px z / fx) max(0.3, 1 + 0.3 N(0,1)) per
                      axis with screen sigma ~ U[1.5, 3.8] px, normalised random quaternions,
                      opacities ~ U[0.05, 0.95], SH degree 3 (dc ~ N(0, 0.5^2), rest ~ N(0, 0.1^2)),
                      all_map = [n, 1, |n . p|] with a random unit normal n facing the camera.
  d2_upstream_grads() the four per-pixel upstream gradients (colour, inverse depth, all_map,
                      plane depth), N(0, std^2) with seed 1.
  d2_binning_workload(scene)   the binning stage's inputs of one view of that scene: each
                      Gaussian's screen centre (its NDC position, by construction (u, v)) and its
                      3-sigma box from the generator's own screen-space sigma, in 16 x 16 tiles;
                      Gaussian-major (tile << 32 | depth bits, id) pairs.  `cluster` concentrates a
                      fraction of the Gaussians into a disc (the hot tiles of a real view).
  binning_workload()  round-3's synthetic keys: w x h tiles with w, h uniform in {1, 2, 3}, placed
                      uniformly on the tile grid; depth bits those of z.

None of this derives from the reference rasterizer: screen-space footprints come from the
generator's own sigma, not from projecting covariances.
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


def _frustum(n: int, g: torch.Generator, width: int, height: int):
    z = 2 + 18 * torch.rand(n, generator=g)
    u = (torch.rand(n, generator=g) * 2 - 1) * 0.95
    v = (torch.rand(n, generator=g) * 2 - 1) * 0.95
    return z, u, v


def projection_matrix(znear: float, zfar: float, tanfovx: float, tanfovy: float) -> torch.Tensor:
    """Column-vector projection with a centred principal point (utils/graphics_utils.py:59-85)."""
    top, right = tanfovy * znear, tanfovx * znear
    P = torch.zeros(4, 4)
    P[0, 0] = 2.0 * znear / (2 * right)
    P[1, 1] = 2.0 * znear / (2 * top)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class Camera:
    width: int
    height: int
    tanfovx: float
    tanfovy: float
    viewmatrix: torch.Tensor  # (4,4) row-vector convention
    projmatrix: torch.Tensor  # (4,4) view @ projection, row-vector convention
    campos: torch.Tensor      # (3,)
    bg: torch.Tensor          # (3,)

    @property
    def focal(self):
        return self.width / (2.0 * self.tanfovx), self.height / (2.0 * self.tanfovy)

    @property
    def grid(self):
        return (self.width + BLOCK - 1) // BLOCK, (self.height + BLOCK - 1) // BLOCK

    def to(self, device) -> "Camera":
        return Camera(self.width, self.height, self.tanfovx, self.tanfovy, self.viewmatrix.to(device),
                      self.projmatrix.to(device), self.campos.to(device), self.bg.to(device))


def d2_camera(width: int = 1920, height: int = 1080) -> Camera:
    tanfovy = TAN_FOVX * height / width
    view = torch.eye(4)  # world_view_transform (already in the stored, transposed form)
    proj = (view @ projection_matrix(0.01, 100.0, TAN_FOVX, tanfovy).t()).contiguous()
    return Camera(width, height, TAN_FOVX, tanfovy, view, proj, torch.zeros(3), torch.zeros(3))


@dataclass
class Scene:
    means3D: torch.Tensor     # (N, 3)
    scales: torch.Tensor      # (N, 3) post-activation
    rotations: torch.Tensor   # (N, 4) unit quaternions (w, x, y, z)
    opacities: torch.Tensor   # (N, 1) post-activation
    shs: torch.Tensor         # (N, 16, 3)
    all_map: torch.Tensor     # (N, 5)
    sigma_px: torch.Tensor    # (N,) the generator's screen-space sigma
    aniso: torch.Tensor       # (N, 3) per-axis factor of the scales
    ndc: torch.Tensor         # (N, 2) (u, v): the screen position by construction
    sh_degree: int = 3

    @property
    def n(self) -> int:
        return self.means3D.shape[0]

    def to(self, device) -> "Scene":
        f = {k: (getattr(self, k).to(device) if isinstance(getattr(self, k), torch.Tensor) else getattr(self, k))
             for k in self.__dataclass_fields__}
        return Scene(**f)

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.means3D, self.scales, self.rotations,
                                                           self.opacities, self.shs, self.all_map))


def d2_scene(n: int, cam: Camera = None, seed: int = 0, cluster: tuple = None) -> Scene:
    """D2's Gaussians (see the module docstring).  cluster = (fraction, radius in NDC units): that
    fraction of the Gaussians is placed inside a disc about a random screen point."""
    cam = cam or d2_camera()
    g = torch.Generator().manual_seed(seed)
    z, u, v = _frustum(n, g, cam.width, cam.height)
    if cluster is not None:
        frac, rad = cluster
        m = torch.rand(n, generator=g) < frac
        c = (torch.rand(2, generator=g) * 2 - 1) * 0.6
        r = rad * torch.sqrt(torch.rand(n, generator=g))
        a = 2 * math.pi * torch.rand(n, generator=g)
        u = torch.where(m, c[0] + r * torch.cos(a), u)
        v = torch.where(m, c[1] + r * torch.sin(a), v)
    means = torch.stack([u * cam.tanfovx * z, v * cam.tanfovy * z, z], 1).contiguous()
    fx, _ = cam.focal
    sigma = 1.5 + 2.3 * torch.rand(n, generator=g)
    aniso = torch.clamp(1 + 0.3 * torch.randn(n, 3, generator=g), min=0.3)
    scales = ((sigma * z / fx)[:, None] * aniso).contiguous()
    q = torch.randn(n, 4, generator=g)
    rotations = (q / q.norm(dim=1, keepdim=True)).contiguous()
    opacities = (0.05 + 0.9 * torch.rand(n, 1, generator=g)).contiguous()
    shs = torch.cat([0.5 * torch.randn(n, 1, 3, generator=g), 0.1 * torch.randn(n, 15, 3, generator=g)], 1).contiguous()
    nrm = torch.randn(n, 3, generator=g)
    nrm = nrm / nrm.norm(dim=1, keepdim=True)
    to_cam = cam.campos[None] - means
    nrm = torch.where(((nrm * to_cam).sum(1) < 0)[:, None], -nrm, nrm)
    all_map = torch.cat([nrm, torch.ones(n, 1), (nrm * means).sum(1, keepdim=True).abs()], 1).contiguous()
    return Scene(means, scales, rotations, opacities, shs, all_map, sigma, aniso, torch.stack([u, v], 1))


def d2_upstream_grads(cam: Camera = None, seed: int = 1, std: float = 1e-3) -> dict:
    """dL/d(colour (3,H,W), inverse depth (1,H,W), all_map (5,H,W), plane depth (1,H,W))."""
    cam = cam or d2_camera()
    g = torch.Generator().manual_seed(seed)
    H, W = cam.height, cam.width
    return {"color": std * torch.randn(3, H, W, generator=g), "invdepth": std * torch.randn(1, H, W, generator=g),
            "all_map": std * torch.randn(5, H, W, generator=g), "plane_depth": std * torch.randn(1, H, W, generator=g)}


def d2_binning_workload(scene: Scene, cam: Camera = None, device: str = "cpu") -> BinningWorkload:
    """The binning inputs of one view of `scene`: tiles met by each Gaussian's 3-sigma box."""
    cam = cam or d2_camera()
    gx, gy = cam.grid
    u, v = scene.ndc[:, 0].cpu(), scene.ndc[:, 1].cpu()
    px = ((u + 1) * cam.width - 1) * 0.5
    py = ((v + 1) * cam.height - 1) * 0.5
    sig = scene.sigma_px.cpu()
    an = scene.aniso.cpu()
    ex = torch.ceil(3 * sig * an[:, 0])
    ey = torch.ceil(3 * sig * an[:, 1])
    x0 = torch.clamp(torch.floor((px - ex) / BLOCK), 0, gx).long()
    x1 = torch.clamp(torch.floor((px + ex) / BLOCK) + 1, 0, gx).long()
    y0 = torch.clamp(torch.floor((py - ey) / BLOCK), 0, gy).long()
    y1 = torch.clamp(torch.floor((py + ey) / BLOCK) + 1, 0, gy).long()
    w, h = (x1 - x0).clamp(min=0), (y1 - y0).clamp(min=0)
    touched = w * h
    K = int(touched.sum())
    n = scene.n
    owner = torch.repeat_interleave(torch.arange(n), touched)
    start = torch.cumsum(touched, 0) - touched
    j = torch.arange(K) - start[owner]
    wo = w[owner].clamp(min=1)
    tx = x0[owner] + j % wo
    ty = y0[owner] + j // wo
    tile = ty * gx + tx
    depth_bits = scene.means3D[:, 2].cpu().contiguous().view(torch.int32).long() & 0xFFFFFFFF
    keys = (tile << 32) | depth_bits[owner]
    return BinningWorkload(touched.int().to(device), keys.to(device), owner.int().to(device), gx * gy, (gx, gy))
