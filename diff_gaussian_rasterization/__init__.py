"""Drop-in `diff_gaussian_rasterization` for HiDeGS, backed by the hidegs_amd C ABI.

Public surface identical to the reference package
(submodules/hierarchy-rasterizer/diff_gaussian_rasterization/__init__.py:17-230):
  * GaussianRasterizationSettings -- the same 18 fields in the same order (the order is ABI);
  * GaussianRasterizer(nn.Module) with forward(...) -> (color, radii, out_observe, out_all_map,
    plane_depth, invdepth) and markVisible(positions);
  * rasterize_gaussians(...) and the `_C` submodule.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_C"]


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    render_indices: torch.Tensor
    parent_indices: torch.Tensor
    interpolation_weights: torch.Tensor
    num_node_kids: torch.Tensor
    do_depth: bool
    render_geo: bool


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, all_maps,
                        raster_settings):
    """Autograd entry point (DGR/__init__.py:17-40)."""
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, all_maps, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    """Forward/backward pair around _C (DGR/__init__.py:42-155).

    `means2D` is an input only so that autograd delivers dL/dmeans2D to it (the
    densification statistics read viewspace_points.grad); its value is unused.
    """

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, all_maps,
                raster_settings):
        s = raster_settings
        (num_rendered, color, radii, out_observe, out_all_map, out_plane_depth, geom, binning, img,
         invdepth) = _C.rasterize_gaussians(
            s.bg, s.render_indices, s.parent_indices, s.interpolation_weights, s.num_node_kids, means3D,
            colors_precomp, all_maps, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp, s.viewmatrix,
            s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree, s.campos,
            s.prefiltered, s.render_geo, s.debug, s.do_depth)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(out_all_map, colors_precomp, all_maps, means3D, scales, rotations, cov3Ds_precomp,
                              radii, sh, opacities, geom, binning, img)
        return color, radii, out_observe, out_all_map, out_plane_depth, invdepth

    @staticmethod
    def backward(ctx, grad_color, _grad_radii, _grad_observe, grad_all_map, grad_plane_depth, grad_invdepth):
        s = ctx.raster_settings
        (all_map_pixels, colors_precomp, all_maps, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities,
         geom, binning, img) = ctx.saved_tensors
        (g_means2D, g_colors, g_opacities, g_means3D, g_cov3D, g_sh, g_scales, g_rotations,
         g_all_map) = _C.rasterize_gaussians_backward(
            s.bg, all_map_pixels, s.render_indices, s.parent_indices, s.interpolation_weights, s.num_node_kids,
            means3D, radii, colors_precomp, all_maps, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_color, grad_all_map, grad_plane_depth,
            grad_invdepth, sh, s.sh_degree, s.campos, geom, ctx.num_rendered, binning, img, s.render_geo, s.debug)
        # gradient order = forward input order (DGR/__init__.py:142-155)
        return (g_means3D, g_means2D, g_sh, g_colors, g_opacities, g_scales, g_rotations, g_cov3D, g_all_map, None)


def _empty_like_ref() -> torch.Tensor:
    # The reference substitutes `torch.Tensor([])` for absent inputs (DGR/__init__.py:204-216).
    return torch.Tensor([])


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Boolean frustum mask (DGR/__init__.py:183-192)."""
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, all_map=None):
        s = self.raster_settings
        # Argument rules and messages of DGR/__init__.py:198-202.
        if (shs is None) == (colors_precomp is None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        have_sr = scales is not None or rotations is not None
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (have_sr and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        shs = _empty_like_ref() if shs is None else shs
        colors_precomp = _empty_like_ref() if colors_precomp is None else colors_precomp
        scales = _empty_like_ref() if scales is None else scales
        rotations = _empty_like_ref() if rotations is None else rotations
        cov3D_precomp = _empty_like_ref() if cov3D_precomp is None else cov3D_precomp
        all_map = _empty_like_ref() if all_map is None else all_map
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                   all_map, s)
