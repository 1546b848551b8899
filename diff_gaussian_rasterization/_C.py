"""`diff_gaussian_rasterization._C` -- the torch-facing half of the drop-in boundary.

Mirrors the reference extension module (submodules/hierarchy-rasterizer/ext.cpp:15-17)
and its glue (rasterize_points.cu:35-279): same entry-point names, the same positional
arguments and return tuples, empty tensor == absent input, zero-filled outputs,
scratch held in uint8 tensors that autograd keeps alive between forward and backward.
The computation itself is delegated to the C ABI (include/hidegs.h) through
hidegs_amd._lib; there is no Python or CPU fallback.
"""
from __future__ import annotations

import torch

from hidegs_amd import _lib

NUM_CHANNELS = 3  # cuda_rasterizer/config.h:15
NUM_ALL_MAP = 5   # cuda_rasterizer/config.h:16

# Anti-aliasing filter variance of the covariance backward.  The reference hard-codes 0.3
# there (backward.cu:211) against 0.1 in the forward (forward.cu:356).  A module attribute
# read on every backward call (not thread-local state), so the value the training thread
# sets is the one autograd's device thread passes to hidegs_rasterize_backward.
H_VAR_BWD = 0.3


def _check_means(means3D: torch.Tensor) -> None:
    if means3D.ndimension() != 2 or means3D.size(1) != 3:  # rasterize_points.cu:64-66
        raise RuntimeError("means3D must have dimensions (num_points, 3)")


def _sh_coeffs(sh: torch.Tensor) -> int:
    """SH coefficients per Gaussian.  The reference reads sh.size(1) only when sh.size(0) != 0
    (rasterize_points.cu:102-106, 189-193), so with zero Gaussians it returns a (0, 0, 3) gradient
    that autograd rejects for a (0, M, 3) input; taking M from the shape avoids that error."""
    return sh.size(1) if sh.dim() >= 2 else 0


def _contig(t):
    return t.contiguous() if t is not None else t


def rasterize_gaussians(background, indices, parent_indices, ts, kids, means3D, colors, all_map, opacity, scales,
                        rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                        image_height, image_width, sh, degree, campos, prefiltered, render_geo, debug, do_depth):
    """RasterizeGaussiansCUDA (rasterize_points.cu:35-147).

    Returns (num_rendered, color, radii, out_observe, out_all_map, out_plane_depth,
             geomBuffer, binningBuffer, imgBuffer, invdepth).
    """
    _check_means(means3D)
    P = indices.size(0) if indices.numel() != 0 else means3D.size(0)
    H, W = int(image_height), int(image_width)
    fopt = dict(dtype=torch.float32, device=means3D.device)
    iopt = dict(dtype=torch.int32, device=means3D.device)

    out_color = torch.zeros((NUM_CHANNELS, H, W), **fopt)
    out_invdepth = torch.zeros((1 if do_depth else 0, H, W), **fopt)
    radii = torch.zeros((P,), **iopt)
    out_observe = torch.zeros((P,), **iopt)
    out_all_map = torch.zeros((NUM_ALL_MAP, H, W), **fopt)
    out_plane_depth = torch.zeros((1, H, W), **fopt)
    geom = torch.empty((0,), dtype=torch.uint8, device=means3D.device)
    binning = torch.empty((0,), dtype=torch.uint8, device=means3D.device)
    img = torch.empty((0,), dtype=torch.uint8, device=means3D.device)

    rendered = 0
    if P != 0:  # rasterize_points.cu:100
        M = _sh_coeffs(sh)
        dev = _lib.device_of(means3D, background, viewmatrix, projmatrix, campos)
        bufs = [_lib.Scratch(dev, t) for t in (geom, binning, img)]
        nr = _lib.C.c_int(0)
        args = [_contig(x) for x in (background, indices, parent_indices, ts, kids, means3D, sh, colors, all_map,
                                     opacity, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, campos)]
        (bg_, idx_, par_, ts_, kids_, m3_, sh_, col_, am_, op_, sc_, rot_, cov_, vm_, pm_, cp_) = args
        rc = _lib.lib().hidegs_rasterize_forward(
            bufs[0].callback, bufs[1].callback, bufs[2].callback, None,
            P, int(degree), M, _lib.ptr(bg_), W, H,
            _lib.ptr(idx_), _lib.ptr(par_), _lib.ptr(ts_), _lib.ptr(kids_),
            _lib.ptr(m3_), _lib.ptr(sh_), _lib.ptr(col_), _lib.ptr(am_),
            _lib.ptr(op_), _lib.ptr(sc_), float(scale_modifier), _lib.ptr(rot_),
            _lib.ptr(cov_), _lib.ptr(vm_), _lib.ptr(pm_), _lib.ptr(cp_),
            float(tan_fovx), float(tan_fovy), int(bool(prefiltered)),
            _lib.ptr(out_color), _lib.ptr(out_invdepth), _lib.ptr(out_observe), _lib.ptr(out_all_map),
            _lib.ptr(out_plane_depth), int(bool(render_geo)), _lib.ptr(radii), int(bool(debug)),
            _lib.stream_handle(dev), _lib.C.byref(nr))
        _lib.check_with(rc, "rasterize_gaussians", *bufs)
        rendered = nr.value
    return (rendered, out_color, radii, out_observe, out_all_map, out_plane_depth, geom, binning, img, out_invdepth)


def rasterize_gaussians_backward(background, all_map_pixels, indices, parent_indices, ts, kids, means3D, radii,
                                 colors, all_maps, opacities, scales, rotations, scale_modifier, cov3D_precomp,
                                 viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dL_dout_all_map,
                                 dL_dout_plane_depth, dL_dout_invdepth, sh, degree, campos, geomBuffer, R,
                                 binningBuffer, imageBuffer, render_geo, debug):
    """RasterizeGaussiansBackwardCUDA (rasterize_points.cu:149-279).

    Returns (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh,
             dL_dscales, dL_drotations, dL_dall_map), each with fullP rows.
    """
    fullP = means3D.size(0)
    P = indices.size(0) if indices.numel() != 0 else fullP
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    M = _sh_coeffs(sh)
    z = lambda *shape: torch.zeros(shape, dtype=means3D.dtype, device=means3D.device)  # noqa: E731
    dL_dmeans3D, dL_dmeans2D = z(fullP, 3), z(fullP, 3)
    dL_dcolors, dL_dall_map = z(fullP, NUM_CHANNELS), z(fullP, NUM_ALL_MAP)
    dL_dopacity, dL_dcov3D = z(fullP, 1), z(fullP, 6)
    dL_dsh, dL_dscales, dL_drotations = z(fullP, M, 3), z(fullP, 3), z(fullP, 4)
    dinv = dL_dout_invdepth if dL_dout_invdepth.size(0) != 0 else None  # rasterize_points.cu:210-216

    if P != 0:  # rasterize_points.cu:218
        dev = _lib.device_of(means3D, background, viewmatrix, projmatrix, campos, geomBuffer)
        args = [_contig(x) for x in (background, all_map_pixels, indices, parent_indices, ts, kids, means3D, sh,
                                     colors, all_maps, scales, opacities, rotations, cov3D_precomp, viewmatrix,
                                     projmatrix, campos, radii, dL_dout_color, dL_dout_all_map, dL_dout_plane_depth,
                                     dinv)]
        (bg_, amp_, idx_, par_, ts_, kids_, m3_, sh_, col_, am_, sc_, op_, rot_, cov_, vm_, pm_, cp_, rad_,
         dpix_, dam_, dpl_, dinv_) = args
        rc = _lib.lib().hidegs_rasterize_backward(
            P, int(degree), M, int(R), _lib.ptr(bg_), _lib.ptr(amp_), W, H,
            _lib.ptr(idx_), _lib.ptr(par_), _lib.ptr(ts_), _lib.ptr(kids_),
            _lib.ptr(m3_), _lib.ptr(sh_), _lib.ptr(col_), _lib.ptr(am_),
            _lib.ptr(sc_), _lib.ptr(op_), _lib.ptr(rot_), float(scale_modifier),
            _lib.ptr(cov_), _lib.ptr(vm_), _lib.ptr(pm_), _lib.ptr(cp_),
            float(tan_fovx), float(tan_fovy), _lib.ptr(rad_), float(H_VAR_BWD),
            _lib.ptr(geomBuffer), _lib.ptr(binningBuffer), _lib.ptr(imageBuffer),
            _lib.ptr(dpix_), _lib.ptr(dam_), _lib.ptr(dpl_), _lib.ptr(dinv_),
            _lib.ptr(dL_dmeans2D), _lib.ptr(dL_dopacity), _lib.ptr(dL_dcolors), _lib.ptr(dL_dmeans3D),
            _lib.ptr(dL_dcov3D), _lib.ptr(dL_dsh), _lib.ptr(dL_dscales), _lib.ptr(dL_drotations),
            _lib.ptr(dL_dall_map), int(bool(render_geo)), int(bool(debug)), _lib.stream_handle(dev))
        _lib.check(rc, "rasterize_gaussians_backward")
    return (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations,
            dL_dall_map)


def mark_visible(means3D, viewmatrix, projmatrix):
    """Frustum visibility mask, bool (P,).  Bound here; the reference's ext.cpp:15-17 lacks it."""
    _check_means(means3D)
    P = means3D.size(0)
    present = torch.zeros((P,), dtype=torch.bool, device=means3D.device)
    if P != 0:
        m3, vm, pm = means3D.contiguous(), viewmatrix.contiguous(), projmatrix.contiguous()
        dev = _lib.device_of(m3, vm, pm)
        rc = _lib.lib().hidegs_mark_visible(P, _lib.ptr(m3), _lib.ptr(vm), _lib.ptr(pm), _lib.ptr(present),
                                            _lib.stream_handle(dev))
        _lib.check(rc, "mark_visible")
    return present
