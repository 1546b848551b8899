"""Drop-in API surface of diff_gaussian_rasterization / simple_knn / gaussian_hierarchy (CPU).

Checks what the reference's Python layer and glue define without running a rasterizer:
the 18-field settings order (DGR/__init__.py:157-175), argument rules (:198-202), the
P == 0 early return with zero-filled outputs (rasterize_points.cu:75-100, 195-218), the
means3D shape error (:64-66) and that P > 0 surfaces the library's error instead of
falling back to any CPU path.
"""
import pytest
import torch

import diff_gaussian_rasterization as dgr
import gaussian_hierarchy
import simple_knn
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C

FIELDS = ("image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
          "sh_degree", "campos", "prefiltered", "debug", "render_indices", "parent_indices",
          "interpolation_weights", "num_node_kids", "do_depth", "render_geo")


def settings(H=32, W=48, do_depth=True, render_geo=True):
    e = torch.empty(0)
    return GaussianRasterizationSettings(H, W, 0.5, 0.5 * H / W, torch.zeros(3), 1.0, torch.eye(4), torch.eye(4), 3,
                                         torch.zeros(3), False, False, e.int(), e.int(), e.float(), e.int(),
                                         do_depth, render_geo)


def test_settings_field_order():
    assert GaussianRasterizationSettings._fields == FIELDS


def test_module_exports():
    assert {"GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_C"} <= set(dir(dgr))
    for name in ("rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible"):
        assert callable(getattr(_C, name))
    assert callable(simple_knn._C.distCUDA2)


@pytest.mark.parametrize("kw", [dict(), dict(shs=torch.zeros(1, 16, 3), colors_precomp=torch.zeros(1, 3))])
def test_exactly_one_color_source(kw):
    r = GaussianRasterizer(settings())
    m = torch.zeros(1, 3)
    with pytest.raises(Exception, match="SHs or precomputed colors"):
        r(m, m.clone(), torch.ones(1, 1), scales=torch.ones(1, 3), rotations=torch.ones(1, 4), **kw)


@pytest.mark.parametrize("kw", [dict(), dict(scales=torch.ones(1, 3)),
                                dict(scales=torch.ones(1, 3), rotations=torch.ones(1, 4), cov3D_precomp=torch.ones(1, 6))])
def test_exactly_one_covariance_source(kw):
    r = GaussianRasterizer(settings())
    m = torch.zeros(1, 3)
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m.clone(), torch.ones(1, 1), shs=torch.zeros(1, 16, 3), **kw)


def test_means3d_shape_error():
    s = settings()
    with pytest.raises(RuntimeError, match=r"means3D must have dimensions \(num_points, 3\)"):
        _C.rasterize_gaussians(s.bg, s.render_indices, s.parent_indices, s.interpolation_weights, s.num_node_kids,
                               torch.zeros(4, 2), torch.empty(0), torch.empty(0), torch.zeros(4, 1), torch.ones(4, 3),
                               torch.ones(4, 4), 1.0, torch.empty(0), s.viewmatrix, s.projmatrix, s.tanfovx,
                               s.tanfovy, s.image_height, s.image_width, torch.zeros(4, 16, 3), 3, s.campos, False,
                               True, False, True)


@pytest.mark.parametrize("do_depth,render_geo", [(True, True), (False, False)])
def test_zero_gaussians_forward_backward(do_depth, render_geo):
    """P == 0: no rasterizer call, zero outputs of the reference shapes, zero grads, autograd works."""
    s = settings(do_depth=do_depth, render_geo=render_geo)
    means3D = torch.zeros(0, 3, requires_grad=True)
    means2D = torch.zeros(0, 3, requires_grad=True)
    shs = torch.zeros(0, 16, 3, requires_grad=True)
    opac = torch.zeros(0, 1, requires_grad=True)
    scales = torch.zeros(0, 3, requires_grad=True)
    rots = torch.zeros(0, 4, requires_grad=True)
    color, radii, observe, all_map, plane, invdepth = GaussianRasterizer(s)(
        means3D, means2D, opac, shs=shs, scales=scales, rotations=rots, all_map=torch.zeros(0, 5))
    H, W = s.image_height, s.image_width
    assert color.shape == (3, H, W) and float(color.abs().sum()) == 0.0
    assert radii.shape == (0,) and radii.dtype == torch.int32
    assert observe.shape == (0,) and observe.dtype == torch.int32
    assert all_map.shape == (5, H, W) and plane.shape == (1, H, W)
    assert invdepth.shape == ((1 if do_depth else 0), H, W)
    (color.sum() + all_map.sum() + plane.sum() + invdepth.sum()).backward()
    for t, shape in ((means3D, (0, 3)), (means2D, (0, 3)), (shs, (0, 16, 3)), (opac, (0, 1)), (scales, (0, 3)),
                     (rots, (0, 4))):
        assert t.grad is not None and t.grad.shape == shape


def test_nonempty_forward_refuses_host_tensors(built_lib):
    """P > 0 host tensors are rejected before the C ABI: the kernels read device pointers, and
    there is no CPU fallback."""
    s = settings()
    P = 4
    with pytest.raises(RuntimeError, match="GPU tensor"):
        GaussianRasterizer(s)(torch.zeros(P, 3), torch.zeros(P, 3), torch.ones(P, 1), shs=torch.zeros(P, 16, 3),
                              scales=torch.ones(P, 3), rotations=torch.ones(P, 4), all_map=torch.zeros(P, 5))


def test_backward_glue_zero_rows_shapes():
    """P == 0 backward returns nine zero tensors with fullP rows in the reference order."""
    e = torch.empty(0)
    out = _C.rasterize_gaussians_backward(torch.zeros(3), torch.zeros(5, 8, 8), e.int(), e.int(), e.float(), e.int(),
                                          torch.zeros(0, 3), torch.zeros(0, dtype=torch.int32), e, torch.zeros(0, 5),
                                          torch.zeros(0, 1), torch.zeros(0, 3), torch.zeros(0, 4), 1.0, e,
                                          torch.eye(4), torch.eye(4), 0.5, 0.5, torch.zeros(3, 8, 8),
                                          torch.zeros(5, 8, 8), torch.zeros(1, 8, 8), torch.zeros(1, 8, 8),
                                          torch.zeros(0, 16, 3), 3, torch.zeros(3), torch.empty(0, dtype=torch.uint8),
                                          0, torch.empty(0, dtype=torch.uint8), torch.empty(0, dtype=torch.uint8),
                                          True, False)
    shapes = [(0, 3), (0, 3), (0, 1), (0, 3), (0, 6), (0, 16, 3), (0, 3), (0, 4), (0, 5)]
    assert [tuple(t.shape) for t in out] == shapes


def test_mark_visible_and_knn_empty():
    assert _C.mark_visible(torch.zeros(0, 3), torch.eye(4), torch.eye(4)).shape == (0,)
    assert simple_knn._C.distCUDA2(torch.zeros(0, 3)).shape == (0,)


def test_knn_nonempty_refuses_host_tensors(built_lib):
    with pytest.raises(RuntimeError, match="GPU tensor"):
        simple_knn._C.distCUDA2(torch.rand(8, 3))
    with pytest.raises(RuntimeError, match="dimensions"):
        simple_knn._C.distCUDA2(torch.rand(8, 2))


def test_backward_hvar_is_a_module_attribute_not_thread_state():
    """h_var of the covariance backward is read per call from _C.H_VAR_BWD (reference value 0.3,
    backward.cu:211), so a value set on the training thread reaches autograd's device thread."""
    import threading
    assert _C.H_VAR_BWD == 0.3
    seen = []
    old = _C.H_VAR_BWD
    try:
        _C.H_VAR_BWD = 0.1
        t = threading.Thread(target=lambda: seen.append(_C.H_VAR_BWD))
        t.start()
        t.join()
    finally:
        _C.H_VAR_BWD = old
    assert seen == [0.1]


def test_hierarchy_stub_raises():
    from gaussian_hierarchy._C import load_hierarchy, write_hierarchy  # scene/gaussian_model.py:24
    with pytest.raises(NotImplementedError):
        load_hierarchy("x.hier")
    with pytest.raises(NotImplementedError):
        write_hierarchy("x.hier")
    assert gaussian_hierarchy._C.expand_to_target is not None
