"""The C-ABI library loads and exports exactly what include/hidegs.h declares, and its
host-side behaviour (argument validation, error channel, allocation-callback failure,
getHigherMsb) works without a GPU: no call here reaches a device."""
import ctypes
import os
import re

import pytest
import torch

from hidegs_amd import _lib
from oracle import binning

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "hidegs.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"^(?!typedef)[A-Za-z_][\w\s\*]*?\b(hidegs_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.M):
        name, params = m.group(1), m.group(2).strip()
        n = 0 if params in ("", "void") else len([p for p in params.split(",") if p.strip()])
        out[name] = n
    return out


def header_parameters():
    """{entry point: [parameter names in order]} from the prototypes of include/hidegs.h."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"^(?!typedef)[A-Za-z_][\w\s\*]*?\b(hidegs_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.M):
        params = m.group(2).strip()
        names = [] if params in ("", "void") else [re.findall(r"\w+", p)[-1] for p in params.split(",")]
        out[m.group(1)] = names
    return out


# The replaced interfaces' parameter names, in order: CudaRasterizer::Rasterizer::markVisible, ::forward and
# ::backward of the reference (submodules/hierarchy-rasterizer/cuda_rasterizer/rasterizer.h:24-29, 33-73, 75-117).
REFERENCE_PARAMETERS = {
    "hidegs_mark_visible": ["P", "means3D", "viewmatrix", "projmatrix", "present"],
    "hidegs_rasterize_forward": [
        "geometryBuffer", "binningBuffer", "imageBuffer", "P", "D", "M", "background", "width", "height", "indices",
        "parent_indices", "ts", "kids", "means3D", "shs", "colors_precomp", "all_map", "opacities", "scales",
        "scale_modifier", "rotations", "cov3D_precomp", "viewmatrix", "projmatrix", "cam_pos", "tan_fovx", "tan_fovy",
        "prefiltered", "out_color", "depth", "out_observe", "out_all_map", "out_plane_depth", "render_geo", "radii",
        "rects", "boxmin", "boxmax", "debug", "skyboxnum", "stream", "num_rendered", "biglimit", "on_cpu"],
    "hidegs_rasterize_backward": [
        "P", "D", "M", "R", "background", "all_map_pixels", "width", "height", "indices", "parent_indices", "ts",
        "kids", "means3D", "shs", "colors_precomp", "all_maps", "scales", "opacities", "rotations", "scale_modifier",
        "cov3D_precomp", "viewmatrix", "projmatrix", "campos", "tan_fovx", "tan_fovy", "radii", "geom_buffer",
        "binning_buffer", "image_buffer", "dL_dpix", "dL_dout_all_map", "dL_dout_plane_depth", "dL_invdepths",
        "dL_dmean2D", "dL_dconic", "dL_dopacity", "dL_dcolor", "dL_dinvdepth", "dL_dmean3D", "dL_dcov3D", "dL_dsh",
        "dL_dscale", "dL_drot", "dL_dall_map", "render_geo", "debug"],
}


def header_deltas():
    """[(entry point, kind, reference name, name here or None, meaning)] from the header's DELTA lines."""
    pat = re.compile(r"^\s*\*\s*DELTA (\w+) (dropped|added|renamed|retyped) (\w+)(?: -> (\w+))? : (.+)$", re.M)
    return [m.groups() for m in pat.finditer(open(HEADER).read())]


def test_abi_deltas_name_exactly_the_parameters_that_differ():
    """The header's DELTA block lists every parameter the ABI drops, adds or renames against
    rasterizer.h:24-118 -- no more, no fewer -- and the other parameters keep the reference's order."""
    ours, deltas = header_parameters(), header_deltas()
    assert {d[0] for d in deltas} == set(REFERENCE_PARAMETERS)
    for fn, ref in REFERENCE_PARAMETERS.items():
        mine = [d for d in deltas if d[0] == fn]
        renamed = {d[2]: d[3] for d in mine if d[1] == "renamed"}
        assert all(renamed.values()), f"{fn}: a rename names its new parameter"
        ref_here = [renamed.get(p, p) for p in ref]
        dropped = {d[2] for d in mine if d[1] == "dropped"}
        added = {d[2] for d in mine if d[1] == "added"}
        assert dropped == set(ref_here) - set(ours[fn]), fn
        assert added == set(ours[fn]) - set(ref_here), fn
        assert [p for p in ref_here if p not in dropped] == [p for p in ours[fn] if p not in added], \
            f"{fn}: the shared parameters are not in the reference's order"
        for d in mine:
            if d[1] == "retyped":
                assert d[2] in ours[fn], f"{fn}: retyped {d[2]} is not a parameter"
            assert len(d[4]) > 10, f"{fn} {d[2]}: no meaning given"
    by = lambda fn, kind: {d[2] for d in deltas if d[0] == fn and d[1] == kind}  # noqa: E731
    # the values the glue fixes (rasterize_points.cu:94,141-144; rasterizer.h:64-73,106,109)
    assert by("hidegs_rasterize_forward", "dropped") == {"rects", "boxmin", "boxmax", "skyboxnum", "biglimit", "on_cpu"}
    assert by("hidegs_rasterize_backward", "dropped") == {"dL_dconic", "dL_dinvdepth"}
    assert "h_var_bwd" in by("hidegs_rasterize_backward", "added")
    text = {d[2]: d[4] for d in deltas if d[0] == "hidegs_rasterize_forward"}
    assert "non-null" in text["rects"] and "NULL" in text["boxmin"] and "NULL" in text["boxmax"]
    assert "0" in text["skyboxnum"] and "INFINITY" in text["biglimit"] and "false" in text["on_cpu"]


def test_header_parses():
    fns = header_functions()
    assert {"hidegs_rasterize_forward", "hidegs_dist_cuda2", "hidegs_sort_pairs_u64", "hidegs_version"} <= set(fns)
    assert len(fns) == 28


def test_error_codes_match_header():
    """The HIDEGS_E_* codes of include/hidegs.h are the ones the binding maps to messages."""
    codes = {m.group(1): int(m.group(2)) for m in
             re.finditer(r"#define HIDEGS_E_(\w+)\s+\((-?\d+)\)", open(HEADER).read())}
    assert codes == {"ARG": _lib.E_ARG, "HIP": _lib.E_HIP, "ALLOC": _lib.E_ALLOC, "UNSUPPORTED": _lib.E_UNSUPPORTED,
                     "ASYNC": _lib.E_ASYNC}
    with pytest.raises(RuntimeError, match="earlier asynchronous failure"):
        _lib.check(_lib.E_ASYNC, "sort_tile_pairs")


def test_no_async_error_pending_without_a_device(built_lib):
    """No sort has run, so no asynchronous error word exists: entry points go on to validate their
    arguments (and hidegs_queue_error is the only reader that synchronises)."""
    assert built_lib.hidegs_inclusive_scan_u32(None, 0, None, None, 0, None) == 0


def test_every_header_symbol_exported(built_lib):
    for name in header_functions():
        assert hasattr(built_lib, name), name


def test_binding_arity_matches_header():
    fns = header_functions()
    assert set(fns) == set(_lib.SIGNATURES)
    for name, n in fns.items():
        assert len(_lib.SIGNATURES[name][1]) == n, name


def test_library_carries_gfx950_code(built_lib):
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data and b"radix_scatter_kernel" in data and b"knn_leaf_kernel" in data


def test_version_and_unbuilt_entry_points_fail_loudly(built_lib):
    assert "hidegs" in _lib.version()
    rc = built_lib.hidegs_mark_visible(0, None, None, None, None, None)
    assert rc == _lib.E_UNSUPPORTED
    assert b"not built" in built_lib.hidegs_last_error()
    with pytest.raises(RuntimeError, match="unsupported"):
        _lib.check(rc, "mark_visible")


def test_higher_msb_through_abi(built_lib):
    for n, bits in [(64, 7), (8160, 13), (32400, 15)]:
        assert built_lib.hidegs_higher_msb(n) == bits
    g = torch.Generator().manual_seed(0)
    samples = list(range(0, 70000)) + torch.randint(0, 2**31, (20000,), generator=g).tolist() + [2**32 - 1, 2**31]
    for n in samples:
        assert built_lib.hidegs_higher_msb(n) == binning.bit_length_at_least_one(n), n


def test_argument_validation_before_any_device_work(built_lib):
    dummy = ctypes.c_void_p(16)
    rc = built_lib.hidegs_sort_pairs_u64(dummy, 1 << 20, dummy, ctypes.c_void_p(32), dummy, ctypes.c_void_p(48),
                                         10, 0, 65, None)
    assert rc == _lib.E_ARG and b"bit range" in built_lib.hidegs_last_error()
    rc = built_lib.hidegs_sort_pairs_u64(None, 0, dummy, ctypes.c_void_p(32), dummy, ctypes.c_void_p(48), 10, 0, 8, None)
    assert rc == _lib.E_ARG and b"scratch" in built_lib.hidegs_last_error()
    rc = built_lib.hidegs_sort_pairs_u32(dummy, 1 << 20, dummy, dummy, dummy, ctypes.c_void_p(48), 10, 0, 8, None)
    assert rc == _lib.E_ARG and b"in-place" in built_lib.hidegs_last_error()
    rc = built_lib.hidegs_inclusive_scan_u32(None, 0, dummy, dummy, -1, None)
    assert rc == _lib.E_ARG
    rc = built_lib.hidegs_identify_tile_ranges(None, 5, None, 3, None)
    assert rc == _lib.E_ARG
    # n == 0 is a no-op everywhere
    assert built_lib.hidegs_sort_pairs_u64(None, 0, None, None, None, None, 0, 0, 64, None) == 0
    assert built_lib.hidegs_inclusive_scan_u32(None, 0, None, None, 0, None) == 0
    assert built_lib.hidegs_scan_scratch_bytes(0) == 0 and built_lib.hidegs_knn_scratch_bytes(0) == 0


def test_scratch_sizes_grow_with_n(built_lib):
    a, b = built_lib.hidegs_sort_pairs_u64_scratch_bytes(1000), built_lib.hidegs_sort_pairs_u64_scratch_bytes(10**6)
    assert 0 < a < b and b >= 12 * 10**6
    assert built_lib.hidegs_knn_scratch_bytes(2_000_000) > 50 * 2_000_000


def test_alloc_callback_invoked_once_and_failure_surfaces(built_lib):
    """distCUDA2 asks its scratch callback exactly once for hidegs_knn_scratch_bytes(P); a callback
    that fails (here: resize_ of a host tensor past a hard limit raises) returns NULL, the library
    reports HIDEGS_E_ALLOC before touching the device, and the Python exception is chained."""

    class Exploding(_lib.Scratch):
        def _alloc(self, user, nbytes):
            self.requests.append(int(nbytes))
            try:
                raise MemoryError(f"refusing {nbytes} bytes")
            except Exception as e:  # noqa: BLE001
                self.error = e
                return None

    s = Exploding("cpu")
    s.callback = _lib.ALLOC_FN(s._alloc)
    P = 1000
    rc = built_lib.hidegs_dist_cuda2(s.callback, None, P, ctypes.c_void_p(64), ctypes.c_void_p(128), None)
    assert rc == _lib.E_ALLOC
    assert s.requests == [built_lib.hidegs_knn_scratch_bytes(P)]
    with pytest.raises(RuntimeError, match="allocation failed") as ei:
        _lib.check_with(rc, "distCUDA2", s)
    assert isinstance(ei.value.__cause__, MemoryError)


def test_alloc_callback_resizes_tensor():
    s = _lib.Scratch("cpu")
    p = s.callback(None, 4096)
    assert p == s.tensor.data_ptr() and s.tensor.numel() == 4096 and s.requests == [4096]
