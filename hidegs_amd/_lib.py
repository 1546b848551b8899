"""ctypes binding of the C ABI in include/hidegs.h (hidegs_amd/libhidegs.so).

This is the only place that loads the native library.  It fails loudly: a missing
library raises ImportError-like RuntimeError at first use, and a non-zero return
code raises RuntimeError carrying hidegs_last_error(), the same exception type the
reference's torch extension surfaces (rasterize_points.cu:64-66, AT_ERROR).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  -- load torch's HIP runtime first; libhidegs binds to the same libamdhip64.so.7

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhidegs.so")

E_ARG, E_HIP, E_ALLOC, E_UNSUPPORTED = -1, -2, -3, -4

P = C.c_void_p
I = C.c_int
F = C.c_float
SZ = C.c_size_t

# hidegs_alloc_fn: char* (*)(void* user, size_t nbytes)   (round-1 header form)
ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_size_t)

# name -> (restype, argtypes); kept in the order of include/hidegs.h
SIGNATURES = {
    "hidegs_rasterize_forward": (I, [ALLOC_FN, ALLOC_FN, ALLOC_FN, P, I, I, I, P, I, I, P, P, P, P, P, P, P, P, P, P,
                                     F, P, P, P, P, P, F, F, I, P, P, P, P, P, I, P, I, P, P]),
    "hidegs_geometry_bytes": (SZ, [I]),
    "hidegs_binning_bytes": (SZ, [I]),
    "hidegs_image_bytes": (SZ, [I, I]),
    "hidegs_rasterize_backward": (I, [ALLOC_FN, P,                # scratch_buffer, alloc_user
                                      I, I, I, I,                 # P, D, M, R
                                      P, P, I, I,                 # background, all_map_pixels, width, height
                                      P, P, P, P,                 # indices, parent_indices, ts, kids
                                      P, P, P, P,                 # means3D, shs, colors_precomp, all_maps
                                      P, P, P, F,                 # scales, opacities, rotations, scale_modifier
                                      P, P, P, P,                 # cov3D_precomp, viewmatrix, projmatrix, campos
                                      F, F, P,                    # tan_fovx, tan_fovy, radii
                                      P, P, P,                    # geom, binning, image buffers
                                      P, P, P, P,                 # dL_dpix, dL_dout_all_map, dL_dplane, dL_dinvdepth
                                      P, P, P, P, P,              # dL_dmean2D, opacity, color, mean3D, cov3D
                                      P, P, P, P,                 # dL_dsh, dL_dscale, dL_drot, dL_dall_map
                                      I, I, P]),                  # render_geo, debug, stream
    "hidegs_mark_visible": (I, [I, P, P, P, P, P]),
    "hidegs_dist_cuda2": (I, [ALLOC_FN, P, I, P, P, P]),
    "hidegs_knn_scratch_bytes": (SZ, [I]),
    "hidegs_set_backward_hvar": (None, [F]),
    "hidegs_get_backward_hvar": (F, []),
    "hidegs_enable_stage_timing": (None, [I]),
    "hidegs_reset_stage_times": (None, []),
    "hidegs_stage_times": (I, [P, P]),
    "hidegs_stage_name": (C.c_char_p, [I]),
    "hidegs_last_error": (C.c_char_p, []),
    "hidegs_version": (C.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


def lib() -> C.CDLL:
    """Load libhidegs.so once; raise RuntimeError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} is missing: run `python -m hidegs_amd.build` "
                                   "(or __graft_entry__.build()) to compile it for gfx950")
            dll = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(dll, name)
                fn.restype = res
                fn.argtypes = args
            _lib = dll
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().hidegs_last_error().decode(errors="replace")
        kind = {E_ARG: "bad argument", E_HIP: "HIP error", E_ALLOC: "allocation failed",
                E_UNSUPPORTED: "unsupported"}.get(rc, f"error {rc}")
        raise RuntimeError(f"{what}: {kind}: {msg}")


def version() -> str:
    return lib().hidegs_version().decode()


def ptr(t) -> int:
    """Device pointer of a tensor, or NULL for None / empty tensors (B3: empty == absent)."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def current_stream_handle() -> int:
    """hipStream_t of PyTorch's current stream (B5), or NULL off-GPU."""
    if torch.cuda.is_available():
        return torch.cuda.current_stream().cuda_stream
    return None
