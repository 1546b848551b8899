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

# HIDEGS_LIB selects another build of the same ABI (tools/build_variant.py experiments)
LIB_PATH = os.environ.get("HIDEGS_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhidegs.so")

E_ARG, E_HIP, E_ALLOC, E_UNSUPPORTED, E_ASYNC = -1, -2, -3, -4, -5

P = C.c_void_p
I = C.c_int
F = C.c_float
SZ = C.c_size_t

# hidegs_alloc_fn: char* (*)(void* user, size_t nbytes)
ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_size_t)
LL = C.c_longlong


class AdamTensor(C.Structure):
    """hidegs_adam_tensor (include/hidegs.h)."""
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("relevant", C.c_void_p), ("rows", C.c_longlong), ("width", C.c_int), ("lr", C.c_double),
                ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_double), ("weight_decay", C.c_double),
                ("step", C.c_longlong)]
U32 = C.c_uint32

# name -> (restype, argtypes); kept in the order of include/hidegs.h
SIGNATURES = {
    "hidegs_rasterize_forward": (I, [ALLOC_FN, ALLOC_FN, ALLOC_FN, P, I, I, I, P, I, I, P, P, P, P, P, P, P, P, P, P,
                                     F, P, P, P, P, P, F, F, I, P, P, P, P, P, I, P, I, P, P]),
    "hidegs_rasterize_backward": (I, [I, I, I, I,                 # P, D, M, R
                                      P, P, I, I,                 # background, all_map_pixels, width, height
                                      P, P, P, P,                 # indices, parent_indices, ts, kids
                                      P, P, P, P,                 # means3D, shs, colors_precomp, all_maps
                                      P, P, P, F,                 # scales, opacities, rotations, scale_modifier
                                      P, P, P, P,                 # cov3D_precomp, viewmatrix, projmatrix, campos
                                      F, F, P, F,                 # tan_fovx, tan_fovy, radii, h_var_bwd
                                      P, P, P,                    # geom, binning, image buffers
                                      P, P, P, P,                 # dL_dpix, dL_dout_all_map, dL_dplane, dL_invdepths
                                      P, P, P, P, P,              # dL_dmean2D, opacity, color, mean3D, cov3D
                                      P, P, P, P,                 # dL_dsh, dL_dscale, dL_drot, dL_dall_map
                                      I, I, P]),                  # render_geo, debug, stream
    "hidegs_mark_visible": (I, [I, P, P, P, P, P]),
    "hidegs_dist_cuda2": (I, [ALLOC_FN, P, I, P, P, P]),
    "hidegs_knn_scratch_bytes": (SZ, [I]),
    "hidegs_scan_scratch_bytes": (SZ, [LL]),
    "hidegs_inclusive_scan_u32": (I, [P, SZ, P, P, LL, P]),
    "hidegs_sort_pairs_u64_scratch_bytes": (SZ, [LL]),
    "hidegs_sort_pairs_u64": (I, [P, SZ, P, P, P, P, LL, I, I, P]),
    "hidegs_sort_pairs_u32_scratch_bytes": (SZ, [LL]),
    "hidegs_sort_pairs_u32": (I, [P, SZ, P, P, P, P, LL, I, I, P]),
    "hidegs_identify_tile_ranges": (I, [P, LL, P, I, P]),
    "hidegs_sort_tile_pairs": (I, [P, SZ, P, P, P, P, LL, I, P, P]),
    "hidegs_queue_error": (I, [P, I, P]),
    "hidegs_set_debug": (None, [I]),
    "hidegs_higher_msb": (U32, [U32]),
    "hidegs_masked_adam": (I, [P, P, P, P, P, LL, I, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                LL, P]),
    "hidegs_masked_adam_multi": (I, [P, I, P]),
    "hidegs_bf16_pack": (I, [P, P, LL, LL, P]),
    "hidegs_bf16_sum_ranks": (I, [P, I, LL, P, P]),
    "hidegs_bf16_unpack": (I, [P, P, LL, P]),
    "hidegs_mask_pack": (I, [P, LL, P, P]),
    "hidegs_mask_union_count": (I, [P, I, LL, P, P, P]),
    "hidegs_kernel_timing": (None, [I]),
    "hidegs_kernel_timing_reset": (None, []),
    "hidegs_kernel_time": (I, [C.c_char_p, P, P]),
    "hidegs_last_error": (C.c_char_p, []),
    "hidegs_version": (C.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


def load_library(path: str) -> C.CDLL:
    """A build of the ABI at `path` with every signature of include/hidegs.h bound (lib() for the
    product build; tests load the build.VARIANTS this way)."""
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run `python -m hidegs_amd.build` "
                           "(or __graft_entry__.build()) to compile it for gfx950")
    dll = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(dll, name)
        fn.restype = res
        fn.argtypes = args
    return dll


def lib() -> C.CDLL:
    """Load libhidegs.so once; raise RuntimeError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = load_library(LIB_PATH)
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().hidegs_last_error().decode(errors="replace")
        kind = {E_ARG: "bad argument", E_HIP: "HIP error", E_ALLOC: "allocation failed",
                E_UNSUPPORTED: "unsupported", E_ASYNC: "earlier asynchronous failure"}.get(rc, f"error {rc}")
        raise RuntimeError(f"{what}: {kind}: {msg}")


def version() -> str:
    return lib().hidegs_version().decode()


def ptr(t) -> int:
    """Device pointer of a tensor, or NULL for None / empty tensors (B3: empty == absent)."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def device_of(*tensors) -> torch.device:
    """The one CUDA device all given (non-empty) tensors live on; raises otherwise.

    Kernels dereference these pointers on that device, so a host tensor or a tensor on
    another GPU must be rejected here rather than handed to the C side."""
    dev = None
    for t in tensors:
        if t is None or t.numel() == 0:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(f"expected a GPU tensor, got one on {t.device}")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} and {t.device}")
    if dev is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def stream_handle(device: torch.device) -> int:
    """hipStream_t of PyTorch's current stream on `device` (B5)."""
    return torch.cuda.current_stream(device).cuda_stream


class Scratch:
    """A uint8 device tensor the C side grows through an hidegs_alloc_fn callback.

    The C form of the reference's resizeFunctional (rasterize_points.cu:27-33): the
    callback resizes the tensor and returns its data pointer.  An exception inside the
    callback must not unwind through the C frame, so it is stored, NULL is returned
    (the library then reports HIDEGS_E_ALLOC) and `check` re-raises it as the cause.
    """

    def __init__(self, device, tensor=None):
        self.tensor = tensor if tensor is not None else torch.empty((0,), dtype=torch.uint8, device=device)
        self.requests = []
        self.error = None
        self.callback = ALLOC_FN(self._alloc)

    def _alloc(self, _user, nbytes):
        self.requests.append(int(nbytes))
        try:
            self.tensor.resize_(int(nbytes))
            return self.tensor.data_ptr() if nbytes else None
        except Exception as e:  # noqa: BLE001 -- reported through check()
            self.error = e
            return None


def check_with(rc: int, what: str, *scratches: "Scratch") -> None:
    """check() that chains a Python exception raised inside an allocation callback."""
    if rc == 0:
        return
    cause = next((s.error for s in scratches if s is not None and s.error is not None), None)
    try:
        check(rc, what)
    except RuntimeError as e:
        if cause is not None:
            raise e from cause
        raise


class kernel_timer:
    """Context manager: per-kernel device times (ms, launches) of this library's kernels.

    with kernel_timer() as kt: ...;  kt.get("radix_scatter_u64") -> (total_ms, launches)
    """

    def __enter__(self):
        lib().hidegs_kernel_timing_reset()
        lib().hidegs_kernel_timing(1)
        return self

    def __exit__(self, *exc):
        lib().hidegs_kernel_timing(0)
        return False

    @staticmethod
    def get(name: str):
        ms, n = C.c_double(0.0), C.c_longlong(0)
        lib().hidegs_kernel_time(name.encode(), C.byref(ms), C.byref(n))
        return ms.value, n.value
