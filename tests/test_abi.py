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
