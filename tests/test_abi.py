"""The C-ABI library loads and exports exactly what include/hidegs.h declares (no compute calls)."""
import ctypes
import os
import re

import pytest

from hidegs_amd import _lib

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
    assert "hidegs_rasterize_forward" in fns and "hidegs_version" in fns
    assert len(fns) == 16


def test_every_header_symbol_exported(built_lib):
    for name in header_functions():
        assert hasattr(built_lib, name), name


def test_binding_arity_matches_header():
    fns = header_functions()
    assert set(fns) == set(_lib.SIGNATURES)
    for name, n in fns.items():
        assert len(_lib.SIGNATURES[name][1]) == n, name


def test_version_and_error_channel(built_lib):
    assert "hidegs" in _lib.version()
    # compute entry points report HIDEGS_E_UNSUPPORTED with a message; no device pointer is touched
    rc = built_lib.hidegs_mark_visible(0, None, None, None, None, None)
    assert rc == _lib.E_UNSUPPORTED
    assert b"not implemented" in built_lib.hidegs_last_error()
    with pytest.raises(RuntimeError, match="unsupported"):
        _lib.check(rc, "mark_visible")


def test_stage_timer_api(built_lib):
    ms = (ctypes.c_double * 12)()
    n = (ctypes.c_longlong * 12)()
    assert built_lib.hidegs_stage_times(ms, n) == 0
    assert list(ms) == [0.0] * 12
