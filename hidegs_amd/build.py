"""Build recipe for hidegs_amd/libhidegs.so (the C-ABI library of include/hidegs.h).

Built in-tree with hipcc for gfx950 so the .so travels to the GPU box with the
repository snapshot.  `python -m hidegs_amd.build` or `__graft_entry__.build()`.
Each source is compiled to its own object (in parallel) and linked once; objects
are rebuilt only when the source or a header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(HERE, "..", "include")
OBJDIR = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libhidegs.so")
SOURCES = ["abi.cpp", "timing.cpp", "primitives.hip", "knn.hip", "adam.hip"]
HEADERS = [os.path.join(CSRC, "common.h"), os.path.join(CSRC, "block_scan.h"), os.path.join(INCLUDE, "hidegs.h")]

# -ffp-contract=off: every fused multiply-add in the kernels is an explicit fmaf, so the
# oracle (oracle/knn_ref.c) can reproduce each rounding step bit for bit.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
         "-Wno-unused-function", "-I", INCLUDE]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libhidegs.so")


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src, *HEADERS])


def _compile(src: str, verbose: bool) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if _stale(obj, src):
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        cmd = [hipcc(), *FLAGS, *lang, "-c", src, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    with cf.ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
