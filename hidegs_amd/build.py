"""Build recipe for hidegs_amd/libhidegs.so (the C-ABI library of include/hidegs.h).

Built in-tree with hipcc for gfx950 so the .so travels to the GPU box with the
repository snapshot.  `python -m hidegs_amd.build` or `__graft_entry__.build()`.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhidegs.so")
SOURCES = ["abi_stub.cpp"]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libhidegs.so")


def build(verbose: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    tmp = LIB + ".tmp"
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(HERE, "..", "include"), *srcs, "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
