"""Build recipe for hidegs_amd/libhidegs.so (the C-ABI library of include/hidegs.h).

Built in-tree with hipcc for gfx950 so the .so travels to the GPU box with the
repository snapshot.  `python -m hidegs_amd.build` or `__graft_entry__.build()`.
Each source is compiled to its own object (in parallel) and linked once.  An object is
rebuilt when its source or a header is newer, or when its compile command (flags and
-D knobs) differs from the one recorded in its stamp file.

Test variants (VARIANTS) are the same library built with extra -D knobs into
hidegs_amd/variants/libhidegs_<tag>.so; the GPU tests load them to drive error paths
that the product build cannot reach (e.g. a tiny partition-queue job capacity).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(HERE, "..", "include")
OBJDIR = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libhidegs.so")
VARIANT_DIR = os.path.join(HERE, "variants")
SOURCES = ["abi.cpp", "timing.cpp", "primitives.hip", "knn.hip", "adam.hip", "wire.hip"]
HEADERS = [os.path.join(CSRC, "common.h"), os.path.join(CSRC, "block_scan.h"), os.path.join(INCLUDE, "hidegs.h")]

# -ffp-contract=off: every fused multiply-add in the kernels is an explicit fmaf, so the
# oracle (oracle/knn_ref.c) can reproduce each rounding step bit for bit.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
         "-Wno-unused-function", "-I", INCLUDE]

# tag -> (extra defines, the sources they change); the other objects are shared with the product build
VARIANTS = {
    # partition-queue overflow -> error word; its starved workers give up after 2^16 polls (~0.2 s), not ~13 s
    "qcap": (["-DHIDEGS_JOB_CAP=64", "-DHIDEGS_MAX_POLLS=65536u"], ["primitives.hip"]),
    "gform": (["-DHIDEGS_QUEUE_MIN=8192"], ["primitives.hip"]),  # tiles of 2049..8192 pairs: one-workgroup global form
    "wscout": (["-DHIDEGS_WIDE_SCOUTS=1"], ["primitives.hip"]),  # hot tiles <= 12288 pairs as WIDE jobs (in place)
    "pcap": (["-DHIDEGS_PIECE_CAP=16"], ["primitives.hip"]),  # piece list full after 16: the rest as SMALL jobs
}


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libhidegs.so")


def _command(src: str, obj: str, defines) -> list:
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    return [hipcc(), *FLAGS, *defines, *lang, "-c", src, "-o", obj + ".tmp"]


def _stamp(cmd: list) -> str:
    # the command without the tool path and the output name: flags, knobs and the source
    return hashlib.sha256(" ".join(cmd[1:-2]).encode()).hexdigest()


def _stale(obj: str, src: str, stamp: str) -> bool:
    if not os.path.exists(obj) or not os.path.exists(obj + ".cmd"):
        return True
    with open(obj + ".cmd") as f:
        if f.read().strip() != stamp:
            return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src, *HEADERS])


def _compile(src: str, objdir: str, defines, verbose: bool) -> str:
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    cmd = _command(src, obj, defines)
    stamp = _stamp(cmd)
    if _stale(obj, src, stamp):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        with open(obj + ".cmd", "w") as f:
            f.write(stamp + "\n")
    return obj


def _link(objs, lib: str, verbose: bool) -> str:
    if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        tmp = lib + ".tmp"
        cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, lib)
    return lib


ABI_CLIENT_SRC = os.path.join(HERE, "..", "tests", "c_abi", "abi_client.cpp")
ABI_CLIENT = os.path.join(HERE, "..", "tests", "c_abi", "abi_client")


def build_abi_client(verbose: bool = False) -> str:
    """tests/c_abi/abi_client: a C++ program calling the ABI with no Python (test infrastructure, run on the
    GPU by tests/test_c_abi_gpu.py), linked against the in-tree library with an $ORIGIN-relative rpath."""
    deps = [ABI_CLIENT_SRC, LIB, os.path.join(INCLUDE, "hidegs.h")]
    if not os.path.exists(ABI_CLIENT) or any(os.path.getmtime(d) > os.path.getmtime(ABI_CLIENT) for d in deps):
        tmp = ABI_CLIENT + ".tmp"
        cmd = [hipcc(), "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off", "-Wall", ABI_CLIENT_SRC,
               "-L" + HERE, "-lhidegs", "-Wl,-rpath,$ORIGIN/../../hidegs_amd", "-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, ABI_CLIENT)
    return ABI_CLIENT


def variant_path(tag: str) -> str:
    return os.path.join(VARIANT_DIR, f"libhidegs_{tag}.so")


def build(verbose: bool = False, variants: bool = True) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    jobs = [(s, OBJDIR, []) for s in srcs]
    if variants:
        for tag, (defs, changed) in VARIANTS.items():
            vdir = os.path.join(VARIANT_DIR, "obj_" + tag)
            os.makedirs(vdir, exist_ok=True)
            jobs += [(os.path.join(CSRC, s), vdir, defs) for s in changed]
    with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
        objs = list(ex.map(lambda j: _compile(j[0], j[1], j[2], verbose), jobs))
    base = objs[:len(srcs)]
    _link(base, LIB, verbose)
    if variants:
        k = len(srcs)
        for tag, (defs, changed) in VARIANTS.items():
            own = dict(zip(changed, objs[k:k + len(changed)]))
            k += len(changed)
            _link([own.get(s, o) for s, o in zip(SOURCES, base)], variant_path(tag), verbose)
        build_abi_client(verbose)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
