"""Build an experimental variant of libhidegs.so with extra compile definitions.

usage: python tools/build_variant.py TAG -DNAME=VALUE ...   ->  variants/libhidegs_TAG.so
Run a tool against it with HIDEGS_LIB=variants/libhidegs_TAG.so (hidegs_amd/_lib.py).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hidegs_amd import build as b  # noqa: E402


def main():
    tag, defs = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "variants")
    objdir = os.path.join(out, "obj_" + tag)
    os.makedirs(objdir, exist_ok=True)
    objs = []
    for src in b.SOURCES:
        obj = os.path.join(objdir, src + ".o")
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        subprocess.run([b.hipcc(), *b.FLAGS, *defs, *lang, "-c", os.path.join(b.CSRC, src), "-o", obj], check=True)
        objs.append(obj)
    lib = os.path.join(out, f"libhidegs_{tag}.so")
    subprocess.run([b.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", lib], check=True)
    print(lib)


if __name__ == "__main__":
    main()
