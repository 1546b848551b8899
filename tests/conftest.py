import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


def pytest_collection_modifyitems(config, items):
    """Without a GPU the gpu-marked tests are skipped, so a plain `pytest` stays green here."""
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this process (run with -m gpu on the MI355X box)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def pytest_sessionfinish(session, exitstatus):
    """With HIDEGS_MAPS_OUT set (tools/gpu_round6.sh), list the in-tree shared objects this
    test process mapped -- the native code the run actually used (profiles/r06_evidence.md)."""
    out = os.environ.get("HIDEGS_MAPS_OUT")
    if not out:
        return
    root, seen = os.path.realpath(ROOT), set()
    with open(f"/proc/{os.getpid()}/maps") as f:
        for line in f:
            path = line.split()[-1] if len(line.split()) >= 6 else ""
            if path.startswith(root) and path.endswith(".so"):
                seen.add(os.path.relpath(path, root))
    with open(out, "w") as f:
        f.write("\n".join(sorted(seen)) + "\n")


@pytest.fixture(scope="session")
def built_lib():
    """Build libhidegs.so in-tree if it is missing or stale (hipcc cross-compiles without a GPU)."""
    from hidegs_amd import _lib, build
    build.build()
    return _lib.lib()


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle
