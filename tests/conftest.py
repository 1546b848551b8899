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
            fields = line.rstrip("\n").split(maxsplit=5)
            path = fields[5] if len(fields) == 6 else ""
            deleted = path.endswith(" (deleted)")  # the file was replaced after it was mapped
            path = path[:-len(" (deleted)")] if deleted else path
            if path.startswith(root) and path.endswith(".so"):
                seen.add(os.path.relpath(path, root) + (" (replaced on disk after it was loaded)" if deleted else ""))
    with open(out, "w") as f:
        f.write("\n".join(sorted(seen)) + "\n")


def _on_gpu_box() -> bool:
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def built_lib():
    """The in-tree libhidegs.so.  Without a GPU (this container) it is built when missing or stale: hipcc
    cross-compiles.  On the GPU box it must already be there -- __graft_entry__.build() makes it on the
    CPU -- and is never rebuilt: a relink there would replace the library the earlier tests have loaded
    (and the box's copy of the tree may carry different file times)."""
    from hidegs_amd import _lib, build
    if not _on_gpu_box():
        build.build()
    elif not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} is missing: run __graft_entry__.build() on the CPU before the GPU tests")
    return _lib.lib()


@pytest.fixture(scope="session")
def oracle_lib():
    """The CPU oracle (test infrastructure), built by make when missing or stale -- here only; on the GPU
    box the prebuilt oracle/_build/liboracle.so is used as it is."""
    import oracle
    if not _on_gpu_box():
        oracle.build()
    return oracle
