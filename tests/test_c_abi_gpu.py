"""The C ABI from C++ with no Python in between: tests/c_abi/abi_client (built by hidegs_amd/build.py) calls
hidegs_inclusive_scan_u32, hidegs_sort_tile_pairs, hidegs_dist_cuda2 (with a resize-functional allocation
callback) and the error channel the way the reference's C++ glue would, and checks every result itself
bit for bit (std::stable_sort of the same pairs, a brute force of distCUDA2's definition)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "tests", "c_abi", "abi_client")


def test_client_is_built_against_the_in_tree_library(built_lib):
    assert os.path.exists(CLIENT), "python -m hidegs_amd.build builds it"
    out = subprocess.run(["readelf", "-d", CLIENT], capture_output=True, text=True).stdout
    assert "libhidegs.so" in out and "$ORIGIN/../../hidegs_amd" in out


@pytest.mark.gpu
def test_cpp_client_runs_the_abi_bit_exact():
    out = subprocess.run([CLIENT], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ABI_CLIENT_OK" in out.stdout
    print(out.stdout)
