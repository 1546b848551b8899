"""The partition queue's hand-offs in the generated gfx950 code (CPU: hipcc cross-compiles).

Every agent-scope release (`buffer_wbl2`) must be followed by `s_waitcnt vmcnt(0)` before the tag
store or countdown that publishes it: ROCm 7.2 may drop its own wait there, and the count then
overtakes the write-back ("Hand-offs, round 4").  release_lane() adds an inline-asm wait
the pass cannot remove; this checks the result in the assembly of every kernel of primitives.hip.
"""
import os
import re
import subprocess

import pytest

from hidegs_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hidegs_amd", "csrc", "primitives.hip")


def _have_hipcc() -> bool:
    try:
        build.hipcc()
        return True
    except RuntimeError:
        return False


@pytest.mark.skipif(not _have_hipcc(), reason="hipcc not available")
def test_every_l2_writeback_is_waited_for(tmp_path):
    out = str(tmp_path / "primitives.s")
    cmd = [c for c in build._command(SRC, out, []) if c != "-c"]
    cmd[cmd.index("-o") + 1] = out
    cmd += ["-S", "--offload-device-only"]
    subprocess.run(cmd, check=True, capture_output=True)
    lines = open(out).read().splitlines()
    fn, seen, bad = None, 0, []
    for k, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            fn = m.group(1)
        if "buffer_wbl2" in ln and not ln.lstrip().startswith(";"):
            seen += 1
            nxt = [x.strip() for x in lines[k + 1:k + 3]]
            if not any(x.startswith("s_waitcnt vmcnt(0)") for x in nxt):
                bad.append((fn, k + 1, nxt))
    assert seen >= 2, "the queue kernels' release fences were not found"
    assert not bad, bad
