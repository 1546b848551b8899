"""Inclusive-scan time of the bench's tiles_touched (2M Gaussians, 1080p) and of 10M u32, HIP events,
median of 20 batches of 10 calls; checked against torch.cumsum (run against a variant library with
HIDEGS_LIB=variants/libhidegs_TAG.so)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib, primitives, synthetic  # noqa: E402

wl = synthetic.binning_workload(2_000_000, 1920, 1080, seed=0, device="cuda")
big = torch.randint(0, 64, (10_000_000,), dtype=torch.int32, device="cuda").view(torch.uint32)
for name, x in (("2M tiles_touched", wl.tiles_touched), ("10M u32", big)):
    out = torch.empty_like(x)
    primitives.inclusive_scan_u32(x, out=out)
    ref = torch.cumsum(x.view(torch.int32).to(torch.int64), 0).to(torch.int32)
    assert torch.equal(out.view(torch.int32), ref), name
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            primitives.inclusive_scan_u32(x, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 100.0)
    with _lib.kernel_timer() as kt:
        for _ in range(10):
            primitives.inclusive_scan_u32(x, out=out)
        torch.cuda.synchronize()
        r_ms, r_n = kt.get("scan_reduce")
        d_ms, d_n = kt.get("scan_downsweep")
    ts.sort()
    print(f"{name}: scan {ts[len(ts) // 2]:7.2f} us median  scan_reduce {r_ms * 1e3 / r_n:6.2f} us"
          f"  scan_downsweep {d_ms * 1e3 / d_n:6.2f} us", flush=True)
