"""Binning sort time when the pairs crowd into one or two tiles (the partition queue's extreme), next to
the bench view: python tools/extreme_time.py [N_PAIRS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib, primitives  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8_600_000
T = 8160
g = torch.Generator().manual_seed(0)
depth = (torch.rand(n, generator=g) * 99.8 + 0.2).view(torch.int32).long() & 0xFFFFFFFF
d2 = (torch.rand(n, generator=g) * 18 + 2).view(torch.int32).long() & 0xFFFFFFFF  # z in [2, 20] (the D2 range)
cases = {"uniform tiles": torch.randint(0, T, (n,), generator=g), "uniform, z 2-20": None,
         "one tile": torch.full((n,), 77),
         "two tiles": torch.where(torch.rand(n, generator=g) < 0.5, 5, 8000),
         "64 tiles": torch.randint(0, 64, (n,), generator=g) * 127}
vals = torch.arange(n, dtype=torch.int32).cuda()
from hidegs_amd import synthetic  # noqa: E402

cam = synthetic.d2_camera(1920, 1080)
for frac, rad in ((0.15, 0.1), (0.5, 0.02)):  # D2 hot-tile views with depths widened to [0.2, 100]
    wl = synthetic.d2_binning_workload(synthetic.d2_scene(2_000_000, cam, seed=1000, cluster=(frac, rad)), cam)
    zg = (torch.rand(2_000_000, generator=g) * 99.8 + 0.2).view(torch.int32).long() & 0xFFFFFFFF
    cases[f"D2 {frac}:{rad} z.2-100"] = ((wl.keys >> 32) << 32) | zg[wl.values.long()]
for name, tiles in cases.items():
    if name.startswith("D2 "):
        keys = tiles.cuda()
        vals_c = torch.arange(keys.numel(), dtype=torch.int32).cuda()
    elif tiles is None:
        keys = ((cases["uniform tiles"].long() << 32) | d2).cuda()
    else:
        keys = ((tiles.long() << 32) | depth).cuda()
    if not name.startswith("D2 "):
        vals_c = vals
    for _ in range(2):
        primitives.sort_tile_pairs(keys, vals_c, T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        primitives.sort_tile_pairs(keys, vals_c, T)
    e1.record()
    torch.cuda.synchronize()
    with _lib.kernel_timer() as kt:
        primitives.sort_tile_pairs(keys, vals_c, T)
        torch.cuda.synchronize()
        per = {k: round(kt.get(k)[0] * 1e3, 1) for k in ("radix_hist_u64", "radix_digit_scan", "radix_scatter_u64",
                                                           "segment_sort", "big_segments")}
    print(f"{name:14s} n={keys.numel()}: sort {e0.elapsed_time(e1) * 1e3 / 5:8.1f} us  {per}  qerr {primitives.queue_error()}",
          flush=True)
