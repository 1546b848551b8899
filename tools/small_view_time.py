"""The binning step of a small view (config 2: 100k D2 Gaussians, 1080p): whole-step HIP-event time and
per-kernel device time from a rocprofv3 kernel trace (run under rocprofv3) or the library's own timer.
usage: python tools/small_view_time.py [n_gaussians]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib, primitives, synthetic  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
cam = synthetic.d2_camera()
wl = synthetic.d2_binning_workload(synthetic.d2_scene(N, cam, seed=0), cam, device="cuda")
off = torch.empty_like(wl.tiles_touched)


def step():
    primitives.inclusive_scan_u32(wl.tiles_touched, out=off)
    primitives.sort_tile_pairs(wl.keys, wl.values, wl.num_tiles)


for _ in range(10):
    step()
ts = []
for _ in range(50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    step()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
print(f"N={N} pairs={wl.num_pairs}: step median {statistics.median(ts):.1f} us (min {min(ts):.1f})", flush=True)
ts = []
for _ in range(50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        step()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / 10)
print(f"back to back: {statistics.median(ts):.1f} us per step", flush=True)

# the same step captured once into a hipGraph and replayed (launch latency off the critical path)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
for _ in range(10):
    g.replay()
ts = []
for _ in range(50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / 10)
print(f"graph replay, back to back: {statistics.median(ts):.1f} us per step", flush=True)
