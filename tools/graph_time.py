"""Binning step (scan + sort_tile_pairs) eager vs captured in a hipGraph (torch.cuda.CUDAGraph)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import primitives, synthetic  # noqa: E402

wl = synthetic.binning_workload(2_000_000, 1920, 1080, seed=0, device="cuda")
offsets = torch.empty_like(wl.tiles_touched)
out = {}


def step():
    primitives.inclusive_scan_u32(wl.tiles_touched, out=offsets)
    out["r"] = primitives.sort_tile_pairs(wl.keys, wl.values, wl.num_tiles)


def timeit(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


eager = timeit(step)
ref = [t.clone() for t in out["r"]]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
graph = timeit(g.replay)
same = all(torch.equal(a, b) for a, b in zip(ref, out["r"]))
print(f"binning step eager {eager * 1e3:.1f} us, graph {graph * 1e3:.1f} us, same result {same}", flush=True)
