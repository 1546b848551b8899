"""Binning sort time on D2 views with hot tiles (synthetic.d2_scene's `cluster`), per kernel.

usage: python tools/skew_time.py [FRACTION:RADIUS ...]   (default: none, 0.05:0.1, 0.15:0.1, 0.3:0.05, 0.5:0.02)
Each line: tile-size profile of the view, whole hidegs_sort_tile_pairs (HIP events, median of 5 x 5
calls) and segment_sort / big_segments per call (library events), and a check of the result against
torch's stable sort of the same keys (values compared: equal keys keep input order).
Run against a variant with HIDEGS_LIB=variants/libhidegs_TAG.so (tools/build_variant.py).
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import _lib, primitives, synthetic  # noqa: E402


def main():
    specs = sys.argv[1:] or ["none", "0.05:0.1", "0.15:0.1", "0.3:0.05", "0.5:0.02"]
    cam = synthetic.d2_camera(1920, 1080)
    for spec in specs:
        cluster = None if spec == "none" else tuple(float(x) for x in spec.split(":"))
        sc = synthetic.d2_scene(2_000_000, cam, seed=1000, cluster=cluster)
        wl = synthetic.d2_binning_workload(sc, cam, device="cuda")
        T = wl.num_tiles
        counts = torch.bincount((wl.keys >> 32).long(), minlength=T)
        ko, vo, _ = primitives.sort_tile_pairs(wl.keys, wl.values, T)
        _, perm = torch.sort(wl.keys, stable=True)
        ok = bool(torch.equal(ko, wl.keys[perm]) and torch.equal(vo, wl.values[perm]))
        qerr = primitives.queue_error()
        times = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                primitives.sort_tile_pairs(wl.keys, wl.values, T)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / 5)
        with _lib.kernel_timer() as kt:
            for _ in range(5):
                primitives.sort_tile_pairs(wl.keys, wl.values, T)
            torch.cuda.synchronize()
            seg_ms, seg_n = kt.get("segment_sort")
            q_ms, q_n = kt.get("big_segments")
            sc_ms, sc_n = kt.get("radix_scatter_u64")
        print(f"{spec:>9}: K {wl.num_pairs:8d}  max tile {int(counts.max()):6d}  tiles >8192 {int((counts > 8192).sum()):3d}"
              f" >2048 {int((counts > 2048).sum()):3d}  sort {statistics.median(times):7.1f} us"
              f"  scatter {sc_ms * 1e3 / max(sc_n, 1):6.1f}  segment_sort {seg_ms * 1e3 / max(seg_n, 1):7.1f}"
              f"  big_segments {q_ms * 1e3 / max(q_n, 1):7.1f}"
              f"  {'bit-exact' if ok else 'MISMATCH'}  qerr {qerr}", flush=True)
        del sc, wl, counts, ko, vo, perm


if __name__ == "__main__":
    main()
