"""Per-job timeline of the per-tile sort's partition queue for one hot tile (experiments only).

Needs a library built with -DHIDEGS_QUEUE_TRACE:
    python tools/build_variant.py qtrace -DHIDEGS_QUEUE_TRACE=1
    HIDEGS_LIB=variants/libhidegs_qtrace.so python tools/queue_trace.py [hot_pairs ...]
Times are wall_clock64 ticks (100 MHz) relative to the first claim, in microseconds."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hidegs_amd import _lib, primitives, synthetic  # noqa: E402

NAMES = {1: "SMALL", 2: "COPY", 3: "REDUCE", 4: "HIST", 5: "SCATTER", 6: "GLOBAL", 7: "WIDE"}
L = _lib.lib()
fn = L.hidegs_debug_queue_trace
fn.restype = C.c_int
fn.argtypes = [C.c_void_p, C.c_int]
wfn = L.hidegs_debug_wide_trace
wfn.restype = C.c_int
wfn.argtypes = [C.c_void_p, C.c_int]
wbuf = np.zeros((4096, 9), np.uint64)
WPHASES = ["load+copy", "and/or", "bucket hist", "scan", "fill", "rank", "(lsd)", "gather"]

CAP = 32768
buf = np.zeros((CAP, 4), np.uint64)
cam = synthetic.d2_camera(1920, 1080)
for spec in sys.argv[1:] or ["4096", "100000", "skew:0.15:0.1", "skew:0.5:0.02"]:
    if spec.startswith("skew:"):  # a D2 view with a fraction of the Gaussians in a disc (tools/skew_time.py)
        frac, rad = (float(x) for x in spec.split(":")[1:])
        wl = synthetic.d2_binning_workload(synthetic.d2_scene(2_000_000, cam, seed=1000, cluster=(frac, rad)), cam,
                                           device="cuda")
        keys, hot = wl.keys, spec
    else:  # `hot` pairs of round 3's synthetic keys moved into tile 4000
        wl = synthetic.binning_workload(2_000_000, 1920, 1080, seed=0, device="cuda")
        hot = int(spec)
        keys = wl.keys.clone()
        idx = torch.randperm(keys.numel(), device="cuda")[:hot]
        keys[idx] = (keys[idx] & 0xFFFFFFFF) | (4000 << 32)
    primitives.sort_tile_pairs(keys, wl.values, wl.num_tiles)
    torch.cuda.synchronize()
    fn(buf.ctypes.data, CAP)  # drop the warm-up's trace
    wfn(wbuf.ctypes.data, 4096)
    primitives.sort_tile_pairs(keys, wl.values, wl.num_tiles)
    n = fn(buf.ctypes.data, CAP)
    nw = wfn(wbuf.ctypes.data, 4096)
    if nw > 0:
        wt = wbuf[:nw].astype(np.int64)
        ok = (wt[:, 1:] > 0).all(axis=1)  # jobs that took every stamp (the bucket form and the gather)
        d = np.diff(wt[ok, 1:], axis=1) / 100.0
        print(f"  WIDE phases over {int(ok.sum())} of {nw} jobs (m p50 {int(np.median(wt[:, 0]))}), p50 us: " +
              ", ".join(f"{nm} {np.median(d[:, k]):.1f}" for k, nm in enumerate(WPHASES[1:])) +
              f"; load+copy {np.median(np.diff(wt[ok, 1:3], axis=1)) / 100.0:.1f}" if ok.any() else "")
    tr = buf[:n].copy()
    t0 = tr[:, 1].min()
    rel = (tr[:, 1:].astype(np.int64) - int(t0)) / 100.0
    order = np.argsort(rel[:, 1])
    print(f"hot tile {hot}: {n} jobs, last end {rel[:, 2].max():.1f} us")
    kinds = {}
    for j in order:
        ty = int(tr[j, 0] & 0x7F)
        last = " last" if tr[j, 0] & 0x80 else ""
        kinds.setdefault(NAMES.get(ty, ty) + last, []).append(rel[j, 2] - rel[j, 1])
    for k, v in kinds.items():
        print(f"  {k:13s} x{len(v):4d}: run p50 {np.median(v):7.1f}  p90 {np.percentile(v, 90):7.1f}  max {np.max(v):7.1f} us")
    wait = rel[:, 1] - rel[:, 0]
    print(f"  claim->got wait p50 {np.median(wait):.1f} us; jobs started per 20 us:",
          np.histogram(rel[:, 1], bins=np.arange(0, rel[:, 2].max() + 20, 20))[0].tolist())
    show = order[:12] if len(order) < 60 else np.argsort(-(rel[:, 2] - rel[:, 1]))[:15]
    for j in show:
        ty = int(tr[j, 0] & 0x7F)
        print(f"  job {int(tr[j, 0] >> 32):5d} {NAMES.get(ty, ty):8s}{'*' if tr[j, 0] & 0x80 else ' '} block "
              f"{int((tr[j, 0] >> 8) & 0xFFFFFF):4d}  claimed {rel[j, 0]:8.1f}  got {rel[j, 1]:8.1f}  end {rel[j, 2]:8.1f}")
