"""Randomised stress of hidegs_sort_tile_pairs' hot-tile paths (scouts, partition queue, WIDE jobs,
deferred pieces): many random skewed views and injected hot tiles, each result compared with torch's
stable sort of the same keys on the GPU (equal keys keep input order), the queue's error word clear.

usage: python tools/queue_stress.py [SECONDS] [SEED]   (prints one line per case, FAIL lines on mismatch)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hidegs_amd import primitives, synthetic  # noqa: E402


def case_keys(g, cam, i):
    kind = i % 3
    if kind == 0:  # a D2 view with a disc of Gaussians
        n = int(torch.randint(200_000, 2_000_001, (1,), generator=g))
        frac = float(torch.rand(1, generator=g)) * 0.9
        rad = 0.005 + float(torch.rand(1, generator=g)) * 0.2
        wl = synthetic.d2_binning_workload(synthetic.d2_scene(n, cam, seed=int(torch.randint(0, 1 << 30, (1,), generator=g)),
                                                              cluster=(frac, rad)), cam, device="cuda")
        return wl.keys, wl.values, wl.num_tiles, f"D2 n={n} cluster=({frac:.2f},{rad:.3f})"
    T = 8160
    k = int(torch.randint(100_000, 6_000_001, (1,), generator=g))
    tiles = torch.randint(0, T, (k,), generator=g)
    if kind == 1:  # hot tiles of random sizes injected into uniform keys
        nhot = int(torch.randint(1, 65, (1,), generator=g))
        hot = torch.randint(0, T, (nhot,), generator=g)
        share = float(torch.rand(1, generator=g))
        pick = torch.rand(k, generator=g) < share
        tiles[pick] = hot[torch.randint(0, nhot, (int(pick.sum()),), generator=g)]
        desc = f"inject k={k} hot={nhot} share={share:.2f}"
    else:  # few distinct depths (ties everywhere) and a narrow or wide depth range
        desc = f"ties k={k}"
    lo, hi = sorted((0.2 + 99.8 * torch.rand(2, generator=g)).tolist())
    depth = lo + (hi - lo) * torch.rand(k, generator=g)
    if kind == 2:
        depth = torch.round(depth * 4) / 4
        tiles[: k // 2] = int(torch.randint(0, T, (1,), generator=g))
    keys = (tiles.to(torch.int64) << 32) | depth.view(torch.int32).to(torch.int64)
    vals = torch.arange(k, dtype=torch.int32)
    return keys.cuda(), vals.cuda(), T, desc + f" depth=[{lo:.1f},{hi:.1f}]"


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    g = torch.Generator().manual_seed(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    cam = synthetic.d2_camera(1920, 1080)
    t0, i, fails = time.time(), 0, 0
    primitives.queue_error()
    while time.time() - t0 < budget:
        keys, vals, T, desc = case_keys(g, cam, i)
        _, perm = torch.sort(keys, stable=True)
        ko, vo, _ = primitives.sort_tile_pairs(keys, vals, T)
        ok = bool(torch.equal(ko, keys[perm]) and torch.equal(vo, vals[perm]))
        qerr = primitives.queue_error()
        if not ok or qerr:
            fails += 1
        print(f"{'ok  ' if ok and not qerr else 'FAIL'} case {i}: {desc} qerr {qerr}", flush=True)
        i += 1
        del keys, vals, ko, vo, perm
    print(f"{i} cases, {fails} failures", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
