"""Randomised parity stress of distCUDA2 (csrc/knn.hip) against the CPU oracle (oracle/knn_ref.c, OpenMP brute
force): random point-set shapes and sizes, every result compared bit for bit (uint32 patterns, inf included).

Shapes: uniform boxes at random scales and far offsets (coarse float spacing: many exact ties), Gaussian
blobs of mixed widths, planes and lines (degenerate boxes), integer lattices (ties everywhere), duplicated
points, far outliers, a dense core inside a sparse shell, and the D2 frustum.  Sizes are log-uniform in
[1, 60000] with every point checked; one case in eight is 200K-2M points with 2048 sampled queries checked
against all points.

usage: python tools/knn_stress.py [SECONDS] [SEED]   (one line per case, FAIL lines on mismatch)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import oracle  # noqa: E402  -- test infrastructure: the checker, never the thing measured
import simple_knn  # noqa: E402

SHAPES = ("box", "blobs", "plane", "line", "lattice", "duplicates", "outliers", "core_shell", "frustum")


def make(g, shape, n):
    if shape == "box":
        scale = 10.0 ** g.uniform(-3, 3)
        off = 10.0 ** g.uniform(0, 5) * g.choice([-1, 1], 3)
        return (g.random((n, 3)) * scale + off).astype(np.float32)
    if shape == "blobs":
        k = int(g.integers(1, 40))
        centres = g.uniform(-100, 100, (k, 3))
        sig = 10.0 ** g.uniform(-3, 1, k)
        lab = g.integers(0, k, n)
        return (centres[lab] + g.normal(size=(n, 3)) * sig[lab, None]).astype(np.float32)
    if shape == "plane":
        p = np.c_[g.uniform(-10, 10, (n, 2)), np.full(n, g.uniform(-5, 5))]
        return p[:, g.permutation(3)].astype(np.float32)
    if shape == "line":
        t = g.uniform(-10, 10, n)
        d = g.normal(size=3)
        return (t[:, None] * d / np.linalg.norm(d)).astype(np.float32)
    if shape == "lattice":
        side = max(1, int(round(n ** (1 / 3))) + 1)
        grid = np.stack(np.meshgrid(*[np.arange(side)] * 3), -1).reshape(-1, 3)
        return (grid[g.choice(grid.shape[0], min(n, grid.shape[0]), replace=False)] * g.uniform(0.1, 3)).astype(np.float32)
    if shape == "duplicates":
        base = g.random((max(1, n // 2), 3)).astype(np.float32)
        return np.concatenate([base, base[g.integers(0, base.shape[0], n - base.shape[0])]])
    if shape == "outliers":
        p = g.normal(size=(n, 3)).astype(np.float32)
        m = max(1, n // 200)
        p[g.choice(n, m, replace=False)] = g.uniform(-1e5, 1e5, (m, 3))
        return p
    if shape == "core_shell":
        k = n // 2
        core = g.normal(0, 0.01, (k, 3))
        d = g.normal(size=(n - k, 3))
        shell = 50 * d / np.linalg.norm(d, axis=1, keepdims=True)
        return np.concatenate([core, shell]).astype(np.float32)
    z = g.uniform(2, 20, n)  # frustum
    tx = np.tan(np.radians(30.0))
    return np.c_[g.uniform(-0.95, 0.95, n) * tx * z, g.uniform(-0.95, 0.95, n) * tx * 0.5625 * z, z].astype(np.float32)


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    g = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    oracle.set_threads(min(16, os.cpu_count() or 1))
    t0, i, fails, checked = time.time(), 0, 0, 0
    while time.time() - t0 < budget:
        shape = SHAPES[i % len(SHAPES)]
        big = i % 8 == 7
        n = int(g.integers(200_000, 2_000_001)) if big else int(np.exp(g.uniform(0, np.log(60_000))))
        pts = make(g, shape, n)
        got = simple_knn._C.distCUDA2(torch.from_numpy(pts).cuda()).cpu().numpy()
        if big:
            idx = g.choice(pts.shape[0], 2048, replace=False).astype(np.int64)
            exp, got = oracle.knn_mean3_subset(pts, idx), got[idx]
        else:
            exp = oracle.knn_mean3(pts)
        bad = int((got.view(np.uint32) != exp.view(np.uint32)).sum())
        checked += exp.size
        fails += bad > 0
        print(f"{'ok  ' if not bad else 'FAIL'} case {i}: {shape} P={pts.shape[0]}{' (2048 sampled)' if big else ''}"
              f" mismatches {bad}", flush=True)
        i += 1
    print(f"{i} cases, {checked} results checked, {fails} failures", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
