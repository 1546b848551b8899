"""Generates the committed fixtures in tests/golden/.

knn_kat.json   hand-checkable known answers, each derived from distCUDA2's definition in
               the reference text (submodules/simple-knn/simple_knn.cu:133-184): three best
               squared distances to OTHER points (index-excluded, so duplicates give 0),
               initialised to FLT_MAX, result ((b0+b1)+b2)/3.0f in float32.  The expected
               values are computed below in explicit float32 steps, independently of the
               C oracle, and the CPU tests check the oracle against them.
knn_random.npz seeded point sets and the oracle's (oracle/knn_ref.c) values for them; the
               GPU tests compare the HIP kernels with these and with the live oracle.
binning.npz    binning sort + tile-range cases (SortPairs over [0, 32 + getHigherMsb(T)),
               identifyTileRanges; rasterizer_impl.cu:35-50,120-142,354-371): raster-like
               (tile << 32 | float depth bits, Gaussian-major ids) inputs and the expected
               permutation and ranges, computed by plain Python sorting on the tuple
               (tile, depth bits, input index) -- the definition of a stable sort over those
               bits -- and cross-checked against oracle/binning.py.  One case is large enough
               (66,000 pairs) for the segmented GPU path.

Run from the repository root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

F32_MAX = np.float32(np.finfo(np.float32).max)


def f32_round(x: Fraction) -> np.float32:
    """x rounded once to the nearest float32 (ties to even): what a fused multiply-add returns."""
    c = np.float32(float(x))  # within one float32 ulp of x (float() itself rounds to float64 first)
    best = None
    for y in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        if not np.isfinite(y):
            continue
        err = abs(Fraction(float(y)) - x)
        key = (err, int(np.float32(y).view(np.uint32)) & 1)  # nearer first, then the even significand
        if best is None or key < best[0]:
            best = (key, y)
    return np.float32(best[1])


def fma32(a, b, c) -> np.float32:
    """fmaf(a, b, c): the exact a*b + c rounded once."""
    return f32_round(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def by_definition(pts):
    """Plain-Python float32 evaluation, independent of the C oracle (small P only)."""
    pts = np.asarray(pts, dtype=np.float32)
    out = []
    with np.errstate(over="ignore"):
        for i in range(len(pts)):
            best = [F32_MAX, F32_MAX, F32_MAX]
            for j in range(len(pts)):
                if i == j:
                    continue
                d = pts[j] - pts[i]
                # d.x*d.x + d.y*d.y + d.z*d.z contracted as fmaf(dz,dz,fmaf(dx,dx,dy*dy)),
                # each fma exact then rounded once
                a = np.float32(d[1] * d[1])
                dist = fma32(d[2], d[2], fma32(d[0], d[0], a))
                for k in range(3):
                    if best[k] > dist:
                        best[k], dist = dist, best[k]
            s = np.float32(np.float32(best[0] + best[1]) + best[2])
            out.append(np.float32(s / np.float32(3.0)))
    return np.array(out, dtype=np.float32)


KAT_CASES = {
    "single_point": [[0.5, -1.0, 2.0]],
    "two_points": [[0, 0, 0], [1, 0, 0]],
    "three_points": [[0, 0, 0], [1, 0, 0], [3, 0, 0]],
    "axis_tetra": [[0, 0, 0], [1, 0, 0], [0, 2, 0], [0, 0, 3]],
    "four_duplicates": [[1, 2, 3]] * 4,
    "duplicate_pair_on_line": [[0, 0, 0], [0, 0, 0], [1, 0, 0], [2, 0, 0]],
    "unit_cube_corners": [[x, y, z] for x in (0, 1) for y in (0, 1) for z in (0, 1)],
    "collinear_powers_of_two": [[2.0 ** k, 0, 0] for k in range(6)],
    "negative_and_far": [[-1e3, 0, 0], [-1e3, 1, 0], [-1e3, 0, 2], [5e3, 5e3, 5e3], [5e3, 5e3, 5e3 + 0.5]],
}


def bits(a):
    return [int(v) for v in np.asarray(a, dtype=np.float32).view(np.uint32)]


def make_kat():
    out = {}
    for name, pts in KAT_CASES.items():
        exp = by_definition(pts)
        out[name] = {"points": [[float(c) for c in p] for p in pts], "expected_f32_bits": bits(exp),
                     "expected": [float(v) for v in exp]}
    with open(os.path.join(HERE, "knn_kat.json"), "w") as f:
        json.dump(out, f, indent=1)


def random_sets(seed=0):
    g = np.random.default_rng(seed)
    sets = {
        "uniform_cube_777": g.random((777, 3), dtype=np.float32),
        "gaussian_blobs_1500": np.concatenate([g.normal(c, 0.05, (300, 3)) for c in g.random((5, 3))]).astype(np.float32),
        "plane_z0_600": np.c_[g.random((600, 2)), np.zeros(600)].astype(np.float32),
        "integer_grid_ties_512": np.stack(np.meshgrid(np.arange(8), np.arange(8), np.arange(8)), -1).reshape(-1, 3).astype(np.float32),
        "with_outliers_400": np.concatenate([g.random((396, 3)), np.array([[50, 50, 50], [-80, 0, 0], [0, 1e4, 0], [3, 3, 3]])]).astype(np.float32),
    }
    return sets


def make_random():
    import oracle
    sets = random_sets()
    arrays = {}
    for name, pts in sets.items():
        arrays[name + "__points"] = pts
        arrays[name + "__expected"] = oracle.knn_mean3(pts)
        # independent float32 cross-check of the oracle on the small sets
        if len(pts) <= 800:
            assert np.array_equal(by_definition(pts).view(np.uint32), arrays[name + "__expected"].view(np.uint32)), name
    np.savez_compressed(os.path.join(HERE, "knn_random.npz"), **arrays)


def binning_cases(seed=11):
    g = np.random.default_rng(seed)
    cases = {}
    # config-1 shape: 64 tiles, Gaussian-major emission, depths in [2, 20]
    def raster(n_gauss, tiles, spread):
        tl, dp = [], []
        for _ in range(n_gauss):
            t0 = int(g.integers(0, tiles))
            z = np.float32(g.uniform(2.0, 20.0))
            for k in range(int(g.integers(1, spread + 1))):
                tl.append((t0 + k) % tiles)
                dp.append(z)
        return np.array(tl, np.uint16), np.array(dp, np.float32).view(np.uint32)
    cases["config1_64_tiles"] = (*raster(256, 64, 4), 64)
    t, d = raster(400, 10, 3)
    d[::3] = d[0]  # equal depths: stability shows
    cases["ties_10_tiles"] = (t, d, 10)
    cases["one_pair"] = (np.array([5], np.uint16), np.array([np.float32(3.5).view(np.uint32)], np.uint32), 8)
    # segmented path (>= 65536 pairs, >= 64 per segment): 256 tiles, crowded depth buckets
    t = g.integers(0, 256, 66_000).astype(np.uint16)
    d = g.uniform(0.5, 60.0, 66_000).astype(np.float32).view(np.uint32)
    d[::4] = (np.float32(7.0).view(np.uint32) & 0xFFFFF000) | g.integers(0, 4096, d[::4].size).astype(np.uint32)
    cases["segmented_256_tiles"] = (t, d, 256)
    return cases


def make_binning():
    from oracle import binning
    arrays = {}
    for name, (tiles, depth, T) in binning_cases().items():
        n = tiles.size
        keys = (tiles.astype(np.uint64) << np.uint64(32)) | depth.astype(np.uint64)
        vals = np.arange(n, dtype=np.uint32)
        perm = np.array(sorted(range(n), key=lambda i: (int(tiles[i]), int(depth[i]), i)), dtype=np.uint32)
        ranges = np.zeros((T, 2), np.uint32)
        for pos, i in enumerate(perm):
            t = int(tiles[i])
            if ranges[t, 1] == 0 and (pos == 0 or int(tiles[perm[pos - 1]]) != t):
                ranges[t, 0] = pos
            ranges[t, 1] = pos + 1
        if n == 1:
            ranges[int(tiles[0]), 1] = 0  # identifyTileRanges' single-key edge
        end = 32 + max(1, T.bit_length())
        ek, ev = binning.stable_sort_pairs(keys, vals, 0, end)
        assert np.array_equal(ev, perm) and np.array_equal(binning.tile_ranges(ek, T), ranges), name
        arrays[name + "__tiles"] = tiles
        arrays[name + "__depth_bits"] = depth
        arrays[name + "__num_tiles"] = np.array([T], np.int64)
        arrays[name + "__perm"] = perm
        arrays[name + "__ranges"] = ranges
    np.savez_compressed(os.path.join(HERE, "binning.npz"), **arrays)


if __name__ == "__main__":
    make_kat()
    make_random()
    make_binning()
    print("wrote", os.listdir(HERE))
