"""Generates the committed distCUDA2 fixtures in tests/golden/.

knn_kat.json   hand-checkable known answers, each derived from distCUDA2's definition in
               the reference text (submodules/simple-knn/simple_knn.cu:133-184): three best
               squared distances to OTHER points (index-excluded, so duplicates give 0),
               initialised to FLT_MAX, result ((b0+b1)+b2)/3.0f in float32.  The expected
               values are computed below in explicit float32 steps, independently of the
               C oracle, and the CPU tests check the oracle against them.
knn_random.npz seeded point sets and the oracle's (oracle/knn_ref.c) values for them; the
               GPU tests compare the HIP kernels with these and with the live oracle.

Run from the repository root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

F32_MAX = np.float32(np.finfo(np.float32).max)


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
                # fmaf(dz,dz,fmaf(dy,dy,dx*dx)): exact in float64 then rounded once per fma
                a = np.float32(d[0] * d[0])
                b = np.float32(np.float64(d[1]) * np.float64(d[1]) + np.float64(a))
                dist = np.float32(np.float64(d[2]) * np.float64(d[2]) + np.float64(b))
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


if __name__ == "__main__":
    make_kat()
    make_random()
    print("wrote", os.listdir(HERE))
