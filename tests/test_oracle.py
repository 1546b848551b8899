"""The CPU oracle (test infrastructure) pinned against the committed known answers.

knn_kat.json holds values derived by hand from distCUDA2's definition in the reference
text (tests/golden/make_golden.py); knn_random.npz holds seeded sets the oracle produced
when the fixtures were made (cross-checked there by an independent float32 evaluation).
Parity against the reference's own outputs is unpinned: the reference ships no tests or
fixtures and its CUDA sources may not be built here.
"""
import json
import os

import numpy as np
import pytest

from oracle import binning

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def kat():
    with open(os.path.join(GOLD, "knn_kat.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", sorted(kat()))
def test_knn_oracle_matches_known_answers(oracle_lib, name):
    case = kat()[name]
    got = oracle_lib.knn_mean3(np.array(case["points"], dtype=np.float32))
    assert got.view(np.uint32).tolist() == case["expected_f32_bits"]


def test_knn_oracle_edge_semantics(oracle_lib):
    # P = 1, 2 keep two FLT_MAX terms -> inf; P = 3 keeps one -> FLT_MAX / 3 (simple_knn.cu:155,183)
    assert np.isinf(oracle_lib.knn_mean3(np.zeros((1, 3), np.float32))).all()
    assert np.isinf(oracle_lib.knn_mean3(np.eye(3, dtype=np.float32)[:2])).all()
    three = oracle_lib.knn_mean3(np.eye(3, dtype=np.float32))
    assert np.all(three == np.float32(np.finfo(np.float32).max) / np.float32(3))


def test_knn_oracle_random_fixture(oracle_lib):
    z = np.load(os.path.join(GOLD, "knn_random.npz"))
    for key in z.files:
        if key.endswith("__points"):
            name = key[:-len("__points")]
            got = oracle_lib.knn_mean3(z[key])
            assert np.array_equal(got.view(np.uint32), z[name + "__expected"].view(np.uint32)), name


def test_knn_oracle_close_to_float64_brute_force(oracle_lib):
    g = np.random.default_rng(7)
    pts = g.normal(size=(300, 3)).astype(np.float32)
    d = ((pts[None, :, :].astype(np.float64) - pts[:, None, :]) ** 2).sum(-1)
    np.fill_diagonal(d, np.inf)
    exp = np.sort(d, axis=1)[:, :3].mean(1)
    got = oracle_lib.knn_mean3(pts)
    np.testing.assert_allclose(got, exp, rtol=1e-5)


def test_knn_oracle_subset_agrees(oracle_lib):
    g = np.random.default_rng(3)
    pts = g.random((2000, 3), dtype=np.float32)
    idx = g.choice(2000, 100, replace=False)
    full = oracle_lib.knn_mean3(pts)
    assert np.array_equal(oracle_lib.knn_mean3_subset(pts, idx), full[idx])


# ---- binning oracles ---------------------------------------------------------------

@pytest.mark.parametrize("n,bits", [(64, 7), (8160, 13), (32400, 15), (0, 1), (1, 1), (2, 2), (255, 8), (256, 9),
                                    (2**31, 32), (2**32 - 1, 32)])
def test_higher_msb_known_answers(n, bits):
    # 64 -> 7, 8160 -> 13, 32400 -> 15: SURVEY.md §8(c) C3(i), tile counts of configs 1, 2/3, 5
    assert binning.bit_length_at_least_one(n) == bits


def test_tile_ranges_oracle():
    keys = np.array([(0 << 32) | 5, (0 << 32) | 9, (2 << 32) | 1, (3 << 32) | 0, (3 << 32) | 7], dtype=np.uint64)
    r = binning.tile_ranges(keys, 5)
    assert r.tolist() == [[0, 2], [0, 0], [2, 3], [3, 5], [0, 0]]
    # the reference's n == 1 edge: the single range keeps end 0
    assert binning.tile_ranges(np.array([(4 << 32) | 1], dtype=np.uint64), 6).tolist()[4] == [0, 0]


def test_stable_sort_oracle_is_stable_over_bit_range():
    keys = np.array([0x1_0000_0003, 0x0_0000_0003, 0x2_0000_0001, 0x0_0000_0001], dtype=np.uint64)
    vals = np.arange(4, dtype=np.uint32)
    k, v = binning.stable_sort_pairs(keys, vals, 0, 32)  # high bits ignored -> ties keep input order
    assert v.tolist() == [2, 3, 0, 1]
    k, v = binning.stable_sort_pairs(keys, vals, 0, 40)
    assert v.tolist() == [3, 1, 0, 2]


def test_scan_oracle_wraps():
    x = np.array([0xFFFFFFFF, 2, 3], dtype=np.uint32)
    assert binning.inclusive_scan_u32(x).tolist() == [0xFFFFFFFF, 1, 4]


def binning_fixture():
    z = np.load(os.path.join(GOLD, "binning.npz"))
    names = sorted({k.split("__")[0] for k in z.files})
    out = {}
    for name in names:
        tiles, depth = z[name + "__tiles"], z[name + "__depth_bits"]
        keys = (tiles.astype(np.uint64) << np.uint64(32)) | depth.astype(np.uint64)
        out[name] = (keys, int(z[name + "__num_tiles"][0]), z[name + "__perm"], z[name + "__ranges"])
    return out


@pytest.mark.parametrize("name", sorted(binning_fixture()))
def test_binning_oracle_matches_committed_fixture(name):
    """tests/golden/binning.npz: expected permutation and ranges from plain Python sorting on
    (tile, depth bits, index) -- the oracle must agree."""
    keys, T, perm, ranges = binning_fixture()[name]
    vals = np.arange(keys.size, dtype=np.uint32)
    ek, ev = binning.stable_sort_pairs(keys, vals, 0, 32 + binning.bit_length_at_least_one(T))
    assert np.array_equal(ev, perm)
    assert np.array_equal(binning.tile_ranges(ek, T), ranges)


@pytest.mark.parametrize("n,begin,end,threads", [(1, 0, 45, 4), (1000, 0, 39, 3), (300_000, 0, 45, 8),
                                                 (200_000, 7, 51, 5), (50_000, 0, 64, 2), (10_000, 32, 32, 4)])
def test_omp_sort_oracle_equals_numpy_definition(oracle_lib, n, begin, end, threads):
    """The multi-threaded radix sort (the binning CPU baseline) is the same stable sort as the
    numpy definition, whatever the thread count, with heavy key ties."""
    g = np.random.default_rng(n + begin)
    keys = (g.integers(0, 64, n).astype(np.uint64) << np.uint64(32)) | g.integers(0, 50, n).astype(np.uint64)
    keys ^= g.integers(0, 2, n).astype(np.uint64) << np.uint64(63)
    vals = np.arange(n, dtype=np.uint32)
    ek, ev = binning.stable_sort_pairs(keys, vals, begin, end)
    ko, vo = oracle_lib.sort_pairs_omp(keys, vals, begin, end, threads)
    assert np.array_equal(ko, ek) and np.array_equal(vo, ev)


def test_omp_adam_oracle_independent_of_threads(oracle_lib):
    g = np.random.default_rng(3)
    p0, g0 = g.standard_normal((5000, 7), dtype=np.float32), g.standard_normal((5000, 7), dtype=np.float32)
    rel = g.random(5000) < 0.5
    outs = []
    before = oracle_lib.set_threads(0)
    for th in (1, 6):
        assert oracle_lib.set_threads(th) == th
        p, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
        oracle_lib.masked_adam(p, g0.copy(), m, v, rel, 1e-3, 0.9, 0.999, 1e-15, 0.0, 3)
        outs.append(p)
    oracle_lib.set_threads(before)
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
