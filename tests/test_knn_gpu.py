"""distCUDA2 on the MI355X: the gfx950 kernels (hidegs_amd/csrc/knn.hip) against the CPU oracle.

Tolerance: none.  The device and the oracle evaluate the same float32 operations in the
same order (explicit fmaf, -ffp-contract=off on both sides, ((b0+b1)+b2)/3.0f), so every
result must be bit-identical (compared as uint32 bit patterns; inf and FLT_MAX/3 included).
Sizes: every point checked up to 100k; at 2M a seeded sample of queries is checked against
all 2M points, plus size-independent properties (permutation equivariance, exact scaling by
powers of two).
"""
import os

import numpy as np
import pytest
import torch

import simple_knn

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def knn(points_np):
    out = simple_knn._C.distCUDA2(torch.from_numpy(np.ascontiguousarray(points_np, np.float32)).cuda())
    torch.cuda.synchronize()
    return out.cpu().numpy()


def assert_bits_equal(got, exp, what=""):
    g, e = got.view(np.uint32), exp.view(np.uint32)
    bad = np.flatnonzero(g != e)
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first {bad[:5]}: got {got[bad[:5]]} expected {exp[bad[:5]]}"


def frustum_points(n, seed=0):
    """SURVEY §8(d) D2 placement: z ~ U[2,20], x = u tan(30°) z, y = v tan(30°)(1080/1920) z, u,v ~ U[-.95,.95]."""
    g = torch.Generator().manual_seed(seed)
    z = 2 + 18 * torch.rand(n, generator=g)
    u = (torch.rand(n, generator=g) * 2 - 1) * 0.95
    v = (torch.rand(n, generator=g) * 2 - 1) * 0.95
    tx = float(np.tan(np.radians(30.0)))
    return torch.stack([u * tx * z, v * tx * (1080 / 1920) * z, z], 1).numpy()


def sfm_like(n, seed=1):
    """Surface-concentrated cloud (two planes and a noisy sphere) with 0.2% far outliers."""
    g = np.random.default_rng(seed)
    k = n // 3
    ground = np.c_[g.uniform(-50, 50, (k, 2)), g.normal(0, 0.02, k)]
    wall = np.c_[g.uniform(-50, 50, k), np.full(k, 20.0) + g.normal(0, 0.02, k), g.uniform(0, 30, k)]
    d = g.normal(size=(n - 2 * k, 3))
    sphere = 10 * d / np.linalg.norm(d, axis=1, keepdims=True) + np.array([0, 0, 15]) + g.normal(0, 0.05, (n - 2 * k, 3))
    pts = np.concatenate([ground, wall, sphere]).astype(np.float32)
    m = max(1, n // 500)
    pts[g.choice(n, m, replace=False)] = g.uniform(-2000, 2000, (m, 3))
    return pts


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 63, 64, 65, 127, 128, 129, 1000, 4095, 4097, 65537])
def test_uniform_sizes_bit_exact(oracle_lib, P):
    pts = np.random.default_rng(P).random((P, 3), dtype=np.float32)
    assert_bits_equal(knn(pts), oracle_lib.knn_mean3(pts), f"P={P}")


def test_committed_known_answers():
    import json
    with open(os.path.join(GOLD, "knn_kat.json")) as f:
        cases = json.load(f)
    for name, case in cases.items():
        got = knn(np.array(case["points"], dtype=np.float32))
        assert got.view(np.uint32).tolist() == case["expected_f32_bits"], name


def test_committed_random_fixtures():
    z = np.load(os.path.join(GOLD, "knn_random.npz"))
    for key in z.files:
        if key.endswith("__points"):
            name = key[:-len("__points")]
            assert_bits_equal(knn(z[key]), z[name + "__expected"], name)


@pytest.mark.parametrize("maker", ["duplicates", "identical", "line", "plane", "ties_grid", "two_far_clusters"])
def test_degenerate_sets_bit_exact(oracle_lib, maker):
    g = np.random.default_rng(11)
    if maker == "duplicates":
        base = g.random((3000, 3), dtype=np.float32)
        pts = np.concatenate([base, base[:1500], base[:700]])
    elif maker == "identical":
        pts = np.full((5000, 3), 0.25, dtype=np.float32)
    elif maker == "line":
        pts = np.c_[g.random(8000), np.zeros(8000), np.zeros(8000)].astype(np.float32)
    elif maker == "plane":
        pts = np.c_[g.random((8000, 2)), np.full(8000, 3.0)].astype(np.float32)
    elif maker == "ties_grid":
        pts = np.stack(np.meshgrid(*[np.arange(20)] * 3), -1).reshape(-1, 3).astype(np.float32)
    else:
        pts = np.concatenate([g.normal(0, 1, (4000, 3)), g.normal(1e5, 1, (3, 3))]).astype(np.float32)
    assert_bits_equal(knn(pts), oracle_lib.knn_mean3(pts), maker)


@pytest.mark.parametrize("case", ["nan_coordinates", "inf_coordinates", "nan_and_inf"])
def test_non_finite_points_bit_exact(oracle_lib, case):
    """Non-finite coordinates (a diverged point): the reference keeps a candidate only if
    `knn[j] > dist` (simple_knn.cu:139), which is false for NaN and for +inf, so such points never enter
    anyone's three best, and a NaN point's own result is (FLT_MAX x 3) / 3 = inf.  The search's Morton
    codes, boxes and bounds must not let a non-finite point hide a finite neighbour."""
    g = np.random.default_rng(23)
    pts = g.random((20000, 3), dtype=np.float32)
    idx = g.choice(20000, 40, replace=False)
    if case in ("nan_coordinates", "nan_and_inf"):
        pts[idx[:10], g.integers(0, 3, 10)] = np.nan
        pts[idx[10:15]] = np.nan
    if case in ("inf_coordinates", "nan_and_inf"):
        pts[idx[15:25], g.integers(0, 3, 10)] = np.inf
        pts[idx[25:30], g.integers(0, 3, 5)] = -np.inf
        pts[idx[30:32]] = np.inf
    assert_bits_equal(knn(pts), oracle_lib.knn_mean3(pts), case)


def test_concurrent_calls_from_host_threads(oracle_lib):
    """Three host threads, each on its own stream, run distCUDA2 on different clouds at once (its scratch
    callback, sort and search interleave on the device); every result bit-identical to the oracle."""
    import threading
    clouds = [frustum_points(30000, seed=s) for s in (31, 32)] + [sfm_like(30000, seed=33)]
    expected = [oracle_lib.knn_mean3(c) for c in clouds]
    dev = [torch.from_numpy(np.ascontiguousarray(c)).cuda() for c in clouds]
    torch.cuda.synchronize()
    got, failures = [None] * 3, []

    def worker(i):
        try:
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.default_stream())
            with torch.cuda.stream(st):
                for _ in range(3):
                    out = simple_knn._C.distCUDA2(dev[i])
                st.synchronize()
                got[i] = out.cpu().numpy()
        except Exception as e:  # noqa: BLE001 -- reported below
            failures.append(repr(e))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    assert not failures, failures
    for i in range(3):
        assert_bits_equal(got[i], expected[i], f"thread {i}")


def test_frustum_100k_every_point(oracle_lib):
    pts = frustum_points(100_000)
    assert_bits_equal(knn(pts), oracle_lib.knn_mean3(pts), "frustum 100k")


def test_sfm_like_200k_sampled(oracle_lib):
    pts = sfm_like(200_000)
    got = knn(pts)
    idx = np.random.default_rng(5).choice(len(pts), 4000, replace=False)
    outl = np.flatnonzero(np.abs(pts).max(1) > 100)
    idx = np.unique(np.concatenate([idx, outl]))
    assert_bits_equal(got[idx], oracle_lib.knn_mean3_subset(pts, idx), "sfm-like 200k")


def test_frustum_2m_sampled_and_properties(oracle_lib):
    pts = frustum_points(2_000_000, seed=3)
    got = knn(pts)
    assert np.isfinite(got).all() and (got >= 0).all()
    idx = np.random.default_rng(9).choice(len(pts), 2048, replace=False)
    assert_bits_equal(got[idx], oracle_lib.knn_mean3_subset(pts, idx), "frustum 2M sample")
    # permutation equivariance (the result may not depend on input order)
    perm = np.random.default_rng(2).permutation(len(pts))
    assert_bits_equal(knn(pts[perm]), got[perm], "permuted 2M")
    # scaling every coordinate by 2 scales every squared distance by exactly 4
    assert_bits_equal(knn(pts * np.float32(2)), got * np.float32(4), "scaled 2M")


def test_runs_on_current_stream_and_device_tensor_types():
    pts = torch.rand(5000, 3, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a = simple_knn._C.distCUDA2(pts)
    s.synchronize()
    b = simple_knn._C.distCUDA2(pts)
    assert torch.equal(a, b)
    assert b.device == pts.device and b.dtype == torch.float32 and b.shape == (5000,)
    # non-contiguous input is made contiguous like the reference's points.contiguous()
    wide = torch.rand(5000, 6, device="cuda")
    assert torch.equal(simple_knn._C.distCUDA2(wide[:, ::2]), simple_knn._C.distCUDA2(wide[:, ::2].contiguous()))


def test_config5_scale_10m_sampled(oracle_lib):
    """Config 5's scene size (10M points): sampled queries bit-exact against the brute-force oracle
    (each against all 10M points), and the result is finite and non-negative everywhere."""
    pts = frustum_points(10_000_000, seed=4)
    got = knn(pts)
    assert got.shape == (10_000_000,) and np.isfinite(got).all() and (got >= 0).all()
    idx = np.random.default_rng(10).choice(len(pts), 256, replace=False)
    assert_bits_equal(got[idx], oracle_lib.knn_mean3_subset(pts, idx), "frustum 10M sample")
