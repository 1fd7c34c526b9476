"""GPU parity of the preprocessing rows on
liborpcd_hip.so against the CPU oracle and the reference's own golden
vectors:

  * SOR (orpcd_sor): kept indices identical to the oracle's
    RemoveStatisticalOutliers restatement; mean distances to 1e-14 relative
    (same neighbour sets, same summation order, correctly rounded sqrt);
  * voxel downsampling (orpcd_voxel_down_sample): every averaged point
    bit-identical (same per-voxel summation order), same voxel order;
  * farthest-point sampling (orpcd_farthest_downsample): the chosen points
    bit-identical to the REFERENCE FarthestDownsampler's (g6_fps.npz) and to
    the numpy restatement on larger clouds, including exact distance ties.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from workloads import armadillo, c2_pair

pytestmark = pytest.mark.gpu


def _outlier_cloud(seed, n=6000, m=60):
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.normal(size=(n, 3)) * np.array([0.3, 0.2, 0.05]), rng.uniform(-2, 2, size=(m, 3))])


@pytest.mark.parametrize("nb,ratio", [(64, 2.0), (20, 1.0), (8, 0.5), (1, 2.0), (33, 3.0)])
def test_sor_matches_oracle(ctx, oracle, nb, ratio):
    pts = _outlier_cloud(nb)
    gi, ga = ctx.sor(pts, nb, ratio, return_avg=True)
    oi, oa = oracle.sor(pts, nb, ratio)
    assert np.allclose(ga, oa, rtol=1e-14, atol=0)
    assert np.array_equal(gi, oi)


def test_sor_edges(ctx, oracle):
    small = np.random.default_rng(1).normal(size=(30, 3))       # nb > n: every point is a neighbour
    assert np.array_equal(ctx.sor(small, 64, 2.0), oracle.sor(small, 64, 2.0)[0])
    dup = np.concatenate([np.zeros((6, 3)), np.random.default_rng(2).normal(size=(200, 3))])
    gi = ctx.sor(dup, 4, 2.0)                                    # mean 0 (all-duplicate neighbourhood): dropped
    assert np.array_equal(gi, oracle.sor(dup, 4, 2.0)[0]) and not np.isin(np.arange(6), gi).any()
    assert len(ctx.sor(np.zeros((0, 3)), 64, 2.0)) == 0         # empty cloud
    with pytest.raises(ValueError):
        ctx.sor(small, 0, 2.0)
    with pytest.raises(ValueError):
        ctx.sor(small, 1025, 2.0)


def test_sor_block_and_c1_preprocessing(oracle):
    """C1's preprocessing: Preprocessor([RandomDownsampler(5000), SOR()]) on ArmadilloBack_330."""
    from orpcd_amd.Preprocessor import Preprocessor
    from orpcd_amd.Preprocessor.Downsamplers import RandomDownsampler
    from orpcd_amd.Preprocessor.Outliers import SOR
    src, _ = armadillo()
    np.random.seed(0)
    got = Preprocessor([RandomDownsampler(5000), SOR()]).preprocess(src)
    np.random.seed(0)
    x = oracle.radius_scale(src)[0]
    x = oracle.random_downsample(x, 5000)
    keep, _ = oracle.sor(x, 64, 2)
    assert np.array_equal(got, x[keep])
    assert 4800 < len(got) < 5000


@pytest.mark.parametrize("vs", [0.003, 0.01, 0.05, 0.3, 5.0])
def test_voxel_matches_oracle(ctx, oracle, vs):
    src, _ = c2_pair(50_000)
    c = (src - src.mean(0)) / np.max(np.linalg.norm(src - src.mean(0), axis=1))
    g = ctx.voxel_down_sample(c, vs)
    o = oracle.voxel_down_sample(c, vs)
    assert g.shape == o.shape and np.array_equal(g, o)
    assert ctx.voxel_down_sample(c, vs, count_only=True) == len(o)


def test_voxel_edges(ctx, oracle):
    one = np.array([[0.1, 0.2, 0.3]])
    assert np.array_equal(ctx.voxel_down_sample(one, 0.01), one)
    dup = np.repeat(np.random.default_rng(3).normal(size=(10, 3)), 7, axis=0)
    assert np.array_equal(ctx.voxel_down_sample(dup, 1e-3), oracle.voxel_down_sample(dup, 1e-3))
    assert ctx.voxel_down_sample(np.zeros((0, 3)), 0.1, count_only=True) == 0
    with pytest.raises(ValueError):
        ctx.voxel_down_sample(one, 0.0)


def test_voxel_downsampler_compass(oracle):
    from orpcd_amd.Preprocessor.Downsamplers import VoxelDownsampler
    src, _ = armadillo()
    c = oracle.radius_scale(src)[0]
    vd = VoxelDownsampler(2000)
    got = vd.process(c)
    # voxelDownsampler.py:87-125 on the oracle's counts
    cur, delta, eps, mn = 0.01, 0.01, 0.0005, 0.0001
    metric = abs(2000 - oracle.voxel_down_sample(c, cur, True))
    best = cur
    while delta >= eps:
        moved = False
        for d in (delta, -delta):
            v = max(cur + d, mn) if cur + d > mn else mn
            m = abs(2000 - oracle.voxel_down_sample(c, v, True))
            if m < metric:
                cur, metric, best, moved = v, m, v, True
                break
        if not moved:
            delta /= 2
    assert vd.voxel_size == best
    assert np.array_equal(got, oracle.voxel_down_sample(c, best))


def test_fps_matches_reference_golden(ctx):
    from make_golden_fps import cases
    z = np.load(os.path.join(GOLDEN, "g6_fps.npz"))
    for name, (cloud, k, seed) in cases().items():
        idx = ctx.farthest_downsample(cloud, k, int(z[name + "_first"]))
        assert np.array_equal(cloud[idx], z[name + "_points"]), name


def test_fps_block_replays_reference_rng():
    from make_golden_fps import cases
    from orpcd_amd.Preprocessor.Downsamplers import FarthestDownsampler
    z = np.load(os.path.join(GOLDEN, "g6_fps.npz"))
    cloud, k, seed = cases()["arm"]
    np.random.seed(seed)
    got = FarthestDownsampler(k).process(cloud)
    assert np.array_equal(got, z["arm_points"]) and np.random.random() == float(z["arm_after"])


@pytest.mark.parametrize("n,k", [(50_000, 600), (200_003, 300), (1000, 1500)])
def test_fps_large_and_oversampled(ctx, oracle, n, k):
    pts = np.random.default_rng(n).normal(size=(n, 3))
    first = n // 3
    g = ctx.farthest_downsample(pts, k, first)
    o = oracle.farthest_downsample(pts, k, first)
    assert np.array_equal(g, o)
