"""CPU oracle for the rows either side of the hot path:
PointToPoint ICP refinement, SOR, voxel downsampling, farthest-point
sampling.  Each restatement is checked against an independent numpy/scipy
computation, and FPS against golden vectors produced by the reference's own
FarthestDownsampler (tests/golden/make_golden_fps.py).
"""
import os

import numpy as np
import pytest
from scipy.spatial import cKDTree

from conftest import GOLDEN
from workloads import rot_xyz, small_pair


def _kabsch(s, d):
    ms, md = s.mean(0), d.mean(0)
    H = (d - md).T @ (s - ms) / len(s)
    U, _, Vt = np.linalg.svd(H)
    S = np.diag([1.0, 1.0, -1.0 if np.linalg.det(U) * np.linalg.det(Vt) < 0 else 1.0])
    R = U @ S @ Vt
    return R, md - R @ ms


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_umeyama_matches_numpy_svd(oracle, seed):
    rng = np.random.default_rng(seed)
    s = rng.normal(size=(400, 3)) * np.array([1.0, 0.5, 0.2])
    R = rot_xyz(*rng.uniform(-90, 90, size=3))
    d = s @ R.T + rng.normal(size=3) + rng.normal(0, 1e-3, size=s.shape)
    T = oracle.umeyama(s, d)
    R2, t2 = _kabsch(s, d)
    assert np.abs(T[:3, :3] - R2).max() < 1e-12
    assert np.abs(T[:3, 3] - t2).max() < 1e-12
    assert np.allclose(T[3], [0, 0, 0, 1])


def test_umeyama_reflection_and_degenerate(oracle):
    # a reflection in the data must still yield a proper rotation (det +1)
    s = np.random.default_rng(3).normal(size=(50, 3))
    d = s * np.array([1.0, 1.0, -1.0])
    T = oracle.umeyama(s, d)
    assert abs(np.linalg.det(T[:3, :3]) - 1.0) < 1e-12
    # planar (rank-2 sigma) and collinear inputs give finite rotations
    p = np.random.default_rng(4).normal(size=(60, 3)) * np.array([1.0, 1.0, 0.0])
    T = oracle.umeyama(p, p @ rot_xyz(0, 0, 30).T)
    assert np.abs(T[:3, :3] - rot_xyz(0, 0, 30)).max() < 1e-12
    line = np.outer(np.arange(10.0), [1.0, 2.0, 3.0])
    T = oracle.umeyama(line, line + 1.0)
    assert np.all(np.isfinite(T)) and abs(np.linalg.det(T[:3, :3]) - 1.0) < 1e-12
    T1 = oracle.umeyama(line[:1], line[:1] + 1.0)  # one pair: sigma = 0 -> R = I, t = d - s
    assert np.array_equal(T1[:3, :3], np.eye(3)) and np.allclose(T1[:3, 3], 1.0)


def test_icp_p2p_recovers_known_transform(oracle):
    src, _ = small_pair(3000, seed=5)
    R = rot_xyz(6, -4, 5)
    t = np.array([0.03, -0.02, 0.01])
    tgt = src @ R.T + t
    r = oracle.icp_p2p(src, tgt, 0.5, np.eye(4), 200)
    assert r["rmse"] < 1e-8 and r["fitness"] == 1.0
    assert np.abs(r["T"][:3, :3] - R).max() < 1e-7 and np.abs(r["T"][:3, 3] - t).max() < 1e-7
    # init is applied as Open3D applies it (column convention) and is part of T
    init = np.eye(4)
    init[:3, :3] = rot_xyz(3, -2, 2)
    init[:3, 3] = [0.01, 0.0, 0.005]
    r2 = oracle.icp_p2p(src, tgt, 0.5, init, 200)
    assert np.abs(r2["T"][:3, :3] - R).max() < 1e-7 and r2["rmse"] < 1e-8
    # max_iteration = 0: T = init, result of the initial correspondences
    r0 = oracle.icp_p2p(src, tgt, 0.5, init, 0)
    assert np.array_equal(r0["T"], init) and r0["iters"] == 0
    with pytest.raises(ValueError):
        oracle.icp_p2p(src, tgt, 0.0, np.eye(4), 10)


def test_sor_matches_independent_kdtree(oracle):
    rng = np.random.default_rng(6)
    pts = np.concatenate([rng.normal(size=(4000, 3)) * 0.1, rng.uniform(-2, 2, size=(40, 3))])
    for nb, ratio in ((64, 2.0), (20, 1.0), (1, 2.0)):
        idx, avg = oracle.sor(pts, nb, ratio)
        d, _ = cKDTree(pts).query(pts, k=nb)
        d = d.reshape(len(pts), -1)
        mean = np.array([sum(np.sqrt(x * x) for x in row) / len(row) for row in d])  # sqrt(d^2), summed in order
        assert np.allclose(avg, mean, rtol=1e-12, atol=1e-15)
        pos = avg > 0
        cm = avg[pos].sum() / len(pts)
        sd = np.sqrt(((avg[pos] - cm) ** 2).sum() / (len(pts) - 1))
        exp = np.nonzero(pos & (avg < cm + ratio * sd))[0]
        assert np.array_equal(idx, exp)
    assert oracle.sor(pts, 64, 2.0)[0].size < len(pts)


def test_sor_quirks(oracle):
    # duplicates: a point whose neighbours all coincide has mean 0 and is dropped
    pts = np.concatenate([np.zeros((5, 3)), np.random.default_rng(7).normal(size=(100, 3))])
    idx, avg = oracle.sor(pts, 4, 2.0)
    assert np.all(avg[:5] == 0) and not np.isin(np.arange(5), idx).any()
    with pytest.raises(ValueError):
        oracle.sor(pts, 0, 2.0)
    with pytest.raises(ValueError):
        oracle.sor(pts, 4, 0.0)


@pytest.mark.parametrize("vs", [0.05, 0.2, 1.0])
def test_voxel_down_sample_matches_numpy(oracle, vs):
    rng = np.random.default_rng(8)
    pts = rng.normal(size=(5000, 3)) * 0.5
    out = oracle.voxel_down_sample(pts, vs)
    vmin = pts.min(0) - vs * 0.5
    key = np.floor((pts - vmin) / vs).astype(np.int64)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)  # lexicographic
    inv = inv.reshape(-1)
    exp = np.zeros((len(uniq), 3))
    cnt = np.zeros(len(uniq))
    for i in range(len(pts)):  # input-order accumulation
        exp[inv[i]] += pts[i]
        cnt[inv[i]] += 1
    exp /= cnt[:, None]
    assert out.shape == exp.shape and np.array_equal(out, exp)
    assert oracle.voxel_down_sample(pts, vs, count_only=True) == len(uniq)


def test_fps_oracle_matches_reference_golden():
    import oracle as O
    from make_golden_fps import cases
    z = np.load(os.path.join(GOLDEN, "g6_fps.npz"))
    for name, (cloud, k, seed) in cases().items():
        np.random.seed(seed)
        first = np.random.randint(low=0, high=cloud.shape[0])
        assert first == int(z[name + "_first"])
        idx = O.farthest_downsample(cloud, k, first)
        assert np.array_equal(cloud[idx], z[name + "_points"]), name
