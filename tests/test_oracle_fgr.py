"""The FastGlobal half of the oracle (FPFH + FGR restated from Open3D 0.18,
which is absent here: "parity unpinned" against Open3D itself).  Pinned
instead against an independent pure-Python restatement of SPFH/FPFH on a
small cloud and against exact known-transform recovery."""
import math

import numpy as np
import pytest
from scipy.spatial import cKDTree

from workloads import bumpy_sphere, rot_xyz


def _pair_features(p1, n1, p2, n2):
    d = p2 - p1
    f4 = np.linalg.norm(d)
    if f4 == 0:
        return 0.0, 0.0, 0.0, 0.0
    a1 = n1 @ d / f4
    a2 = n2 @ d / f4
    if math.acos(abs(a1)) > math.acos(abs(a2)):
        n1, n2, d, f3 = n2, n1, -d, -a2
    else:
        f3 = a1
    v = np.cross(d, n1)
    vn = np.linalg.norm(v)
    if vn == 0:
        return 0.0, 0.0, 0.0, 0.0
    v = v / vn
    w = np.cross(n1, v)
    return math.atan2(w @ n2, n1 @ n2), v @ n2, f3, f4


def _bin(x):
    return min(max(int(math.floor(x)), 0), 10)


def _python_fpfh(pts, normals, radius, knn):
    tree = cKDTree(pts)
    nbrs = []
    for i in range(len(pts)):
        d, j = tree.query(pts[i], k=knn)
        keep = d ** 2 < radius ** 2
        nbrs.append((j[keep], d[keep] ** 2))
    spfh = np.zeros((len(pts), 33))
    for i, (js, _) in enumerate(nbrs):
        if len(js) > 1:
            inc = 100.0 / (len(js) - 1)
            for j in js[1:]:
                f = _pair_features(pts[i], normals[i], pts[j], normals[j])
                spfh[i, _bin(11 * (f[0] + math.pi) / (2 * math.pi))] += inc
                spfh[i, _bin(11 * (f[1] + 1) * 0.5) + 11] += inc
                spfh[i, _bin(11 * (f[2] + 1) * 0.5) + 22] += inc
    feat = np.zeros_like(spfh)
    for i, (js, d2) in enumerate(nbrs):
        if len(js) > 1:
            s = np.zeros(3)
            for j, dd in zip(js[1:], d2[1:]):
                if dd == 0:
                    continue
                val = spfh[j] / dd
                s += val.reshape(3, 11).sum(axis=1)
                feat[i] += val
            s = np.where(s != 0, 100.0 / np.where(s != 0, s, 1), 0)
            feat[i] = feat[i] * np.repeat(s, 11) + spfh[i]
    return feat


def test_fpfh_matches_python_restatement(oracle):
    rng = np.random.default_rng(11)
    pts = bumpy_sphere(600, rng) * np.array([1.0, 0.8, 0.6])
    normals, feat = oracle.fpfh(pts, 0.25, 20, 0.3, 16)
    assert np.allclose(np.linalg.norm(normals, axis=1), 1.0)
    ref = _python_fpfh(pts, normals, 0.3, 16)
    assert np.allclose(feat, ref, rtol=1e-9, atol=1e-9)
    # each of the three SPFH blocks of the FPFH sums to 200 (100 own + 100 neighbours)
    full = feat[feat.sum(axis=1) > 0]
    assert np.allclose(full.reshape(-1, 3, 11).sum(axis=2), 200.0)


def test_fpfh_isolated_points_have_zero_features(oracle):
    pts = np.array([[0.0, 0, 0], [5.0, 0, 0], [0, 5.0, 0]])
    normals, feat = oracle.fpfh(pts, 0.1, 20, 0.1, 20)
    assert np.all(feat == 0)
    assert np.allclose(normals, [[0, 0, 1]] * 3) or np.all(np.isfinite(normals))


@pytest.mark.parametrize("compat_q4", [False, True])
def test_fgr_recovers_rigid_transform(oracle, compat_q4):
    rng = np.random.default_rng(4)
    src = bumpy_sphere(3000, rng) * np.array([1.0, 0.8, 0.6])
    R, t = rot_xyz(25, -10, 40), np.array([0.1, -0.05, 0.2])
    tgt = src @ R.T + t
    _, fs = oracle.fpfh(src, 0.1, 20, 0.25, 40)
    ft = fs if compat_q4 else oracle.fpfh(tgt, 0.1, 20, 0.25, 40)[1]
    r = oracle.fgr(src, tgt, fs, ft, maximum_correspondence_distance=0.05, seed=3)
    assert r["n_mutual"] > 500 and r["n_tuple_corr"] == 3000   # 1000 tuples x 3
    if compat_q4:   # identical feature lists: every mutual match is the true one -> exact
        assert np.allclose(r["T"][:3, :3], R, atol=1e-6) and np.allclose(r["T"][:3, 3], t, atol=1e-6)
        assert r["fitness"] == 1.0 and r["rmse"] < 1e-6
    else:           # robust (Geman-McClure) estimate over matches with outliers
        ang = math.degrees(math.acos(np.clip((np.trace(r["T"][:3, :3].T @ R) - 1) / 2, -1, 1)))
        assert ang < 0.5 and np.linalg.norm(r["T"][:3, 3] - t) < 5e-3 and r["fitness"] > 0.99


def test_fgr_seed_changes_tuples_not_result(oracle):
    rng = np.random.default_rng(4)
    src = bumpy_sphere(2000, rng)
    tgt = src @ rot_xyz(0, 0, 30).T
    _, fs = oracle.fpfh(src, 0.1, 20, 0.25, 40)
    a = oracle.fgr(src, tgt, fs, fs, seed=1)
    b = oracle.fgr(src, tgt, fs, fs, seed=2)
    assert a["n_mutual"] == b["n_mutual"]
    assert np.allclose(a["T"], b["T"], atol=1e-6)


def test_fgr_few_correspondences_returns_mean_alignment(oracle):
    # < 10 tuple correspondences -> IRLS returns identity in normalised space:
    # the result only re-centres the means (GetInvTransformationOriginalScale)
    src = np.random.default_rng(0).normal(size=(40, 3))
    tgt = src + np.array([3.0, 0, 0])
    fs = np.zeros((40, 33))
    r = oracle.fgr(src, tgt, fs, fs, seed=0)
    # all-zero features tie everywhere: lowest index wins both ways -> the only
    # mutual match is (0, 0), whose degenerate tuples never pass the test
    assert r["n_mutual"] == 1 and r["n_tuple_corr"] == 0
    assert np.allclose(r["T"][:3, :3], np.eye(3))
    assert np.allclose(r["T"][:3, 3], tgt.mean(0) - src.mean(0))
