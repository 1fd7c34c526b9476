"""The CPU oracle pinned against the reference's golden vectors and against
independent numpy/scipy computations (no GPU)."""
import numpy as np
import pytest
from scipy.spatial import cKDTree
from scipy.spatial.transform import Rotation

from conftest import GOLDEN


def test_fast_eigen3x3_is_smallest_eigenvector(oracle):
    rng = np.random.default_rng(0)
    for _ in range(500):
        A = rng.normal(size=(3, 3))
        A = A @ A.T * rng.uniform(1e-6, 10)
        n = oracle.fast_eigen3x3(A)
        w, V = np.linalg.eigh(A)
        assert abs(abs(n @ V[:, 0]) - 1) < 1e-6


def test_fast_eigen3x3_degenerate_cases(oracle):
    assert np.allclose(oracle.fast_eigen3x3(np.zeros((3, 3))), 0)          # zero matrix -> zero normal
    assert np.allclose(oracle.fast_eigen3x3(np.eye(3)), [0, 0, 1])          # identity -> (0,0,1)
    assert np.allclose(oracle.fast_eigen3x3(np.diag([1.0, 0.1, 2.0])), [0, 1, 0])
    assert np.allclose(oracle.fast_eigen3x3(np.diag([0.1, 1.0, 2.0])), [1, 0, 0])


def test_gicp_cov_from_normal(oracle):
    rng = np.random.default_rng(1)
    for _ in range(200):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        C = oracle.gicp_cov_from_normal(n, 1e-3)
        if n[0] < -0.99:  # GetRotationFromE1ToX quirk
            assert np.allclose(C, np.diag([1e-3, 1, 1]))
        else:
            assert np.allclose(C, np.eye(3) - (1 - 1e-3) * np.outer(n, n), atol=1e-12)
    C = oracle.gicp_cov_from_normal(np.array([-1.0, 0, 0]), 1e-3)
    assert np.allclose(C, np.diag([1e-3, 1, 1]))


def test_solve_psd6_and_det_gate(oracle):
    rng = np.random.default_rng(2)
    A = rng.normal(size=(6, 6))
    A = A @ A.T
    b = rng.normal(size=6)
    ok, x, det = oracle.solve_psd6(A, b)
    assert ok and np.allclose(x, np.linalg.solve(A, b), rtol=1e-10)
    assert np.isclose(det, np.linalg.det(A))
    ok, x, _ = oracle.solve_psd6(A * 1e-3, b)  # |det| = det(A) 1e-18 < 1e-6 -> Open3D refuses
    assert not ok and np.all(x == 0)


def test_vec6_to_m4_matches_zyx_euler(oracle):
    rng = np.random.default_rng(3)
    for _ in range(20):
        x = rng.normal(size=6) * 0.4
        T = oracle.vec6_to_m4(x)
        R = Rotation.from_euler("ZYX", [x[2], x[1], x[0]]).as_matrix()
        assert np.allclose(T[:3, :3], R, atol=1e-15)
        assert np.array_equal(T[:3, 3], x[3:]) and np.array_equal(T[3], [0, 0, 0, 1])


def test_nn1_and_knn_match_scipy(oracle):
    rng = np.random.default_rng(4)
    t = rng.normal(size=(4000, 3))
    q = rng.normal(size=(3000, 3)) * 1.3
    idx, d2 = oracle.nn1_radius(q, t, 0.25)
    dd, ii = cKDTree(t).query(q, distance_upper_bound=0.25)
    m = np.isfinite(dd)
    assert np.array_equal(idx[m], ii[m]) and np.all(idx[~m] == -1)
    assert np.allclose(d2[m], dd[m] ** 2, rtol=1e-12)
    ki, kd, kc = oracle.knn(t, t[:200], 20)
    dd, ii = cKDTree(t).query(t[:200], k=20)
    assert np.array_equal(ki, ii) and np.all(kc == 20)
    ki, kd, kc = oracle.knn(t, t[:200], 20, radius=0.2)  # hybrid
    for r in range(200):
        inside = np.sort(((t - t[r]) ** 2).sum(1))
        assert kc[r] == min(20, int((inside < 0.04).sum()))


def test_nn1_ties_resolve_to_lowest_index(oracle):
    t = np.array([[1.0, 0, 0], [-1.0, 0, 0], [0, 1.0, 0], [1.0, 0, 0]])
    idx, d2 = oracle.nn1_radius(np.zeros((1, 3)), t, 2.0)
    assert idx[0] == 0 and d2[0] == 1.0
    idx, _ = oracle.nn1_radius(np.zeros((1, 3)), t, 1.0)  # strict d2 < r2
    assert idx[0] == -1


def test_gicp_recovers_known_transform(oracle):
    from workloads import small_pair, rot_xyz
    src, _ = small_pair(3000, noise=0.0)
    R = rot_xyz(10, -5, 7)
    t = np.array([0.02, -0.01, 0.03])
    r = oracle.gicp(src, src @ R.T + t, trace=True)
    assert np.allclose(r["T"][:3, :3], R, atol=1e-9) and np.allclose(r["T"][:3, 3], t, atol=1e-9)
    assert r["fitness"] == 1.0 and r["rmse"] < 1e-9
    assert len(r["trace_rmse"]) == r["iters"] + 1


def test_gicp_zero_correspondences(oracle):
    src = np.random.default_rng(5).normal(size=(50, 3))
    r = oracle.gicp(src, src + 100.0)
    assert r["rmse"] == 0 and r["fitness"] == 0 and r["iters"] == 1 and np.allclose(r["T"], np.eye(4))


# ------------------------------------------------- golden vectors (reference)
def test_oracle_rng_replay_matches_reference_G1(oracle):
    g = np.load(f"{GOLDEN}/g1_rng.npz")
    for seed in (0, 1, 42):
        np.random.seed(seed)
        al = oracle.OracleAligner(None)
        for n in range(64):
            R, t = al.initialize_rotation()
            assert np.array_equal(R, g[f"R_{seed}"][n]) and np.array_equal(t, g[f"t_{seed}"][n])


def test_oracle_preprocess_matches_reference_G2(oracle):
    from workloads import armadillo
    g = np.load(f"{GOLDEN}/g2_preprocess.npz")
    for name, cloud in zip(("ArmadilloBack_330", "ArmadilloBack_0"), armadillo()):
        np.random.seed(0)
        scaled, mean, scale = oracle.radius_scale(cloud)
        out = oracle.random_downsample(scaled, 5000)
        assert np.allclose(mean, g[f"{name}_mean"], rtol=0, atol=1e-12)
        assert np.isclose(scale, g[f"{name}_scale"], rtol=1e-15)
        assert np.allclose(out, g[f"{name}_out"], rtol=0, atol=1e-15)


@pytest.mark.parametrize("mode,attempts,seed", [("scripted", 4, 7), ("never_improves", 30, 0), ("constant", 2, 3)])
def test_oracle_aligner_matches_reference_G3(oracle, mode, attempts, seed):
    from scripted import ScriptedOptimizer
    g = np.load(f"{GOLDEN}/g3_aligner_trace.npz")
    np.random.seed(seed)
    opt = ScriptedOptimizer(g["goal"], mode=mode)
    T, m, sf, err = oracle.OracleAligner(opt, attempts=attempts).align(g["src"].copy(), g["tgt"].copy())
    assert np.array_equal(T, g[f"{mode}_T"]) and m == g[f"{mode}_metric"]
    assert np.array_equal(sf, g[f"{mode}_sf"]) and np.array_equal(err, g[f"{mode}_errors"])
    assert len(opt.calls) == len(g[f"{mode}_call_rmse"])
    assert np.array_equal(np.random.uniform(size=4), g[f"{mode}_rng_after"])


def test_oracle_reproduces_g4_g5_regression_fixtures(oracle):
    """G4/G5 (tests/golden/make_golden_oracle.py): the oracle's GICP traces and
    FPFH/FGR outputs are stable across rounds (regression anchors, not Open3D)."""
    import os
    from conftest import GOLDEN
    from make_golden_oracle import c1_pair, g5_pair
    from workloads import small_pair
    z = np.load(os.path.join(GOLDEN, "g45_oracle.npz"))
    for name, (s, t) in {"p300": small_pair(300, seed=0), "c1": c1_pair()}.items():
        r = oracle.gicp(s, t, 0.5, 100, trace=True)
        assert np.allclose(r["T"], z[f"g4_{name}_T"], rtol=0, atol=1e-12)
        assert r["iters"] == int(z[f"g4_{name}_iters"])
        assert np.array_equal(r["trace_ncorr"], z[f"g4_{name}_trace_ncorr"])
        assert np.allclose(r["trace_rmse"], z[f"g4_{name}_trace_rmse"], rtol=1e-12, atol=0)
    s, t = g5_pair()
    _, fs = oracle.fpfh(s)
    assert np.allclose(fs, z["g5_src_feat"], rtol=0, atol=1e-9)
    r = oracle.fgr(s, t, fs, z["g5_tgt_feat"], seed=0)
    assert r["n_mutual"] == int(z["g5_n_mutual"]) and r["n_tuple_corr"] == int(z["g5_n_tuple"])
    assert np.allclose(r["T"], z["g5_T"], rtol=0, atol=1e-12)
