"""GPU parity of the PointToPoint refinement:
Aligner.refine_registration (Aligner.py:319-364) -> registration_icp(...,
TransformationEstimationPointToPoint()) on liborpcd_hip.so
(orpcd_icp_p2p_batch) against the CPU oracle (oracle_icp_p2p).

Tolerances as the GICP path: T elementwise <= 1e-6, inlier RMSE <= 1e-7,
fitness <= 1e-4, iteration count within 1.  The device forms Umeyama's
sigma from one-pass first moments (fp64, fixed order); the oracle from
demeaned products like Eigen: they agree to ~1e-15 relative.
"""
import numpy as np
import pytest

from workloads import rot_xyz, small_pair

pytestmark = pytest.mark.gpu

T_TOL, RMSE_TOL = 1e-6, 1e-7


def _init(deg, t):
    T = np.eye(4)
    T[:3, :3] = rot_xyz(*deg)
    T[:3, 3] = t
    return T


def _check(g, o, b=0):
    assert np.abs(g["T"][b] - o["T"]).max() <= T_TOL
    assert abs(g["rmse"][b] - o["rmse"]) <= RMSE_TOL
    assert abs(g["fitness"][b] - o["fitness"]) <= 1e-4
    assert abs(int(g["iters"][b]) - o["iters"]) <= 1


def test_icp_p2p_batch_matches_oracle(ctx, oracle):
    src, tgt = small_pair(3001, 2777, seed=3)
    inits = np.stack([np.eye(4), _init((4, -3, 5), (0.02, 0.0, -0.01)), _init((-10, 8, 3), (0.0, 0.05, 0.0))])
    ctx.set_target_points(tgt)
    ctx.set_source_points(src)
    for max_corr, max_iter in ((0.5, 200), (0.05, 30), (0.5, 0), (0.5, 1)):
        g = ctx.icp_p2p_batch(inits, max_correspondence_distance=max_corr, max_iteration=max_iter)
        for b in range(len(inits)):
            o = oracle.icp_p2p(src, tgt, max_corr, inits[b], max_iter)
            _check(g, o, b)


def test_icp_p2p_known_transform_and_edges(ctx, oracle):
    src, _ = small_pair(2000, seed=4)
    R = rot_xyz(5, -4, 6)
    tgt = src @ R.T + np.array([0.02, -0.01, 0.03])
    ctx.set_target_points(tgt)
    ctx.set_source_points(src)
    g = ctx.icp_p2p_batch(np.eye(4)[None])
    assert g["rmse"][0] < 1e-8 and np.abs(g["T"][0][:3, :3] - R).max() < 1e-7
    # nothing within the radius: T = init, rmse 0, fitness 0 (Open3D returns the empty result)
    far = _init((0, 0, 0), (100.0, 0, 0))
    g = ctx.icp_p2p_batch(far[None], max_correspondence_distance=0.1, max_iteration=10)
    o = oracle.icp_p2p(src, tgt, 0.1, far, 10)
    assert g["rmse"][0] == 0.0 and g["fitness"][0] == 0.0 and np.array_equal(g["T"][0], o["T"])
    with pytest.raises(ValueError):
        ctx.icp_p2p_batch(np.eye(4)[None], max_correspondence_distance=0.0)
    bad = np.eye(4)
    bad[0, 3] = np.nan
    with pytest.raises(ValueError):
        ctx.icp_p2p_batch(bad[None])


def test_gicp_after_points_only_source(ctx, oracle):
    """A PointToPoint source layout must not be mistaken for a GICP source."""
    src, tgt = small_pair(1500, 1600, seed=5)
    ctx.set_target_points(tgt)
    ctx.set_source_points(src)
    ctx.icp_p2p_batch(np.eye(4)[None], max_iteration=5)
    ctx.set_target(tgt)
    ctx.set_source(src)
    r = ctx.gicp_batch(np.eye(3)[None], np.zeros((1, 3)))
    o = oracle.gicp(src, tgt)
    assert np.abs(r["T"][0] - o["T"]).max() <= T_TOL


def test_aligner_refine_registration(oracle):
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    src, tgt = small_pair(2500, 2400, seed=6)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(), attempts=4)
    T0 = np.eye(4)
    T0[:3, :3] = rot_xyz(3, -2, 4).T  # a row-convention T as align() composes it
    T0[:3, 3] = [0.01, 0.0, -0.02]
    T, rmse = al.refine_registration(src, tgt, T0, icp_type="PointToPoint")
    o = oracle.icp_p2p(src, tgt, 0.5, T0, 200)  # Open3D reads the row-convention T as column convention (Q5)
    assert np.abs(T - o["T"]).max() <= T_TOL and abs(rmse - o["rmse"]) <= RMSE_TOL
    with pytest.raises(RuntimeError):
        al.refine_registration(src, tgt, T0, icp_type="PointToPlane")
    with pytest.raises(TypeError):
        al.refine_registration(src, tgt, T0, icp_type="Colored")


def test_align_with_refinement_matches_oracle(oracle):
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    src_raw, tgt_raw = small_pair(2000, 1900, seed=7, deg=(20, -10, 15))
    np.random.seed(3)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(), attempts=6, delta=0.2, eps=0.1)
    T, metric, sf, errors = al.align(src_raw, tgt_raw, refine_registration=True, icp_type="PointToPoint")
    np.random.seed(3)
    oal = oracle.OracleAligner(oracle.OracleGeneralizedICP(), attempts=6, delta=0.2, eps=0.1)
    To, mo, sfo, erro = oal.align(src_raw, tgt_raw)
    assert np.array_equal(sf, sfo)
    s = oracle.radius_scale(src_raw)[0]
    t = oracle.radius_scale(tgt_raw)[0] * sfo
    o = oracle.icp_p2p(s, t, 0.5, To, 200)
    assert np.abs(T - o["T"]).max() <= 1e-4 and abs(metric - o["rmse"]) <= 1e-5
    assert len(errors) == len(erro) + 1 and errors[-1] == metric
