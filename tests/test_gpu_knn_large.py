"""GPU: neighbourhoods of more than 64 points (knn_wave_multi_kernel, up to
1024).  The reference accepts any positive FastGlobalOptimizer
normal_estimate_knn / fpfh_knn and SOR nb_neighbors
(fastGlobalOptimizer.py:86-105, sor.py:51-79); the device KNN keeps the K
nearest as sorted chunks of 64 per query wave.  Against the oracle's KD-tree:

* raw neighbourhood covariances to 1e-12 and normals to 1e-10 at K = 65, 100,
  128, 129, 200, 300 (pure KNN and hybrid radius), the chunk boundaries
  included;
* SOR with 100 / 250 neighbours: per-point mean distances to 1e-14 (the
  neighbour list in (d^2, index) order) and the kept set identical;
* FPFH at k = 100 (the VERDICT's case) and larger: from given normals every
  feature row to 1e-9; with its own normals, normals to 1e-10 and at most 2%
  of the rows moved by the pair-feature swap test's last-bit decisions (as at
  k <= 64, test_gpu_fgr.py);
* a FastGlobalOptimizer with fpfh_knn = normal_estimate_knn = 100 runs end to
  end and recovers the known transform of an index-aligned pair.
"""
import numpy as np
import pytest

from workloads import bumpy_sphere, rot_xyz, small_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("knn,radius", [(65, -1.0), (100, -1.0), (128, -1.0), (129, -1.0), (200, 0.3),
                                        (300, -1.0)])
def test_estimate_normals_large_k(ctx, oracle, knn, radius):
    src, _ = small_pair(3000, seed=7)
    on, oraw, ocov = oracle.estimate_normals(src, knn, radius, 1e-3)
    gn, graw, gcov = ctx.estimate_normals(src, knn, radius, 1e-3)
    assert np.abs(graw - oraw).max() < 1e-12
    assert np.abs(gn - on).max() < 1e-10
    assert np.abs(gcov - ocov).max() < 1e-10


@pytest.mark.parametrize("nb", [100, 250])
def test_sor_large_k(ctx, oracle, nb):
    rng = np.random.default_rng(nb)
    pts = np.concatenate([rng.normal(size=(5000, 3)) * np.array([0.3, 0.2, 0.05]), rng.uniform(-2, 2, size=(50, 3))])
    gi, ga = ctx.sor(pts, nb, 2.0, return_avg=True)
    oi, oa = oracle.sor(pts, nb, 2.0)
    assert np.allclose(ga, oa, rtol=1e-14, atol=0)
    assert np.array_equal(gi, oi)


def _cloud(n=4000, seed=9):
    return bumpy_sphere(n, np.random.default_rng(seed)) * np.array([1.0, 0.8, 0.6])


@pytest.mark.parametrize("nr,nk,fr,fk", [(0.35, 100, 0.4, 100), (0.5, 200, 0.5, 180), (0.8, 300, 0.9, 700)])
def test_fpfh_large_k_matches_oracle(ctx, oracle, nr, nk, fr, fk):
    src = _cloud()
    normals, _ = oracle.fpfh(src, nr, nk, fr, fk)
    of = oracle.fpfh_from_normals(src, normals, fr, fk)
    gf = ctx.fpfh_from_normals(src, normals, fr, fk)
    assert np.allclose(gf, of, atol=1e-9, rtol=0), np.abs(gf - of).max()
    on, of = oracle.fpfh(src, nr, nk, fr, fk)
    gn, gf = ctx.fpfh(src, nr, nk, fr, fk)
    assert np.allclose(gn, on, atol=1e-10, rtol=0)
    bad = np.nonzero(~np.all(np.abs(gf - of) <= 1e-9, axis=1))[0]
    assert len(bad) <= 0.02 * len(src), f"{len(bad)} feature rows differ"


def test_fast_global_optimizer_knn_100():
    from orpcd_amd import FastGlobalOptimizer
    src = _cloud(6000, seed=3)
    R = rot_xyz(10, -5, 20)
    tgt = src @ R.T + np.array([0.05, -0.02, 0.03])   # index-aligned (the reference's Q4 needs it)
    opt = FastGlobalOptimizer(normal_estimate_knn=100, fpfh_knn=100, normal_estimate_radius=0.3, fpfh_radius=0.4)
    T, rmse = opt.optimize(src, tgt)
    Rt = T[:3, :3].T                                  # the plugin returns R transposed (Q1)
    assert np.abs(Rt - R).max() < 1e-6 and rmse < 1e-6, (np.abs(Rt - R).max(), rmse)
