"""GPU: the lane-per-query KNN (knn_tiles_kernel: one query per lane, the
default from knn_lane_min = 65536 points on: C3's 100k and C5's 1M-point clouds)
returns what the wave-per-query KNN (knn_wave_kernel) returns, bit for bit, on
every path that runs a KNN: raw covariances / normals / GICP covariances
(pure KNN and hybrid radius), FPFH, SOR's mean distances, and the source's
KNN-20 covariances with their boundary ties (listed ties and GICP results).
Forced on small clouds with knn_lane_min = 1 (0: never)."""
import numpy as np
import pytest

from test_gpu_ties import _c1_source
from workloads import bumpy_sphere, rot_xyz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pair():
    from orpcd_amd import _native
    if _native.device_count() == 0:
        pytest.skip("no HIP device")
    wave, lane = _native.Context(0), _native.Context(0)
    wave.set_option("knn_lane_min", 0)
    lane.set_option("knn_lane_min", 1)
    yield wave, lane
    wave.close()
    lane.close()


def _cloud(n=20011, seed=0):
    return bumpy_sphere(n, np.random.default_rng(seed)) * np.array([1.0, 0.8, 0.6])


@pytest.mark.parametrize("knn,radius", [(20, -1.0), (10, 0.05), (64, -1.0), (7, 0.1), (33, 0.08)])
def test_normals_and_covariances_identical(pair, knn, radius):
    wave, lane = pair
    x = _cloud()
    a, b = wave.estimate_normals(x, knn, radius), lane.estimate_normals(x, knn, radius)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("args", [(0.1, 20, 0.25, 40), (0.3, 8, 0.2, 64), (0.05, 30, 0.1, 20)])
def test_fpfh_identical(pair, args):
    wave, lane = pair
    x = _cloud(8003, 1)
    for u, v in zip(wave.fpfh(x, *args), lane.fpfh(x, *args)):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("nb", [64, 20])
def test_sor_identical(pair, nb):
    wave, lane = pair
    x = _cloud(30001, 2)
    x[::97] += np.random.default_rng(3).normal(0, 0.05, size=x[::97].shape)
    (ka, aa), (kb, ab) = wave.sor(x, nb, 2.0, return_avg=True), lane.sor(x, nb, 2.0, return_avg=True)
    assert np.array_equal(ka, kb) and np.array_equal(aa, ab)


def test_source_ties_and_gicp_identical(pair, oracle):
    """C1's source has 8 boundary ties (test_gpu_ties): both kernels list the
    same ones, and a 16-start GICP batch returns the same bits."""
    wave, lane = pair
    s, t = _c1_source(oracle)
    for c in pair:
        c.set_target(t, 1e-3)
        c.set_source(s, cache=False)
    ia, ib = wave.source_ties(), lane.source_ties()
    assert ia["n_ties"] == ib["n_ties"] == 8 and ia["complete"] and ib["complete"]
    assert sorted(ia["rows"].tolist()) == sorted(ib["rows"].tolist())
    rng = np.random.default_rng(7)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(16)])
    t0 = rng.normal(size=(16, 3)) * 0.05
    ra, rb = wave.gicp_batch(R0, t0), lane.gicp_batch(R0, t0)
    for k in ("T", "rmse", "iters"):
        assert np.array_equal(ra[k], rb[k]), k


@pytest.mark.parametrize("kind", ["duplicates", "bucket_ties", "mixed"])
@pytest.mark.parametrize("knn,radius", [(20, -1.0), (8, -1.0), (24, 0.2)])
def test_packed_network_ties_identical(pair, kind, knn, radius):
    """The lane kernel's packed network (64-bit keys: d^2 truncated to a
    bucket of relative width 2^-25 over the input index) on clouds built to
    stress it: exact duplicates (every point 2-7 times: equal-d^2 runs past
    the list's slack, the exact fallback), copies displaced by ~1e-9 of the
    extent (distinct fp64 d^2 in one bucket: the in-bucket exact re-order), and
    both.  Normals / covariances identical to the wave kernel's, bit for bit."""
    wave, lane = pair
    rng = np.random.default_rng({"duplicates": 7, "bucket_ties": 8, "mixed": 9}[kind])
    base = _cloud(3001, 4)
    reps = rng.integers(2, 8, size=len(base))
    x = np.repeat(base, reps, axis=0)
    if kind != "duplicates":
        tiny = rng.normal(size=x.shape) * 1e-9
        if kind == "mixed":
            tiny[rng.random(len(x)) < 0.5] = 0.0
        x = x + tiny
    x = x[rng.permutation(len(x))]
    a, b = wave.estimate_normals(x, knn, radius), lane.estimate_normals(x, knn, radius)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
