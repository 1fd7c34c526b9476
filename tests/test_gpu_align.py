"""The metric's "final RMSE vs ref" leg on the GPU: a complete Aligner.align()
(Aligner.py:228-317, refine off) against the committed COMPLETE CPU-oracle
align() of the same config (tests/golden/g7_align_*.npz, made by
tests/golden/make_golden_align.py: every optimize call on the C++/OpenMP
restatement of Open3D's GICP, the reference's control flow and RNG stream).

Gates:
* C2 (50k <-> 50k, configs[1]) in the default exact mode: identical scale
  factors and compass decisions; every multistart's 30 per-start iteration
  counts identical and RMSEs within 1e-10, in reference order; final RMSE
  within 1e-12 and T within 1e-9 (the correspondences are the oracle's; only
  summation order differs).
  In the fp32-answer mode (exact_nn=False): scale factors identical, final
  RMSE within 1e-5 (north_star), T within 1e-4.
* C4 (C2 with 64 starts per multistart, configs[3]; the one-GPU run of the
  strong-scaling case bench.py times at every N): the same gates as C2.
* C1 (Armadillo 330->0, Random(5000) + SOR, configs[0]): the same gates as
  C2.  The build computes the source's KNN-20 covariances once and rotates
  them per start, while the oracle (like Open3D in the reference) recomputes
  them on every posed copy; the C1 source has 8 points whose 20th and 21st
  neighbours are within the posing rounding of each other, and the batch
  re-decides exactly those per start from the posed coordinates
  (runtime.hip SourceTies, tests/test_gpu_ties.py).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _fixture(cfg):
    path = os.path.join(GOLDEN, f"g7_align_{cfg}.npz")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    return np.load(path)


def _per_start(history):
    rmse = np.concatenate([h["rmse"] for h in history])
    iters = np.concatenate([h["iters_per_start"] for h in history])
    return rmse, iters


def test_c2_align_matches_complete_oracle_align():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    z = _fixture("c2")
    src, tgt = c2_pair(50_000)
    np.random.seed(0)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(), attempts=30)
    T, m, sf, errors = al.align(src, tgt, refine_registration=False)
    assert np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"]), (sf, z["sf"])
    assert len(errors) == len(z["errors"]) and np.abs(np.asarray(errors) - z["errors"]).max() <= 1e-12
    rmse, iters = _per_start(al.history)
    assert len(rmse) == len(z["call_rmse"])          # the same multistarts in the same order
    assert np.array_equal(iters, z["call_iters"])
    # per start: the same correspondences every pass, so only round-off of the
    # summation order and of the rotated (vs recomputed) source covariances;
    # measured 2.9e-12 worst over the 660 starts (starts that run to the
    # 100-iteration cap in a flat basin carry it furthest)
    assert np.abs(rmse - z["call_rmse"]).max() <= 1e-10
    assert abs(m - float(z["metric"])) <= 1e-12 and np.abs(T - z["T"]).max() <= 1e-9
    print(f"C2 align exact: |d rmse| {abs(m - float(z['metric'])):.1e} |dT| {np.abs(T - z['T']).max():.1e}")
    # the fp32-answer mode: the north_star's stated tolerance
    np.random.seed(0)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(exact_nn=False), attempts=30)
    T, m, sf, errors = al.align(src, tgt, refine_registration=False)
    assert np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"])
    assert abs(m - float(z["metric"])) <= 1e-5 and np.abs(T - z["T"]).max() <= 1e-4


def test_c1_align_matches_complete_oracle_align():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from orpcd_amd.Preprocessor.Downsamplers import RandomDownsampler
    from orpcd_amd.Preprocessor.Outliers import SOR
    from workloads import armadillo
    z = _fixture("c1")
    src, tgt = armadillo()
    np.random.seed(0)
    al = Aligner(Preprocessor([RandomDownsampler(5000), SOR()]), Preprocessor([RandomDownsampler(5000), SOR()]),
                 GeneralizedICP(), attempts=30)
    T, m, sf, errors = al.align(src, tgt, refine_registration=False)
    assert np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"]), (sf, z["sf"])
    assert len(errors) == len(z["errors"])
    assert np.abs(np.asarray(errors) - z["errors"]).max() <= 1e-12
    rmse, iters = _per_start(al.history)
    assert len(rmse) == len(z["call_rmse"])
    print(f"C1 align: |d rmse| {abs(m - float(z['metric'])):.1e} |dT| {np.abs(T - z['T']).max():.1e} "
          f"per-start iterations identical {int((iters == z['call_iters']).sum())}/{len(iters)}, "
          f"worst per-start |d rmse| {np.abs(rmse - z['call_rmse']).max():.1e}")
    assert np.array_equal(iters, z["call_iters"])
    assert np.abs(rmse - z["call_rmse"]).max() <= 1e-10
    assert abs(m - float(z["metric"])) <= 1e-12 and np.abs(T - z["T"]).max() <= 1e-9


def test_c4_align_matches_complete_oracle_align():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    z = _fixture("c4")
    src, tgt = c2_pair(50_000)
    np.random.seed(0)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(), attempts=64)
    T, m, sf, errors = al.align(src, tgt, refine_registration=False)
    assert np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"]), (sf, z["sf"])
    assert len(errors) == len(z["errors"]) and np.abs(np.asarray(errors) - z["errors"]).max() <= 1e-12
    rmse, iters = _per_start(al.history)
    assert len(rmse) == len(z["call_rmse"])
    assert np.array_equal(iters, z["call_iters"])
    assert np.abs(rmse - z["call_rmse"]).max() <= 1e-10
    assert abs(m - float(z["metric"])) <= 1e-12 and np.abs(T - z["T"]).max() <= 1e-9
    print(f"C4 align: {len(rmse)} starts, |d rmse| {abs(m - float(z['metric'])):.1e} "
          f"|dT| {np.abs(T - z['T']).max():.1e}, worst per-start {np.abs(rmse - z['call_rmse']).max():.1e}")
