"""The zero-code-change drop-in path on the GPU: the reference-shaped Aligner
(one optimize() per attempt, Aligner.py:178-202 -- the plugin offers nothing
else) over GeneralizedICP, whose optimize() recognises rigid images of its
cached cloud and runs the predicted next attempts ahead as one batch
(generalizedICP.py speculate).

* C2 complete align() through that path against the complete CPU-oracle
  align() fixture (tests/golden/g7_align_c2.npz): every one of the 660 calls'
  RMSE within 1e-10, in the reference's order, final RMSE within 1e-12; the
  speculation serves the calls (no prediction missed).
* A caller whose draws the model does not predict (Aligner deg = pi/4 while
  the plugin assumes pi/2): no chain of predicted draws is confirmed, nothing
  runs ahead; every result equals the non-speculating plugin's to 1e-12.
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


class OnlyOptimize:
    """An IOptimizer with nothing but optimize(): the Aligner takes its
    sequential path, exactly the reference's calls."""

    def __init__(self, inner):
        self.inner = inner
        self.rmse = []

    def optimize(self, source, target, **kw):
        try:
            T, m = self.inner.optimize(source, target, **kw)
        except ValueError:
            self.rmse.append(0.0)
            raise
        self.rmse.append(m)
        return T, m


def test_dropin_c2_align_matches_complete_oracle_align():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import c2_pair
    path = os.path.join(GOLDEN, "g7_align_c2.npz")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    z = np.load(path)
    src, tgt = c2_pair(50_000)
    opt = GeneralizedICP()
    plug = OnlyOptimize(opt)
    np.random.seed(0)
    al = Aligner(Preprocessor([]), Preprocessor([]), plug, attempts=30)
    T, m, sf, errors = al.align(src, tgt, refine_registration=False)
    assert np.array_equal(np.asarray(sf).reshape(1, 3), z["sf"]), (sf, z["sf"])
    rmse = np.array(plug.rmse)
    assert len(rmse) == len(z["call_rmse"])
    assert np.abs(rmse - z["call_rmse"]).max() <= 1e-10
    assert abs(m - float(z["metric"])) <= 1e-12 and np.abs(T - z["T"]).max() <= 1e-9
    st = opt.spec_stats
    print(f"drop-in C2 align: {len(rmse)} calls, speculation {st}, |d rmse| {abs(m - float(z['metric'])):.1e}")
    assert st["missed"] == 0 and st["served"] >= len(rmse) - 2 * 22 - 8


def test_dropin_wrong_draw_model_is_detected():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import small_pair
    src, tgt = small_pair(3000, 3200, seed=4)
    res = []
    for spec in (29, 0):
        opt = GeneralizedICP(speculate=spec)
        plug = OnlyOptimize(opt)
        np.random.seed(3)
        al = Aligner(Preprocessor([]), Preprocessor([]), plug, attempts=12, deg=math.pi / 4)
        al.multistart_registration(Preprocessor([]).preprocess(src), Preprocessor([]).preprocess(tgt))
        res.append((np.array(plug.rmse), opt.spec_stats))
    (r_spec, st), (r_plain, _) = res
    assert st["batches"] == 0 and st["served"] == 0, st
    assert len(r_spec) == len(r_plain) == 12 and np.abs(r_spec - r_plain).max() <= 1e-12
