"""The seed grid (orpcd_set_option "seed_grid"): every query's
search bound is also seeded by the target nearest its cell of the target's
48^3 grid.  A bound only limits which tiles are scanned, never the answer
(the search returns the lexicographic minimum below it, and the seed is a
real target's distance x (1 + 1e-4)), so every GICP result must be
bit-identical with and without it -- for one target and for several targets
in one batch (their grids built by one launch), in both search modes, and
for queries far outside the target's box (clamped to the grid's border)."""
import numpy as np
import pytest

from workloads import c2_pair, rot_xyz, small_pair

pytestmark = pytest.mark.gpu

KEYS = ("T", "rmse", "fitness", "iters", "ncorr")


def _with_grid(ctx, on, fn):
    try:
        ctx.set_option("seed_grid", on)
        return fn()
    finally:
        ctx.set_option("seed_grid", 1)


def _same(a, b):
    for k in KEYS:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("exact_nn", [1, 0])
def test_seed_grid_bit_identical_c2(ctx, exact_nn):
    from orpcd_amd import Preprocessor
    s, t = c2_pair(50_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    rng = np.random.default_rng(21)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(8)])
    t0 = rng.normal(size=(8, 3)) * 0.1
    t0[7] = [3.0, -2.5, 1.0]  # far outside the target's box: every query clamps to the grid's border
    ctx.set_target(t)
    ctx.set_source(s)
    ctx.set_option("exact_nn", exact_nn)
    try:
        ref = _with_grid(ctx, 0, lambda: ctx.gicp_batch(R0, t0))
        got = _with_grid(ctx, 1, lambda: ctx.gicp_batch(R0, t0))
        _same(got, ref)
        assert len(set(got["iters"].tolist())) > 2
    finally:
        ctx.set_option("exact_nn", 1)


def test_seed_grid_bit_identical_multi_target(ctx):
    src, tgt = small_pair(4000, 4500, seed=31)
    targets = [tgt * np.array(sc) for sc in ((1.0, 1.0, 1.0), (1.1, 1.0, 1.0), (1.0, 0.9, 1.0))]
    rng = np.random.default_rng(5)
    R0 = np.array([rot_xyz(*rng.uniform(-60, 60, 3)) for _ in range(12)])
    t0 = rng.normal(size=(12, 3)) * 0.05
    tids = np.repeat(np.arange(3, dtype=np.int32), 4)
    ctx.set_targets(targets)
    ctx.set_source(src)

    def run():
        return ctx.gicp_batch_targets(R0, t0, tids)

    ref = _with_grid(ctx, 0, run)
    got = _with_grid(ctx, 1, run)
    _same(got, ref)
