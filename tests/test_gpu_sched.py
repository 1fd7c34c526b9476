"""The cost-ordered search dispatch (orpcd_set_option "sched") against the
uniform-split dispatch: the per-pass work items (splits chosen from the
previous pass's measured wave costs, heaviest first) only change which wave
scans which tiles and when, never an answer -- so every GICP result must be
bit-identical."""
import numpy as np
import pytest

from workloads import rot_xyz, small_pair

pytestmark = pytest.mark.gpu

KEYS = ("T", "rmse", "fitness", "iters", "ncorr")


def _run(ctx, opts, fn):
    try:
        for k, v in opts.items():
            ctx.set_option(k, v)
        return fn()
    finally:
        ctx.set_option("sched", 1)
        ctx.set_option("sched_min_starts", 16)
        ctx.set_option("sched_items", 10240)


def _same(a, b):
    for k in KEYS:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("exact_nn", [1, 0])
def test_sched_matches_uniform_multistart(ctx, exact_nn):
    """40 posed starts (>= sched_min_starts) finishing at many passes, max
    iteration reached and not, and a small sched_items (many splits); both
    search modes."""
    src, tgt = small_pair(6000, 5500, seed=41)
    rng = np.random.default_rng(12)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(40)])
    t0 = rng.normal(size=(40, 3)) * 0.1
    ctx.set_target(tgt)
    ctx.set_source(src)

    def run():
        return [ctx.gicp_batch(R0, t0), ctx.gicp_batch(R0[:20], t0[:20], max_iteration=9)]

    ctx.set_option("exact_nn", exact_nn)
    try:
        ref = _run(ctx, {"sched": 0}, run)
        for opts in ({"sched": 1}, {"sched": 1, "sched_items": 64}, {"sched": 1, "sched_items": 200000}):
            got = _run(ctx, opts, run)
            assert len(set(got[0]["iters"].tolist())) > 5
            for g, r in zip(got, ref):
                _same(g, r)
    finally:
        ctx.set_option("exact_nn", 1)


def test_sched_matches_uniform_multi_target(ctx):
    """Several targets in one batch: the item carries its start's target."""
    src, tgt = small_pair(3000, 2800, seed=43)
    targets = [tgt * s for s in ([1, 1, 1], [1.1, 1, 1], [1, 0.9, 1], [1, 1, 1.05])]
    rng = np.random.default_rng(13)
    B = 32
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    tids = np.repeat(np.arange(4, dtype=np.int32), B // 4)
    ctx.set_source(src)
    ctx.set_targets(targets)
    ref = _run(ctx, {"sched": 0}, lambda: ctx.gicp_batch_targets(R0, t0, tids))
    ctx.set_targets(targets)
    got = _run(ctx, {"sched": 1}, lambda: ctx.gicp_batch_targets(R0, t0, tids))
    _same(got, ref)


def test_sched_many_groups_single_start(ctx):
    """A start with more than 2048 query groups (item words with bit 31 set:
    the wave-uniform item must not sign-extend) and the ordered dispatch
    forced on a one-start batch."""
    src, tgt = small_pair(300_000, 280_000, seed=44)
    R0 = rot_xyz(10, -5, 8)[None]
    t0 = np.array([[0.02, -0.01, 0.01]])
    ctx.set_target(tgt)
    ctx.set_source(src)
    ref = _run(ctx, {"sched": 0}, lambda: ctx.gicp_batch(R0, t0, max_iteration=6))
    got = _run(ctx, {"sched": 1, "sched_min_starts": 1}, lambda: ctx.gicp_batch(R0, t0, max_iteration=6))
    _same(got, ref)
