"""GPU: one GICP with the source rows split over ranks (C5's multi-GPU path),
through the C-ABI (orpcd_set_source_rows / orpcd_gicp_shard_*).

* one rank: bit-identical to orpcd_gicp_batch with B = 1 (same reduction);
* two ranks emulated by two contexts in one process, the 29 sums added on the
  host as the all-reduce would: T within 1e-9 of the un-sharded run (only the
  summation order of the sums differs), same iteration count;
* against the CPU oracle: the usual GICP tolerances (T <= 1e-6, rmse <= 1e-7).
"""
import numpy as np
import pytest

from workloads import small_pair

pytestmark = pytest.mark.gpu


def _pair():
    return small_pair(6007, 5003, seed=11)


def test_shard_single_rank_is_bitwise_gicp_batch(ctx):
    from orpcd_amd import parallel
    src, tgt = _pair()
    r = parallel.gicp_rows_sharded(ctx, src, tgt, max_correspondence_distance=0.3)
    ctx.set_target(tgt, 1e-3, cache=False)
    ctx.set_source(src, cache=False)
    b = ctx.gicp_batch(np.eye(3)[None], np.zeros((1, 3)), max_correspondence_distance=0.3)
    assert np.array_equal(r["T"], b["T"][0]) and r["rmse"] == b["rmse"][0]
    assert r["iters"] == b["iters"][0] and r["ncorr"] == b["ncorr"][0] and r["fitness"] == b["fitness"][0]


def test_shard_device_collectives_single_rank_is_bitwise_gicp_batch():
    """The pass loop with the all-reduce on the device (RCCL communicator of
    one rank, orpcd_gicp_shard_run): bit-identical to orpcd_gicp_batch B = 1
    and to the host-collective row path; a second run on the same
    communicator as well (a context of its own: comm state per context)."""
    from orpcd_amd import _native, parallel
    src, tgt = _pair()
    c = _native.Context(0)
    r = parallel.gicp_rows_sharded(c, src, tgt, max_correspondence_distance=0.3, device_collectives=True)
    h = parallel.gicp_rows_sharded(c, src, tgt, max_correspondence_distance=0.3)
    r2 = parallel.gicp_rows_sharded(c, src, tgt, max_correspondence_distance=0.3, device_collectives=True)
    c.set_target(tgt, 1e-3, cache=False)
    c.set_source(src, cache=False)
    b = c.gicp_batch(np.eye(3)[None], np.zeros((1, 3)), max_correspondence_distance=0.3)
    for x in (r, h, r2):
        assert np.array_equal(x["T"], b["T"][0]) and x["rmse"] == b["rmse"][0]
        assert x["iters"] == b["iters"][0] and x["ncorr"] == b["ncorr"][0] and x["fitness"] == b["fitness"][0]
    c.comm_destroy()
    c.close()


@pytest.mark.parametrize("splits", [2, 3])
def test_shard_emulated_ranks_match_unsharded(ctx, oracle, splits):
    from orpcd_amd import _native, parallel
    src, tgt = _pair()
    ctxs = [_native.Context(0) for _ in range(splits)]
    for k, c in enumerate(ctxs):
        lo, hi = parallel.shard(len(src), k, splits)
        c.set_target(tgt, 1e-3)
        c.set_source_rows(src, lo, hi)
        c.shard_begin(np.eye(3), np.zeros(3), n_total=len(src), max_correspondence_distance=0.3)
    while True:
        parts = [c.shard_pass() for c in ctxs]
        assert len({a for _, a in parts}) == 1
        if not parts[0][1]:
            break
        total = np.sum([s for s, _ in parts], axis=0)
        done = {c.shard_update(total) for c in ctxs}
        assert len(done) == 1
        if done.pop():
            break
    res = [c.shard_result() for c in ctxs]
    for r in res[1:]:
        assert np.array_equal(r["T"], res[0]["T"]) and r["rmse"] == res[0]["rmse"]
    ref = parallel.gicp_rows_sharded(ctx, src, tgt, max_correspondence_distance=0.3)
    assert res[0]["iters"] == ref["iters"] and res[0]["ncorr"] == ref["ncorr"]
    assert np.allclose(res[0]["T"], ref["T"], atol=1e-9, rtol=0)
    o = oracle.gicp(src, tgt, 0.3)
    assert np.allclose(res[0]["T"], o["T"], atol=1e-6, rtol=0) and abs(res[0]["rmse"] - o["rmse"]) <= 1e-7


def test_shard_errors(ctx):
    src, tgt = _pair()
    with pytest.raises(ValueError):
        ctx.set_source_rows(src, 10, 5)
    with pytest.raises(ValueError):
        ctx.set_source_rows(src, 0, len(src) + 1)


def test_shard_c5_size_two_ranks_match_oracle(oracle):
    """C5's multi-GPU path at its own size (1M <-> 1M, BASELINE configs[4];
    VERDICT r03 missing #3): the source rows split over 2 emulated ranks (two
    contexts, the all-reduce of the 29 sums done on the host), two GICP
    passes, against the oracle's two passes (T <= 1e-6, rmse <= 1e-7 -- the
    per-optimize gate; measured far tighter) and identical across ranks."""
    from orpcd_amd import _native, parallel
    from workloads import c5_pair
    src, tgt = c5_pair()
    ctxs = [_native.Context(0) for _ in range(2)]
    for k, c in enumerate(ctxs):
        lo, hi = parallel.shard(len(src), k, 2)
        c.set_target(tgt, 1e-3)
        c.set_source_rows(src, lo, hi)
        c.shard_begin(np.eye(3), np.zeros(3), n_total=len(src), max_iteration=2)
    while True:
        parts = [c.shard_pass() for c in ctxs]
        if not parts[0][1]:
            break
        total = np.sum([s for s, _ in parts], axis=0)
        if {c.shard_update(total) for c in ctxs}.pop():
            break
    res = [c.shard_result() for c in ctxs]
    assert np.array_equal(res[0]["T"], res[1]["T"]) and res[0]["rmse"] == res[1]["rmse"]
    o = oracle.gicp(src, tgt, 0.5, 2)
    assert res[0]["iters"] == o["iters"] and res[0]["ncorr"] == o["ncorr"]
    assert np.abs(res[0]["T"] - o["T"]).max() <= 1e-6 and abs(res[0]["rmse"] - o["rmse"]) <= 1e-7
    print(f"C5 2 ranks: |dT| {np.abs(res[0]['T'] - o['T']).max():.1e} |d rmse| {abs(res[0]['rmse'] - o['rmse']):.1e}")
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("lane_min", [0, 1])
def test_target_rows_emulated_ranks_assemble_the_full_target(lane_min):
    """orpcd_set_target_rows over 3 emulated ranks (3 contexts; both KNN
    kernels): each rank's Morton rows are the full orpcd_set_target's, bit for
    bit; their concatenation through orpcd_set_target_cov gives a target on
    which a GICP batch returns the same bits; an incomplete target is refused
    by the GICP calls; one rank alone is complete at once."""
    from orpcd_amd import _native
    from shard_fake import FakeShardContext
    src, tgt = _pair()
    full = _native.Context(0)
    full.set_option("knn_lane_min", lane_min)
    full.set_target(tgt, 1e-3, cache=False)
    want = full.target_cov_rows(0, len(tgt))
    ctxs = [_native.Context(0) for _ in range(3)]
    parts, rows = [], []
    for r, c in enumerate(ctxs):
        c.set_option("knn_lane_min", lane_min)
        lo, hi = c.set_target_rows(tgt, r, 3, 1e-3)
        assert lo % 64 == 0 and (hi % 64 == 0 or hi == len(tgt))
        sl = FakeShardContext.target_slice(len(tgt), 3)    # the layout the CPU gloo tests' fake uses
        assert (lo, hi) == (min(len(tgt), r * sl), min(len(tgt), r * sl + sl))
        rows.append((lo, hi))
        parts.append(c.target_cov_rows(lo, hi))
        assert np.array_equal(parts[-1], want[lo:hi])
    assert rows[0][0] == 0 and rows[-1][1] == len(tgt) and all(rows[k][1] == rows[k + 1][0] for k in range(2))
    with pytest.raises(ValueError, match="no target"):
        ctxs[1].set_source(src, cache=False)
        ctxs[1].gicp_batch(np.eye(3)[None], np.zeros((1, 3)))
    with pytest.raises(ValueError):
        ctxs[1].target_cov_rows(0, len(tgt))       # rows another rank computed
    ctxs[0].set_target_cov(np.concatenate(parts))
    ctxs[0].set_source(src, cache=False)
    full.set_source(src, cache=False)
    R0 = np.array([np.eye(3), np.eye(3)[[1, 2, 0]]])
    t0 = np.zeros((2, 3))
    a, b = ctxs[0].gicp_batch(R0, t0, max_correspondence_distance=0.3), full.gicp_batch(R0, t0,
                                                                                       max_correspondence_distance=0.3)
    for k in ("T", "rmse", "iters", "ncorr"):
        assert np.array_equal(a[k], b[k]), k
    one = _native.Context(0)
    one.set_option("knn_lane_min", lane_min)
    assert one.set_target_rows(tgt, 0, 1, 1e-3) == (0, len(tgt))
    assert np.array_equal(one.target_cov_rows(0, len(tgt)), want)
    for c in ctxs + [full, one]:
        c.close()
