"""GPU parity of the exact-nearest-neighbour mode (option ``exact_nn``, the default).

With ``exact_nn`` every correspondence is the oracle's: the fp64 lexicographic
(d^2, input index) minimum of oracle/orpcd_oracle.cpp KDTree::nn1 (:192-217).
The fp32 search tracks each query's runner-up; a query whose runner-up (or
another split's winner) lies within the fp32 error band of its winner is
re-searched in fp64 (nn_exact_kernel); every other query's fp32 winner is
provably the fp64 one.  Tolerances:
  * correspondences: identical indices (integer work: bit-exact);
  * per-optimize GICP at full C2 size: identical iteration counts, T within
    1e-9 elementwise and inlier RMSE within 1e-12 -- the two sides differ only
    in the summation order of the 29 normal-equation terms and in how the
    posed points are formed (oracle: pcd.Transform per iteration; GPU: the
    composed pose), ~1e-16 relative per pass.
"""
import numpy as np
import pytest

from workloads import rot_xyz, small_pair

pytestmark = pytest.mark.gpu


def _posed(src, R0, t0):
    """The query transform's fp64 arithmetic (xform, no contraction):
    q_i = ((Q_i0 p0 + Q_i1 p1) + Q_i2 p2) + Q_i3 with Q = [R0^T | t0]."""
    p0, p1, p2 = src[:, 0], src[:, 1], src[:, 2]
    return np.stack([((R0[0, i] * p0 + R0[1, i] * p1) + R0[2, i] * p2) + t0[i] for i in range(3)], axis=1)


@pytest.fixture
def exact(ctx):
    ctx.set_option("exact_nn", 1)  # the default; tests of the other mode restore it
    yield ctx


def _c2():
    from orpcd_amd import Preprocessor
    from workloads import c2_pair
    s, t = c2_pair(50_000)
    return Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)


def _check_corr(ctx, oracle, src, tgt, R0, t0, radius):
    B = len(R0)
    g = ctx.gicp_correspondences(B, len(src))
    r2 = radius * radius
    for b in range(B):
        q = _posed(src, R0[b], t0[b])
        oi, _ = oracle.nn1_radius(q, tgt, radius)
        diff = np.nonzero(oi != g[b])[0]
        for i in diff:  # only the fp32 search radius' margin may differ: a target with r^2 <= d^2 (< 1.0001 r^2)
            assert oi[i] == -1 and g[b][i] >= 0, (b, i, oi[i], g[b][i])
            d2 = ((q[i] - tgt[g[b][i]]) ** 2).sum()
            assert r2 <= d2 <= r2 * 1.001, (b, i, d2)
    return g


@pytest.mark.parametrize("B", [3, 20])  # uniform splits / ordered dispatch (>= 16 starts)
def test_exact_correspondences_c2_size(exact, oracle, B):
    """Pass-0 correspondences of posed C2 starts: the oracle's KD-tree answers, index for index."""
    s, t = _c2()
    rng = np.random.default_rng(1000 + B)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    exact.set_target(t)
    exact.set_source(s)
    exact.reset_stats()
    exact.gicp_batch(R0, t0, max_iteration=0)
    _check_corr(exact, oracle, s, t, R0, t0, 0.5)


def test_exact_ties_resolve_to_lowest_input_index(exact, oracle):
    """Exact fp64 ties (lattice targets, queries at cell/face/edge centres: 8-, 4-
    and 2-way ties, every coordinate and distance exact in fp32 and fp64) go to the
    lowest input index, as KDTree::nn1 does; the fast mode resolves them by
    Morton position instead."""
    h = 0.125
    k = np.arange(-8, 9) * h
    lat = np.stack(np.meshgrid(k, k, k, indexing="ij"), -1).reshape(-1, 3)
    rng = np.random.default_rng(5)
    tgt = lat[rng.permutation(len(lat))]                    # input order != Morton order
    c = (np.arange(-8, 8) + 0.5) * h
    cells = np.stack(np.meshgrid(c, c, c, indexing="ij"), -1).reshape(-1, 3)
    faces = cells.copy()
    faces[:, 2] = np.round(faces[:, 2] / h - 0.5) * h      # z on the lattice: 4-way ties
    edges = faces.copy()
    edges[:, 1] = np.round(edges[:, 1] / h - 0.5) * h      # y too: 2-way ties
    src = np.concatenate([cells, faces, edges])
    src = src[rng.permutation(len(src))]
    exact.set_target(tgt)
    exact.set_source(src)
    R0, t0 = np.eye(3)[None], np.zeros((1, 3))
    exact.gicp_batch(R0, t0, max_iteration=0)
    g = _check_corr(exact, oracle, src, tgt, R0, t0, 0.5)
    d2 = ((src - tgt[g[0]]) ** 2).sum(1)
    assert np.all(np.isin(np.round(d2 / (h * h) * 4), [1, 2, 3]))  # every query tied (2, 4 or 8 ways)


def test_exact_gicp_full_c2_size_matches_oracle(exact, oracle):
    """Three of the bench's posed starts at full C2 size, to convergence: with
    exact correspondences the trajectories are the oracle's (compare
    test_gpu_gicp.py::test_gicp_full_c2_size_posed_starts_match_oracle, whose
    fp32 near-tie flips allow 1e-5 / 2e-4)."""
    s, t = _c2()
    rng = np.random.default_rng(1000)
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(3)])
    t0 = rng.normal(size=(3, 3)) * 0.1
    exact.set_target(t)
    exact.set_source(s)
    exact.reset_stats()
    r = exact.gicp_batch(R0, t0)
    st = exact.stats()
    for b in range(3):
        o = oracle.gicp(np.dot(s, R0[b]) + t0[b], t, 0.5, 100)
        assert r["iters"][b] == o["iters"], (b, r["iters"][b], o["iters"])
        assert abs(r["rmse"][b] - o["rmse"]) <= 1e-12, (b, r["rmse"][b], o["rmse"])
        assert np.abs(r["T"][b] - o["T"]).max() <= 1e-9, (b, np.abs(r["T"][b] - o["T"]).max())
        assert r["ncorr"][b] == o["ncorr"]
    assert 0 < st["exact_filed"] < 0.05 * st["exact_queries"], st  # the band test files a small share


def test_exact_mode_small_pairs_and_multi_target(exact, oracle):
    """Ragged small clouds (not tile multiples), several posed starts, and a
    multi-target batch: per start the oracle's iterations, T to 1e-9."""
    src, tgt = small_pair(1500, 1800, seed=3)
    rng = np.random.default_rng(7)
    B = 6
    R0 = np.array([rot_xyz(*rng.uniform(-90, 90, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.1
    exact.set_target(tgt)
    exact.set_source(src)
    r = exact.gicp_batch(R0, t0)
    for b in range(B):
        o = oracle.gicp(np.dot(src, R0[b]) + t0[b], tgt, 0.5, 100)
        assert r["iters"][b] == o["iters"]
        assert np.abs(r["T"][b] - o["T"]).max() <= 1e-9
        assert abs(r["rmse"][b] - o["rmse"]) <= 1e-12
    # two targets in one batch: each start's result equals its single-target run
    tgt2 = tgt * np.array([1.1, 1.0, 0.95])
    exact.set_targets([tgt, tgt2])
    which = np.array([0, 1, 0, 1, 1, 0], dtype=np.int32)
    rm = exact.gicp_batch_targets(R0, t0, which)
    for b in range(B):
        o = oracle.gicp(np.dot(src, R0[b]) + t0[b], [tgt, tgt2][which[b]], 0.5, 100)
        assert rm["iters"][b] == o["iters"]
        assert np.abs(rm["T"][b] - o["T"]).max() <= 1e-9


def _init(deg, t):
    T = np.eye(4)
    T[:3, :3] = rot_xyz(*deg)
    T[:3, 3] = t
    return T


def test_exact_refinement_p2p_matches_oracle(exact, oracle):
    """PointToPoint ICP (the refinement row) in exact mode: the oracle's
    iterations, T to 1e-9 (its correspondences come from the same search)."""
    from orpcd_amd import Preprocessor
    from workloads import c2_pair
    s, t = c2_pair(20_000)
    s, t = Preprocessor([]).preprocess(s), Preprocessor([]).preprocess(t)
    inits = np.stack([np.eye(4), _init((4, -3, 5), (0.02, 0.0, -0.01)), _init((-10, 8, 3), (0.0, 0.05, 0.0))])
    exact.set_target_points(t)
    exact.set_source_points(s)
    g = exact.icp_p2p_batch(inits, max_correspondence_distance=0.5, max_iteration=60)
    for b in range(len(inits)):
        o = oracle.icp_p2p(s, t, 0.5, inits[b], 60)
        assert g["iters"][b] == o["iters"], (b, g["iters"][b], o["iters"])
        assert np.abs(g["T"][b] - o["T"]).max() <= 1e-9
        assert abs(g["rmse"][b] - o["rmse"]) <= 1e-12


@pytest.mark.parametrize("offset", [1e4, -3e5])
def test_exact_far_from_origin_correspondences(exact, oracle, offset):
    """Clouds far from the world origin (|x| ~ 1e4 .. 3e5, the fp32 frame's
    origin at the target's box centre): the correspondences are still the
    oracle's, index for index."""
    src, tgt = small_pair(3000, 3500, seed=6)
    src, tgt = src + offset, tgt + offset
    rng = np.random.default_rng(2)
    R0 = np.array([rot_xyz(*rng.uniform(-30, 30, 3)) for _ in range(4)])
    ov = np.full(3, offset)
    t0 = np.array([ov - ov @ R for R in R0])  # rotate about the cloud, not the world origin
    exact.set_target(tgt)
    exact.set_source(src)
    exact.gicp_batch(R0, t0, max_iteration=0)
    _check_corr(exact, oracle, src, tgt, R0, t0, 0.5)


def test_exact_row_sharded_gicp_matches_oracle(exact, oracle):
    """One GICP split by source rows over emulated ranks (the C5 path) in exact
    mode: the ranks agree bit for bit and match the oracle's trajectory."""
    from orpcd_amd import _native, parallel
    src, tgt = small_pair(6007, 5003, seed=11)
    ctxs = [_native.Context(0) for _ in range(2)]
    for k, c in enumerate(ctxs):
        c.set_option("exact_nn", 1)
        lo, hi = parallel.shard(len(src), k, 2)
        c.set_target(tgt, 1e-3)
        c.set_source_rows(src, lo, hi)
        c.shard_begin(np.eye(3), np.zeros(3), n_total=len(src), max_correspondence_distance=0.3)
    while True:
        parts = [c.shard_pass() for c in ctxs]
        if not parts[0][1]:
            break
        total = np.sum([s for s, _ in parts], axis=0)
        done = {c.shard_update(total) for c in ctxs}
        if done.pop():
            break
    res = [c.shard_result() for c in ctxs]
    assert np.array_equal(res[0]["T"], res[1]["T"]) and res[0]["rmse"] == res[1]["rmse"]
    o = oracle.gicp(src, tgt, 0.3)
    assert res[0]["iters"] == o["iters"]
    assert np.abs(res[0]["T"] - o["T"]).max() <= 1e-9 and abs(res[0]["rmse"] - o["rmse"]) <= 1e-12
    for c in ctxs:
        c.close()


def test_exact_align_matches_oracle_aligner(oracle):
    """Full Aligner.align (speculative compass, multi-target batches; refine
    off) with GeneralizedICP(exact_nn=True) on a small anisotropic pair: the
    oracle Aligner's decisions, metric and T to round-off."""
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    src, tgt = small_pair(800, 900, seed=6)
    tgt = tgt * np.array([1.15, 1.0, 0.9])
    np.random.seed(0)
    o = oracle.OracleAligner(oracle.OracleGeneralizedICP(), attempts=4)
    To, mo, sfo, eo = o.align(src.copy(), tgt.copy())
    np.random.seed(0)
    al = Aligner(Preprocessor([]), Preprocessor([]), GeneralizedICP(exact_nn=True), attempts=4)
    T, m, sf, e = al.align(src.copy(), tgt.copy(), refine_registration=False)
    assert np.array_equal(sf, sfo) and len(e) == len(eo)
    assert np.abs(np.asarray(e) - np.asarray(eo)).max() <= 1e-12
    assert abs(m - mo) <= 1e-12 and np.abs(T - To).max() <= 1e-9


def test_exact_multi_target_ordered_dispatch(exact, oracle):
    """20 starts over two targets in one batch (the ordered dispatch, >= 16
    starts, as the speculative compass runs): every start is the oracle's."""
    src, tgt = small_pair(2500, 2200, seed=9)
    tgt2 = tgt * np.array([0.95, 1.05, 1.0])
    rng = np.random.default_rng(11)
    B = 20
    R0 = np.array([rot_xyz(*rng.uniform(-60, 60, 3)) for _ in range(B)])
    t0 = rng.normal(size=(B, 3)) * 0.05
    which = (np.arange(B) % 2).astype(np.int32)
    exact.set_source(src)
    exact.set_targets([tgt, tgt2])
    r = exact.gicp_batch_targets(R0, t0, which)
    for b in range(0, B, 3):
        o = oracle.gicp(np.dot(src, R0[b]) + t0[b], [tgt, tgt2][which[b]], 0.5, 100)
        assert r["iters"][b] == o["iters"], (b, r["iters"][b], o["iters"])
        assert np.abs(r["T"][b] - o["T"]).max() <= 1e-9 and abs(r["rmse"][b] - o["rmse"]) <= 1e-12


def test_exact_tiny_clouds_and_iteration_caps(exact, oracle):
    """Edge sizes in exact mode: a 2-point source, a 7-point target (one
    ragged tile), 1 and 3 iterations: the oracle's results to round-off."""
    src, tgt = small_pair(400, seed=5)
    for it in (1, 3):
        exact.set_target(tgt)
        exact.set_source(src)
        r = exact.gicp_batch(np.eye(3)[None], np.zeros((1, 3)), max_iteration=it)
        o = oracle.gicp(src, tgt, 0.5, it)
        assert r["iters"][0] == o["iters"] == it
        assert np.abs(r["T"][0] - o["T"]).max() <= 1e-12 and abs(r["rmse"][0] - o["rmse"]) <= 1e-14
    exact.set_source(src[:2])
    r = exact.gicp_batch(np.eye(3)[None], np.zeros((1, 3)))
    o = oracle.gicp(src[:2], tgt, 0.5, 100)
    assert r["iters"][0] == o["iters"] and np.abs(r["T"][0] - o["T"]).max() <= 1e-9
    exact.set_target(tgt[:7])
    exact.set_source(src)
    r = exact.gicp_batch(np.eye(3)[None], np.zeros((1, 3)), max_iteration=5)
    o = oracle.gicp(src, tgt[:7], 0.5, 5)
    assert r["iters"][0] == o["iters"] and np.abs(r["T"][0] - o["T"]).max() <= 1e-9
    assert abs(r["rmse"][0] - o["rmse"]) <= 1e-12


@pytest.mark.parametrize("m", [1, 7, 8, 9, 63, 64, 65, 71, 127, 129, 4095, 4097])
def test_exact_correspondences_ragged_target_sizes(exact, oracle, m):
    """Every partial-tile shape of the in-tile boxes (8 points since round 4;
    a box without points is stored as the point (3e38, 3e38, 3e38), see
    tile_aabb_kernel): pass-0 correspondences index for index, exact and fp32
    mode (the latter within its tie tolerance: the same d^2 to 2^-17)."""
    rng = np.random.default_rng(m)
    tgt = rng.normal(size=(m, 3)) * 0.3
    src = rng.normal(size=(700, 3)) * 0.3
    R0 = np.array([np.eye(3), rot_xyz(10, -20, 30)])
    t0 = np.array([[0.0, 0.0, 0.0], [0.02, 0.01, -0.03]])
    exact.set_target(tgt)
    exact.set_source(src)
    exact.gicp_batch(R0, t0, max_correspondence_distance=5.0, max_iteration=0)
    _check_corr(exact, oracle, src, tgt, R0, t0, 5.0)
    exact.set_option("exact_nn", 0)
    try:
        exact.gicp_batch(R0, t0, max_correspondence_distance=5.0, max_iteration=0)
        g = exact.gicp_correspondences(2, len(src))
        for b in range(2):
            q = _posed(src, R0[b], t0[b])
            oi, od2 = oracle.nn1_radius(q, tgt, 5.0)
            assert np.all(g[b] >= 0)
            d2 = ((q - tgt[g[b]]) ** 2).sum(1)
            assert np.all(d2 <= od2 * (1 + 2e-5) + 1e-30)
    finally:
        exact.set_option("exact_nn", 1)


@pytest.mark.parametrize("extent", [1.0, 100.0])
@pytest.mark.parametrize("rel", [0.0, 1e-9, 6e-8, 5e-7, 1e-5])
def test_exact_adversarial_near_ties(exact, oracle, extent, rel):
    """Near-ties at and below fp32's resolution: every posed query gets two
    targets on opposite sides at distances r and r (1 + rel s) (s uniform in
    [-1, 1], r in [1e-3, 1e-2] of the extent), among as many random decoys.
    With rel below 2^-24 the fp32 keys cannot order the pair, and with the
    extent at 100 the band's cloud-frame term (4.04 u A) is ~1e4 times the
    distance term: the runner-up tracking, the band test and the fp64
    re-search must still return the oracle's lexicographic (d^2, index)
    minimum, index for index."""
    rng = np.random.default_rng(int(rel * 1e12) + int(extent))
    n = 2500
    src = rng.uniform(-0.5, 0.5, size=(n, 3)) * extent
    R0, t0 = rot_xyz(17.0, -23.0, 41.0)[None], np.array([[0.01, -0.02, 0.03]]) * extent
    q = _posed(src, R0[0], t0[0])
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    r = rng.uniform(1e-3, 1e-2, size=(n, 1)) * extent
    s = rng.uniform(-1.0, 1.0, size=(n, 1))
    near = np.concatenate([q + r * u, q - r * (1.0 + rel * s) * u])
    decoys = rng.uniform(-0.6, 0.6, size=(n, 3)) * extent
    tgt = np.concatenate([near, decoys])
    tgt = tgt[rng.permutation(len(tgt))]
    exact.set_target(tgt)
    exact.set_source(src)
    exact.reset_stats()
    exact.gicp_batch(R0, t0, max_correspondence_distance=0.05 * extent, max_iteration=0)
    st = exact.stats()
    _check_corr(exact, oracle, src, tgt, R0, t0, 0.05 * extent)
    if rel <= 6e-8:  # pairs fp32 cannot order: most queries go to the fp64 re-search
        assert st["exact_filed"] >= n // 2, st
        # ... and the fp32 answers (exact_nn 0) differ from the oracle's for many of
        # them: the case the exact mode exists for
        exact.set_option("exact_nn", 0)
        try:
            exact.gicp_batch(R0, t0, max_correspondence_distance=0.05 * extent, max_iteration=0)
            g = exact.gicp_correspondences(1, n)[0]
        finally:
            exact.set_option("exact_nn", 1)
        oi, _ = oracle.nn1_radius(q, tgt, 0.05 * extent)
        assert (g != oi).sum() >= n // 10, (g != oi).sum()
