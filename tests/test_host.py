"""Host logic of the product package against the reference's golden vectors
(no GPU: the optimizers here are scripted, the native library is not called)."""
import numpy as np
import pytest

from conftest import GOLDEN


class BatchedScripted:
    """optimize_batch twin of ScriptedOptimizer: identical values per attempt."""

    zero_rmse_message = "Optimization failed with loss = 0."

    def __init__(self, inner):
        self.inner = inner
        self.batches = []

    def optimize_batch(self, source, target, R0, t0):
        Ts, rm = [], []
        for R, t in zip(R0, t0):
            T, m = self.inner.optimize(np.dot(source.copy(), R) + t, target)
            Ts.append(T)
            rm.append(m)
        self.batches.append(len(R0))
        n = len(R0)
        return dict(T=np.array(Ts), rmse=np.array(rm), fitness=np.ones(n), iters=np.ones(n, np.int32),
                    ncorr=np.ones(n, np.int64))


def test_rng_replay_matches_reference_G1():
    from orpcd_amd import Aligner, Preprocessor
    g = np.load(f"{GOLDEN}/g1_rng.npz")
    for seed in (0, 1, 42):
        np.random.seed(seed)
        al = Aligner(Preprocessor([]), Preprocessor([]), optimizer=None)
        for n in range(64):
            R, t = al.initialize_rotation()
            assert np.array_equal(R, g[f"R_{seed}"][n]) and np.array_equal(t, g[f"t_{seed}"][n])


@pytest.mark.parametrize("seed,n", [(0, 64), (1, 1), (42, 31), (7, 384)])
def test_draw_block_matches_initialize_rotation(seed, n):
    """The batched draw of a multistart's starts is the reference's sequence of
    initialize_rotation() calls bit for bit (R0, t0 and the RNG state after),
    and the lazily rebuilt per-attempt states equal get_state() after each
    sequential draw (G1 covers the first 64 of seeds 0/1/42 as well)."""
    from orpcd_amd import Aligner, Preprocessor
    al = Aligner(Preprocessor([]), Preprocessor([]), optimizer=None, attempts=n)
    np.random.seed(seed)
    ref, states = [], []
    for _ in range(n):
        ref.append(al.initialize_rotation())
        states.append(np.random.get_state())
    after_ref = np.random.uniform(size=5)
    np.random.seed(seed)
    R0s, t0s, lazy = al._draw_starts()
    after = np.random.uniform(size=5)
    assert np.array_equal(after, after_ref)
    for k in range(n):
        assert np.array_equal(R0s[k], ref[k][0]) and np.array_equal(t0s[k], ref[k][1]), k
    if seed == 0:
        g = np.load(f"{GOLDEN}/g1_rng.npz")
        assert np.array_equal(np.array(R0s), g["R_0"][:n]) and np.array_equal(np.array(t0s), g["t_0"][:n])
    probe = np.random.get_state()
    for k in sorted({0, n // 2, n - 1, -1}):
        st, want = lazy[k], states[k]
        assert st[0] == want[0] and np.array_equal(st[1], want[1]) and st[2:] == want[2:], k
    cur = np.random.get_state()  # rebuilding a state leaves the current stream untouched
    assert np.array_equal(cur[1], probe[1]) and cur[2:] == probe[2:]


def test_preprocess_matches_reference_G2():
    from orpcd_amd import Preprocessor
    from orpcd_amd.Preprocessor.Downsamplers import RandomDownsampler
    from workloads import armadillo
    g = np.load(f"{GOLDEN}/g2_preprocess.npz")
    for name, cloud in zip(("ArmadilloBack_330", "ArmadilloBack_0"), armadillo()):
        np.random.seed(0)
        pp = Preprocessor([RandomDownsampler(5000)])
        out = pp.preprocess(cloud)
        sc = pp.preprocessor_blocks[0]
        assert np.array_equal(out, g[f"{name}_out"])
        assert np.array_equal(sc.mean, g[f"{name}_mean"]) and sc.scale == g[f"{name}_scale"]


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("mode,attempts,seed", [("scripted", 4, 7), ("never_improves", 30, 0), ("constant", 2, 3)])
def test_aligner_matches_reference_G3(mode, attempts, seed, batched):
    from orpcd_amd import Aligner, Preprocessor
    from scripted import ScriptedOptimizer
    g = np.load(f"{GOLDEN}/g3_aligner_trace.npz")
    np.random.seed(seed)
    inner = ScriptedOptimizer(g["goal"], mode=mode)
    opt = BatchedScripted(inner) if batched else inner
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=attempts)
    T, m, sf, err = al.align(g["src"].copy(), g["tgt"].copy(), refine_registration=False)
    assert np.array_equal(T, g[f"{mode}_T"]) and m == g[f"{mode}_metric"]
    assert np.array_equal(sf, g[f"{mode}_sf"]) and np.array_equal(err, g[f"{mode}_errors"])
    assert np.array_equal(np.array([c[2] for c in inner.calls]), g[f"{mode}_call_rmse"])
    assert np.array_equal(np.array([c[1] for c in inner.calls]), g[f"{mode}_call_s0"])
    assert np.array_equal(np.random.uniform(size=4), g[f"{mode}_rng_after"])
    assert al._delta == g[f"{mode}_delta_after"]  # Q3: delta is instance state
    if batched:
        assert all(b == attempts for b in opt.batches)


def test_batched_zero_rmse_raises_like_reference():
    """The reference raises ValueError inside attempt n's optimize(); the RNG
    is then positioned right after attempt n's draws (not after all B)."""
    from orpcd_amd import Aligner, Preprocessor

    class Fails(BatchedScripted):
        def __init__(self):
            self.batches = []

        def optimize_batch(self, source, target, R0, t0):
            n = len(R0)
            rm = np.linspace(1, 2, n)
            rm[2] = 0.0
            return dict(T=np.tile(np.eye(4), (n, 1, 1)), rmse=rm, fitness=np.ones(n), iters=np.ones(n),
                        ncorr=np.ones(n))

    np.random.seed(11)
    al = Aligner(Preprocessor([]), Preprocessor([]), Fails(), attempts=6)
    src = np.random.default_rng(0).normal(size=(20, 3))
    np.random.seed(11)
    with pytest.raises(ValueError):
        al.multistart_registration(src, src)
    after = np.random.uniform(size=3)
    np.random.seed(11)
    for _ in range(3):
        al.initialize_rotation()
    assert np.array_equal(after, np.random.uniform(size=3))


def test_batched_error_hook_raises_the_optimizers_exception():
    """An optimizer's own failure (FastGlobalOptimizer raises Warning when an
    attempt finds no correspondence, fastGlobalOptimizer.py:181-188) replays
    through batch_error: the same exception at attempt n, with the RNG right
    after attempt n's draws; earlier attempts' failures come first."""
    from orpcd_amd import Aligner, Preprocessor

    class NoCorr(BatchedScripted):
        def __init__(self):
            self.batches = []

        def optimize_batch(self, source, target, R0, t0):
            n = len(R0)
            nc = np.full(n, 7, np.int64)
            nc[3] = nc[5] = 0
            return dict(T=np.tile(np.eye(4), (n, 1, 1)), rmse=np.linspace(1, 2, n), fitness=np.ones(n),
                        iters=np.ones(n), ncorr=nc)

        def batch_error(self, table, n):
            return Warning("no correspondences") if table["ncorr"][n] == 0 else None

    al = Aligner(Preprocessor([]), Preprocessor([]), NoCorr(), attempts=8)
    src = np.random.default_rng(1).normal(size=(20, 3))
    np.random.seed(5)
    with pytest.raises(Warning, match="no correspondences"):
        al.multistart_registration(src, src)
    after = np.random.uniform(size=3)
    np.random.seed(5)
    for _ in range(4):
        al.initialize_rotation()
    assert np.array_equal(after, np.random.uniform(size=3))


def test_fgr_batch_table_follows_optimize_conventions():
    """FastGlobalOptimizer's batched records: T with R transposed (as optimize
    returns it), IRLS iterations (0 below 10 tuple correspondences), and
    batch_error's Warning exactly where optimize() would raise (no device)."""
    from orpcd_amd import FastGlobalOptimizer
    opt = FastGlobalOptimizer(iteration_number=64)
    R = np.array([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    T = np.tile(np.eye(4), (2, 1, 1))
    T[0, :3, :3] = R
    T[0, :3, 3] = [1.0, 2.0, 3.0]
    r = dict(T=T, rmse=np.array([0.1, 0.0]), fitness=np.array([0.5, 0.0]), ncorr=np.array([40, 0]),
             n_mutual=np.array([90, 3]), n_tuple_corr=np.array([60, 6]))
    tb = opt._table(r)
    assert np.array_equal(tb["T"][0, :3, :3], R.T) and np.array_equal(tb["T"][0, :3, 3], [1.0, 2.0, 3.0])
    assert list(tb["iters"]) == [64, 0]
    assert opt.batch_error(tb, 0) is None and isinstance(opt.batch_error(tb, 1), Warning)


def test_refine_registration_behaviour():
    from orpcd_amd import Aligner, Preprocessor
    al = Aligner(Preprocessor([]), Preprocessor([]), None)
    with pytest.raises(RuntimeError):  # Q5: PointToPlane without target normals
        al.refine_registration(np.zeros((3, 3)), np.zeros((3, 3)), np.eye(4), icp_type="PointToPlane")


def test_constructor_validation_falls_back_to_defaults():
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    al = Aligner(Preprocessor([]), Preprocessor([]), None, attempts=0, deg=-1, mu=-1, std=0, delta=0,
                 max_iter=0, eps=0)
    assert (al._attempts, al._deg, al._mu, al._std, al._delta, al._max_iter, al._eps) == (
        30, np.pi / 2, 0.0, 0.1, 0.2, 100, 0.05)
    g = GeneralizedICP(max_correspondence_distance=-1, max_iterations=0)
    assert g._max_correspondence_distance == 0.5 and g._max_iterations == 100


def test_shard_covers_every_attempt_once():
    from orpcd_amd.parallel import shard
    for B in (1, 7, 30, 64, 65):
        for W in (1, 2, 3, 8):
            seen = []
            for r in range(W):
                lo, hi = shard(B, r, W)
                seen.extend(range(lo, hi))
            assert seen == list(range(B))


def test_transfrom_matches_reference_formula():
    from orpcd_amd import Aligner, Preprocessor
    rng = np.random.default_rng(0)
    src, tgt = rng.normal(size=(30, 3)), rng.normal(size=(25, 3))
    ps, pt = Preprocessor([]), Preprocessor([])
    s, t = ps.preprocess(src), pt.preprocess(tgt)
    al = Aligner(ps, pt, None)
    al.transfromation = np.eye(4)
    al.transfromation[:3, 3] = [0.1, 0, 0]
    al.scale_factors = np.array([[1.1, 0.9, 1.0]])
    sc_s, sc_t = ps.preprocessor_blocks[0], pt.preprocessor_blocks[0]
    expect = (((src - sc_s.mean) / sc_s.scale) + [0.1, 0, 0]) / al.scale_factors * sc_t.scale + sc_t.mean
    assert np.allclose(al.transfrom(src), expect)


class SpeculativeScripted(BatchedScripted):
    """Adds optimize_batch_multi, which turns on the Aligner's speculative compass."""

    def __init__(self, inner):
        super().__init__(inner)
        self.multi_calls = []

    def optimize_batch_multi(self, source, targets, R0s, t0s):
        self.multi_calls.append(sum(len(r) for r in R0s))
        return [self.optimize_batch(source, tg, r, t) for tg, r, t in zip(targets, R0s, t0s)]


@pytest.mark.parametrize("depth", [None, 1, 2, 3])
@pytest.mark.parametrize("mode,attempts,seed", [("scripted", 4, 7), ("constant", 2, 3)])
def test_speculative_compass_matches_reference_G3(mode, attempts, seed, depth):
    """The speculative compass (the initial multistart with the first compass
    iteration, every iteration's six candidates and `depth` - 1 further
    iterations along the fail path drawn and run up front, the reference's
    order replayed) reproduces the reference's align() exactly: T, metric,
    scale factors, errors, the RNG position and delta (G3).  The scripted
    optimizer is a pure function of its inputs in these modes."""
    from orpcd_amd import Aligner, Preprocessor
    from scripted import ScriptedOptimizer
    g = np.load(f"{GOLDEN}/g3_aligner_trace.npz")
    np.random.seed(seed)
    opt = SpeculativeScripted(ScriptedOptimizer(g["goal"], mode=mode))
    al = Aligner(Preprocessor([]), Preprocessor([]), opt, attempts=attempts, speculative_depth=depth)
    T, m, sf, err = al.align(g["src"].copy(), g["tgt"].copy(), refine_registration=False)
    assert np.array_equal(T, g[f"{mode}_T"]) and m == g[f"{mode}_metric"]
    assert np.array_equal(sf, g[f"{mode}_sf"]) and np.array_equal(err, g[f"{mode}_errors"])
    assert np.array_equal(np.random.uniform(size=4), g[f"{mode}_rng_after"])
    assert al._delta == g[f"{mode}_delta_after"]
    # the replayed multistarts are exactly the reference's calls, in order
    assert len(al.history) * attempts == len(g[f"{mode}_call_rmse"])
    assert np.array_equal(np.concatenate([h["rmse"] for h in al.history]), g[f"{mode}_call_rmse"])
    # one device batch per plan: the initial multistart never runs alone
    assert opt.multi_calls[0] >= 7 * attempts


def test_speculative_plan_follows_the_fail_path():
    """_plan: the initial multistart, then compass iterations along the fail
    path (blocks p .. p+5, then p+6 .. p+11 at delta / 2, same scale factors),
    cut where the reference's loop condition (delta >= eps, iteration <=
    max_iter) stops."""
    from orpcd_amd import Aligner, Preprocessor
    al = Aligner(Preprocessor([]), Preprocessor([]), None, attempts=4, delta=0.2, eps=0.05, max_iter=100)
    sf = np.ones((1, 3))
    items = al._plan(1, sf, 0.2, 0, 3, initial=True)
    assert [b for b, _ in items] == list(range(19))
    assert np.array_equal(items[0][1], np.ones((1, 3)))
    assert np.array_equal(items[1][1], sf + [0.2, 0, 0]) and np.array_equal(items[6][1], sf + [0, 0, -0.2])
    assert np.array_equal(items[7][1], sf + [0.1, 0, 0]) and np.array_equal(items[18][1], sf + [0, 0, -0.05])
    assert len(al._plan(1, sf, 0.05, 0, 3, initial=False)) == 6  # 0.025 < eps: no second iteration
    assert len(al._plan(5, sf, 0.2, 100, 3, initial=False)) == 6  # iteration 101 > max_iter
    assert al._plan(5, sf, 0.2, 101, 3, initial=False) == []


def test_radius_scaler_matches_reference_formula():
    """RadiusScaler (radiusScaler.py:25-30): mean, then max(cdist(center,
    cloud)); the build takes the max of the squared norms before the sqrt and
    must give the same bits."""
    from scipy.spatial.distance import cdist
    from orpcd_amd.Preprocessor.Scalers import RadiusScaler
    rng = np.random.default_rng(3)
    for k in range(20):
        cloud = rng.normal(size=(5000 + 37 * k, 3)) * rng.uniform(1e-3, 1e3) + rng.normal(size=3) * 50
        sc = RadiusScaler()
        out = sc.process(cloud)
        center = np.mean(cloud, axis=0, keepdims=True)
        radius = np.max(cdist(center, cloud))
        assert np.array_equal(sc.mean, center) and sc.scale == radius
        assert np.array_equal(out, (cloud - center) / radius)


@pytest.mark.parametrize("seed", [0, 5, 42])
def test_native_rng_replay_matches_numpy(seed):
    """_native.LegacyDraws (orpcd_rng_draw_attempts) replays numpy's legacy
    RandomState bit for bit: the draws of uniform(low, high, 3) + randn(3) per
    attempt and the state after them, across block sizes (odd counts leave a
    cached gaussian) and from states with and without a cached gaussian."""
    from orpcd_amd._native import LegacyDraws
    rs = np.random.RandomState(seed)
    ld = LegacyDraws(rs.get_state())
    for n in (1, 2, 7, 64, 333, 1000):
        th, g = ld.draw(n, -np.pi / 2, np.pi / 2)
        for k in range(n):
            assert np.array_equal(th[k], rs.uniform(-np.pi / 2, np.pi / 2, 3)), (n, k)
            assert np.array_equal(g[k], rs.randn(3)), (n, k)
        a, b = ld.state(), rs.get_state()
        assert a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2:] == b[2:]


def test_generalized_icp_sets_its_search_mode_on_the_shared_context():
    """GeneralizedICP(exact_nn=...) selects the search mode on the process-wide
    context every time it hands the context out, so two optimizers with
    different modes can share it (bench.py runs both)."""
    from orpcd_amd import GeneralizedICP

    class FakeCtx:
        def __init__(self):
            self.options = []

        def set_option(self, key, value):
            self.options.append((key, value))

    fake = FakeCtx()
    fast, exact = GeneralizedICP(exact_nn=False), GeneralizedICP()  # exact is the default
    fast._ctx = exact._ctx = fake
    assert exact.context is fake and fake.options[-1] == ("exact_nn", 1)
    assert fast.context is fake and fake.options[-1] == ("exact_nn", 0)


def test_generalized_icp_drop_in_reuses_rigid_images():
    """GeneralizedICP.optimize called once per attempt (the reference's own
    Aligner, Aligner.py:183-190): a source that is a rigid image of the last
    cloud runs on that cloud's cached device layout with the recovered pose;
    anything else (deformed, reordered) becomes the new base."""
    from orpcd_amd import GeneralizedICP
    from workloads import rot_xyz, small_pair

    class FakeCtx:
        def __init__(self):
            self.sources, self.poses = [], []

        def set_option(self, key, value):
            pass

        def set_target(self, xyz, eps):
            pass

        def set_source(self, xyz):
            self.sources.append(xyz)

        def source_ties(self):
            return dict(n_ties=0, rows=np.zeros(0, np.int64), complete=True)

        def gicp_batch(self, R0, t0, **kw):
            self.poses.append((R0[0].copy(), t0[0].copy()))
            return dict(T=np.eye(4)[None], rmse=np.array([0.5]))

    src, tgt = small_pair(500, seed=3)
    opt = GeneralizedICP(speculate=0)
    fake = opt._ctx = FakeCtx()
    fake._target_key = None
    opt.optimize(src, tgt)
    R0, t0 = rot_xyz(30, -40, 70), np.array([0.1, -0.2, 0.05])
    posed = np.dot(src.copy(), R0) + t0                # Aligner.py:183-185
    T, rmse = opt.optimize(posed, tgt)
    assert fake.sources[1] is fake.sources[0]         # the cached base, not the posed copy
    R, t = fake.poses[1]
    assert np.abs(R - R0).max() < 1e-13 and np.abs(t - t0).max() < 1e-13
    bent = posed.copy()
    bent[7] += 1e-6                                   # not rigid: a new base
    opt.optimize(bent, tgt)
    assert fake.sources[2] is not fake.sources[0] and np.array_equal(fake.sources[2], bent)
    assert np.array_equal(fake.poses[2][0], np.eye(3))
    opt.optimize(posed[::-1].copy(), tgt)             # reordered: a new base
    assert np.array_equal(fake.poses[3][0], np.eye(3))
    off = GeneralizedICP(rigid_cache=False)
    fake2 = off._ctx = FakeCtx()
    fake2._target_key = None
    off.optimize(src, tgt)
    off.optimize(posed, tgt)
    assert np.array_equal(fake2.sources[1], posed) and np.array_equal(fake2.poses[1][0], np.eye(3))


def test_generalized_icp_drop_in_speculates_the_callers_draws():
    """The drop-in path over the reference-shaped Aligner (one optimize() per
    attempt): from the second call on, the plugin predicts the caller's next
    draws from np.random's state (without advancing it) and runs them as one
    batch; every later call is served from that batch only after its source
    is verified to be the predicted pose.  The results per call are those of
    the call's own pose; np.random ends where the reference leaves it.  With
    draws the model does not predict (deg pi/3) no chain is ever confirmed,
    so nothing runs ahead."""
    import math

    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import small_pair

    class FakeCtx:  # rmse = a function of the start's posed cloud
        def __init__(self):
            self.batches = []
            self._target_key = None

        def set_option(self, key, value):
            pass

        def set_target(self, xyz, eps):
            self._target_key = (xyz.shape, float(xyz.sum()))

        def set_source(self, xyz):
            self.base = xyz

        def source_ties(self):
            return dict(n_ties=0, rows=np.zeros(0, np.int64), complete=True)

        def gicp_batch(self, R0, t0, **kw):
            self.batches.append(len(R0))
            rm = np.array([0.1 + float(np.abs(self.base @ R + t).sum()) * 1e-6 for R, t in zip(R0, t0)])
            return dict(T=np.repeat(np.eye(4)[None], len(R0), 0), rmse=rm)

    class OnlyOptimize:
        def __init__(self, inner):
            self.inner, self.rmse, self.expect = inner, [], []

        def optimize(self, source, target, **kw):
            T, m = self.inner.optimize(source, target, **kw)
            self.rmse.append(m)
            self.expect.append(0.1 + float(np.abs(source).sum()) * 1e-6)  # the call's own pose
            return T, m

    src, tgt = small_pair(400, seed=5)
    # deg pi/2: the model's draws; two multistarts re-seeded between them (the
    # second's first call is unpredictable: the leftover predictions of the
    # first are checked, found wrong and dropped; the second's chain is
    # confirmed at its third call).  deg pi/3: never confirmed.
    for deg, batches, served, missed in ((math.pi / 2, [1, 1, 30, 1, 1, 30], 27 + 27, 1),
                                         (math.pi / 3, [1] * 60, 0, 0)):
        opt = GeneralizedICP()
        fake = opt._ctx = FakeCtx()
        plug = OnlyOptimize(opt)
        al = Aligner(Preprocessor([]), Preprocessor([]), plug, attempts=30, deg=deg)
        for seed in (7, 8):
            np.random.seed(seed)
            al.multistart_registration(src, tgt)
            after = np.random.get_state()
            np.random.seed(seed)
            for _ in range(30):
                al.initialize_rotation()
            ref = np.random.get_state()
            assert np.array_equal(after[1], ref[1]) and after[2:] == ref[2:]  # the stream is not advanced
        assert opt.spec_stats["served"] == served and opt.spec_stats["missed"] == missed, opt.spec_stats
        assert fake.batches == batches, fake.batches
        assert np.allclose(plug.rmse, plug.expect, rtol=0, atol=1e-12)
    # an align()-like sequence: each multistart on a new (scaled) cloud, the
    # stream never re-seeded -- a confirmed chain that ends on a new cloud is
    # followed at once (its first call already runs the batch)
    opt = GeneralizedICP()
    fake = opt._ctx = FakeCtx()
    plug = OnlyOptimize(opt)
    al = Aligner(Preprocessor([]), Preprocessor([]), plug, attempts=30)
    np.random.seed(9)
    for k in range(3):
        al.multistart_registration(src * (1.0 + 0.1 * k), tgt)
    assert fake.batches == [1, 1, 30, 30, 30], fake.batches  # the attempts learned from the first switch
    assert opt.spec_stats["missed"] == 0 and np.allclose(plug.rmse, plug.expect, rtol=0, atol=1e-12)


def test_posed_rows_match_numpy():
    """orpcd_pose_rows (the posing the batch applies to boundary-tie rows) is
    numpy's np.dot(source, R0) + t0 bit for bit (Aligner.py:183-185): the
    oracle fixtures' inputs were formed by numpy, so the tie decisions see the
    same coordinates.  All 870 starts of the complete C1 align() fixture, on
    the C1-like cloud and a cloud far from the origin; and row subsets."""
    from orpcd_amd import _native
    z = np.load(f"{GOLDEN}/g7_align_c1.npz")
    rng = np.random.default_rng(11)
    for cloud in (rng.standard_normal((3000, 3)) * 0.3, rng.standard_normal((500, 3)) * 50.0 + 1e3):
        for R, t in zip(z["R0"], z["t0"]):
            assert np.array_equal(_native.pose_rows(cloud, R, t), np.dot(cloud, R) + t)
        idx = rng.integers(0, len(cloud), 37)
        assert np.array_equal(_native.pose_rows(cloud, z["R0"][5], z["t0"][5], idx),
                              (np.dot(cloud, z["R0"][5]) + z["t0"][5])[idx])


def test_generalized_icp_drop_in_hands_over_posed_tie_rows():
    """With KNN-20 boundary ties on the source (orpcd_source_ties), the
    drop-in path hands the device each call's OWN posed coordinates of the tie
    rows (the copy Open3D would re-estimate the covariances on,
    generalizedICP.py:54-70); a predicted start (posed from the cached base)
    is served only if its tie decisions equal the ones the call's own
    coordinates give, else the call runs alone with its rows."""
    from orpcd_amd import Aligner, GeneralizedICP, Preprocessor
    from workloads import small_pair

    rows = np.array([3, 17, 40, 41, 99])

    def decide(P):  # a tie decision that flips on the last bits of the posed rows
        return np.array([[int(np.ascontiguousarray(P).view(np.int64).sum() & 3)] * 20], np.int32)

    class FakeCtx:
        def __init__(self):
            self.batches, self.given, self.last = [], [], []
            self._target_key = None
            self.posed = None

        def set_option(self, key, value):
            pass

        def set_target(self, xyz, eps):
            self._target_key = (xyz.shape, float(xyz.sum()))

        def set_source(self, xyz):
            self.base = xyz

        def source_ties(self):
            return dict(n_ties=1, rows=rows, complete=True)

        def set_posed_tie_rows(self, xyz):
            self.posed = None if xyz is None else np.array(xyz)

        def gicp_batch(self, R0, t0, **kw):
            B = len(R0)
            P = self.posed if self.posed is not None else np.full((B, len(rows), 3), np.nan)
            assert len(P) == B
            self.posed = None
            self.last = []
            for b in range(B):
                pb = P[b] if np.isfinite(P[b, 0, 0]) else np.dot(self.base[rows], R0[b]) + t0[b]
                self.last.append(decide(pb))
            self.given.append(P)
            self.batches.append(B)
            # rmse: the start's pose and its tie decision
            rm = np.array([0.1 + float(np.abs(self.base @ R + t).sum()) * 1e-6 + 1e-3 * self.last[b][0, 0]
                           for b, (R, t) in enumerate(zip(R0, t0))])
            return dict(T=np.repeat(np.eye(4)[None], B, 0), rmse=rm)

        def tie_sets(self, b=-1, posed_rows=None, n_ties=None):
            return decide(posed_rows) if posed_rows is not None else self.last[b]

    class OnlyOptimize:
        def __init__(self, inner):
            self.inner, self.rmse, self.expect = inner, [], []

        def optimize(self, source, target, **kw):
            T, m = self.inner.optimize(source, target, **kw)
            self.rmse.append(m)
            self.expect.append(0.1 + float(np.abs(source).sum()) * 1e-6 + 1e-3 * decide(source[rows])[0, 0])
            return T, m

    src, tgt = small_pair(400, seed=5)
    opt = GeneralizedICP()
    fake = opt._ctx = FakeCtx()
    plug = OnlyOptimize(opt)
    al = Aligner(Preprocessor([]), Preprocessor([]), plug, attempts=30)
    np.random.seed(7)
    al.multistart_registration(src, tgt)
    st = opt.spec_stats
    assert st["served"] + st["tie_reruns"] == 27 and st["tie_reruns"] > 0, st
    # every call got its own coordinates' decision, served or re-run
    assert np.allclose(plug.rmse, plug.expect, rtol=0, atol=1e-12)
    # direct calls (and re-runs) handed over exactly their own rows
    assert all(np.isfinite(g[0]).all() for g in fake.given)
