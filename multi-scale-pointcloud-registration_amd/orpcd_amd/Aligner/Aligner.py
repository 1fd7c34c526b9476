"""Aligner — the outer compass (pattern) search over (sx, sy, sz).

Reference: or_pcd/Aligner/Aligner.py:32-408.  Same constructor, defaults,
validation, RNG consumption (global legacy ``np.random``: three
``uniform`` + one ``randn(3)`` per attempt, Aligner.py:129-160), the same
composition T = [R0·Rc, t0·Rc + tc] (:192-202), the strict ``<`` over
attempts (:192) and the ``<=`` acceptance / δ-halving of the compass (:263-298),
including the reference's stateful δ (Q3).

What is different is HOW a multistart runs: when the optimizer offers
``optimize_batch`` (the build's GeneralizedICP), all attempts of one scale run
as one device batch, sharded over the ranks of an initialised
``torch.distributed`` group (``orpcd_amd.parallel``), and the per-attempt
records are replayed through the reference's selection loop in attempt order.
Any other IOptimizer (including the reference's own) is called per attempt,
exactly as the reference does.

With a batched optimizer the compass search is also speculative
(``speculative_compass=True``, keyword-only).  Every multistart the reference
evaluates draws the next ``attempts`` starts of one RNG stream, so the
stream is a sequence of blocks whatever the search decides; the build draws
them once (``_Tape``), runs the multistarts the reference MAY evaluate next
(the initial multistart with the first compass iteration, then each compass
iteration's six candidates, optionally followed along the "all six fail"
path by the next iteration at delta / 2: ``speculative_depth``) as one
device batch, and replays the reference's decisions in order.  Results, the
RNG position and delta are identical to the sequential search.
"""
import copy
import time
from typing import List, Tuple

import numpy as np

from .. import _native, parallel
from ..Optimizer.iOptimizer import IOptimizer
from ..Preprocessor.Scalers.BaseScaler import BaseScaler
from ..utils.constants import (
    __ALIGNER_DEG__,
    __ALIGNER_DELTA__,
    __ALIGNER_EPS__,
    __ALIGNER_MAX_ITER__,
    __ALIGNER_MU__,
    __ALIGNER_STD__,
    __MULTISTART_ATTEMPTS__,
    __REFINER_DISTANCE_THRESHOLD__,
    __REFINER_MAX_ITER__,
)
from ..utils.logger_factory import LoggerFactory


def draw_block(n: int, deg: float, mu: float, std: float, rs=None):
    """n consecutive initialize_rotation() draws (Aligner.py:125-162) of an
    Aligner with (deg, mu, std), bit for bit: the same stream consumption
    (three uniform, then randn(3), per attempt) and the same translation
    expression; the cos / sin of all 3n
    angles by one ufunc call each and the n products r_1 (r_2 r_3) by one
    stacked matmul, which give the scalar calls' and np.dot's values
    (checked against the sequential draws in
    tests/test_host.py::test_draw_block_matches_initialize_rotation).
    rs: the global legacy RandomState (default; advanced through numpy's
    API), another RandomState, or a _native.LegacyDraws (the same stream
    replayed in C++, ~25 ns instead of ~4.6 us per attempt)."""
    if isinstance(rs, _native.LegacyDraws):
        th, g = rs.draw(n, -deg, deg)
    else:
        rs = np.random if rs is None else rs
        uni, randn = rs.uniform, rs.randn
        th = np.empty((n, 3))
        g = np.empty((n, 3))
        for k in range(n):
            # uniform(size=3) consumes the stream as three scalar uniform()
            # calls and returns the same values (low + (high - low) * double);
            # the Gaussians stay one randn(3) per attempt (its cached second
            # deviate makes the order matter)
            th[k] = uni(-deg, deg, 3)
            g[k] = randn(3)
    t0s = list(mu + g * std)  # elementwise, as per attempt
    c, s = np.cos(th), np.sin(th)
    r = np.zeros((3, n, 3, 3))
    r[0, :, 0, 0] = 1.0
    r[0, :, 1, 1], r[0, :, 1, 2], r[0, :, 2, 1], r[0, :, 2, 2] = c[:, 0], -s[:, 0], s[:, 0], c[:, 0]
    r[1, :, 1, 1] = 1.0
    r[1, :, 0, 0], r[1, :, 0, 2], r[1, :, 2, 0], r[1, :, 2, 2] = c[:, 1], s[:, 1], -s[:, 1], c[:, 1]
    r[2, :, 2, 2] = 1.0
    r[2, :, 0, 0], r[2, :, 0, 1], r[2, :, 1, 0], r[2, :, 1, 1] = c[:, 2], -s[:, 2], s[:, 2], c[:, 2]
    R = np.matmul(r[0], np.matmul(r[1], r[2]))
    return list(R), t0s


class Aligner:
    transfromation: np.ndarray = np.eye(4)
    scale_factors: np.ndarray = np.ones((1, 3))

    def __init__(self, source_preprocessor, target_preprocessor, optimizer: IOptimizer,
                 attempts: int = __MULTISTART_ATTEMPTS__, deg: float = __ALIGNER_DEG__, mu: float = __ALIGNER_MU__,
                 std: float = __ALIGNER_STD__, delta: float = __ALIGNER_DELTA__, max_iter: int = __ALIGNER_MAX_ITER__,
                 eps: float = __ALIGNER_EPS__, visualize_intermediate_steps: bool = False, *,
                 speculative_compass: bool = True, speculative_depth: int = None, shard_interleave: bool = False):
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)
        checks = [("attempts", attempts, lambda v: v <= 0, __MULTISTART_ATTEMPTS__),
                  ("deg", deg, lambda v: v <= 0, __ALIGNER_DEG__),
                  ("mu", mu, lambda v: v < 0, __ALIGNER_MU__),
                  ("std", std, lambda v: v <= 0, __ALIGNER_STD__),
                  ("delta", delta, lambda v: v <= 0, __ALIGNER_DELTA__),
                  ("max_iter", max_iter, lambda v: v <= 0, __ALIGNER_MAX_ITER__),
                  ("eps", eps, lambda v: v <= 0, __ALIGNER_EPS__)]
        vals = {}
        for name, v, bad, default in checks:  # Aligner.py:69-116
            if bad(v):
                self._LOG.warning(f"{name} cannot be 0 or less. Provided: {v}")
                v = default
            vals[name] = v
        self._attempts = vals["attempts"]
        self._deg = vals["deg"]
        self._mu = vals["mu"]
        self._std = vals["std"]
        self._delta = vals["delta"]
        self._max_iter = vals["max_iter"]
        self._eps = vals["eps"]
        self._visualize_intermediate_steps = visualize_intermediate_steps
        self._source_preprocessor = source_preprocessor
        self._target_preprocessor = target_preprocessor
        self._optimizer = optimizer
        # instrumentation (not in the reference): per-multistart records
        self.history: List[dict] = []
        self.last_refine = None
        self._refine_ctx = None  # device context for refine_registration when the optimizer has none
        self._speculative_compass = speculative_compass
        # compass iterations per device batch along the "all six fail" path:
        # None = 2 when a one-iteration batch per device is small (<= 96 starts
        # of 50k points: latency-bound, so a second iteration is nearly free),
        # else 1
        self._speculative_depth = speculative_depth
        self._shard_interleave = shard_interleave
        self.speculative_history: List[dict] = []  # candidates run ahead but not reached by the reference's order

    # ----------------------------------------------------------------- RNG
    def initialize_rotation(self) -> Tuple[np.ndarray, np.ndarray]:
        """Aligner.py:125-162 (bit-identical draws and matrix products)."""
        theta_1 = np.random.uniform(low=-self._deg, high=self._deg)
        theta_2 = np.random.uniform(low=-self._deg, high=self._deg)
        theta_3 = np.random.uniform(low=-self._deg, high=self._deg)
        r_1 = np.array([[1, 0, 0], [0, np.cos(theta_1), -np.sin(theta_1)], [0, np.sin(theta_1), np.cos(theta_1)]])
        r_2 = np.array([[np.cos(theta_2), 0, np.sin(theta_2)], [0, 1, 0], [-np.sin(theta_2), 0, np.cos(theta_2)]])
        r_3 = np.array([[np.cos(theta_3), -np.sin(theta_3), 0], [np.sin(theta_3), np.cos(theta_3), 0], [0, 0, 1]])
        rotation_matrix = np.dot(r_1, np.dot(r_2, r_3))
        translation = self._mu + np.random.randn(3) * self._std
        return rotation_matrix, translation

    # ----------------------------------------------------------- multistart
    def multistart_registration(self, source: np.ndarray, target: np.ndarray) -> Tuple[np.ndarray, float]:
        if hasattr(self._optimizer, "optimize_batch"):
            return self._multistart_batched(source, target)
        return self._multistart_sequential(source, target)

    def _multistart_sequential(self, source, target):
        """Aligner.py:164-204 verbatim in behaviour (one optimize per attempt)."""
        metric = np.inf
        best_transformation = np.eye(4)
        for _ in range(self._attempts):
            source_copy = copy.deepcopy(source)
            initial_rotation, initial_translation = self.initialize_rotation()
            source_initialized = np.dot(source_copy, initial_rotation) + initial_translation
            current_transform, current_metric = self._optimizer.optimize(source_initialized, target)
            if current_metric < metric:
                metric = current_metric
                best_transformation = self._compose(initial_rotation, initial_translation, current_transform)
        return best_transformation, metric

    @staticmethod
    def _compose(R0, t0, Tc):
        """Aligner.py:196-201."""
        T = np.eye(4)
        T[:3, :3] = np.dot(R0, Tc[:3, :3])
        T[:3, 3] = np.dot(t0, Tc[:3, :3]).ravel() + Tc[:3, 3]
        return T

    def _draw_block(self, n: int, rs=None):
        """n consecutive initialize_rotation() draws of this Aligner (draw_block)."""
        return draw_block(n, self._deg, self._mu, self._std, rs)

    class _BlockStates:
        """The RNG state after attempt n of a drawn block, rebuilt on demand:
        [-1] is the state after the whole block (kept); any other n (needed only
        when attempt n fails, Aligner.py:188-190 raising inside optimize) is
        reached by replaying the block's first n + 1 draws from the state before
        it.  One get_state per block instead of one per attempt (~60 us each)."""

        def __init__(self, aligner, before, after, n):
            self._al, self._before, self._after, self._n = aligner, before, after, n

        def __getitem__(self, k):
            k = k + self._n if k < 0 else k
            if k == self._n - 1:
                return self._after
            cur = np.random.get_state()
            np.random.set_state(self._before)
            for _ in range(k + 1):
                self._al.initialize_rotation()
            st = np.random.get_state()
            np.random.set_state(cur)
            return st

    def _draw_starts(self):
        """The attempts' (R0, t0) in the reference's order, and the RNG state after each."""
        before = np.random.get_state()
        rs = _native.LegacyDraws(before)
        R0s, t0s = self._draw_block(self._attempts, rs)  # same draws, same order as the sequential loop
        after = rs.state()
        np.random.set_state(after)
        return R0s, t0s, Aligner._BlockStates(self, before, after, self._attempts)

    def _positions(self, K):
        """Flat-list positions of the K multistarts' B attempts each: target-major
        blocks (k * B + a), or interleaved (a * K + k, shard_interleave=True)."""
        B = self._attempts
        if self._shard_interleave:
            return [k + K * np.arange(B) for k in range(K)]
        return [k * B + np.arange(B) for k in range(K)]

    def _run_tables(self, source, targets, draws, keys=None):
        """Per target k, the gathered per-attempt table of the starts draws[k].
        The K tables are sharded as ONE flat list of K x B starts: this rank
        runs its contiguous block of positions as one batch
        (optimize_batch_multi when it spans several targets); one all-gather
        of the flat table follows.  Positions are target-major by default, so
        a rank's block touches one or two targets rather than all K (it sets
        up only those); with shard_interleave they are attempt-major, so every
        rank runs an equal slice of every multistart (all K targets) and
        costly candidates spread over the ranks.  `keys` (the multistarts'
        (block, scale) identities) is for instrumentation only."""
        B, K = self._attempts, len(draws)
        rank, ws = parallel.world()
        lo, hi = parallel.shard(K * B, rank, ws)
        pos = self._positions(K)
        local = np.zeros((0, parallel.REC))
        if hi > lo:
            ks, R0, t0, sel = [], [], [], []
            for k in range(K):
                at = np.nonzero((pos[k] >= lo) & (pos[k] < hi))[0]  # this rank's attempts of multistart k
                if len(at):
                    ks.append(k)
                    sel.append(pos[k][at])
                    R0.append(np.array([draws[k][0][i] for i in at]))
                    t0.append(np.array([draws[k][1][i] for i in at]))
            tg = targets(ks) if callable(targets) else [targets[k] for k in ks]
            if len(tg) > 1 and hasattr(self._optimizer, "optimize_batch_multi"):
                res = self._optimizer.optimize_batch_multi(source, tg, R0, t0)
            else:
                res = [self._optimizer.optimize_batch(source, g, r, t) for g, r, t in zip(tg, R0, t0)]
            local = np.zeros((hi - lo, parallel.REC))
            for p_k, r in zip(sel, res):
                local[p_k - lo] = parallel.pack(r)
        table = parallel.allgather_records(local, K * B)
        return [parallel.unpack(table[pos[k]]) for k in range(K)]

    def _select(self, table, draw):
        """Aligner.py:178-202 over a finished table, in attempt order: strict <,
        and the exception optimize() raises for a failed attempt (the
        optimizer's batch_error: GeneralizedICP's ValueError on rmse == 0,
        FastGlobalOptimizer's Warning without correspondences), with the RNG
        left after the failing attempt's draw."""
        R0s, t0s, states = draw
        metric = np.inf
        best_transformation = np.eye(4)
        batch_error = getattr(self._optimizer, "batch_error", None)
        for n in range(self._attempts):
            current_metric = float(table["rmse"][n])
            if batch_error is not None:
                err = batch_error(table, n)
            elif current_metric == 0 and hasattr(self._optimizer, "zero_rmse_message"):
                err = ValueError(self._optimizer.zero_rmse_message)
            else:
                err = None
            if err is not None:
                # the reference raises inside optimize() of attempt n, before
                # drawing attempt n+1: leave the RNG exactly there
                np.random.set_state(states[n])
                raise err
            if current_metric < metric:
                metric = current_metric
                best_transformation = self._compose(R0s[n], t0s[n], table["T"][n])
        return best_transformation, metric

    def _multistart_batched(self, source, target):
        draw = self._draw_starts()
        t_start = time.perf_counter()
        table = self._run_tables(source, [target], [draw])[0]
        self.history.append(dict(B=self._attempts, seconds=time.perf_counter() - t_start,
                                 iters=int(table["iters"].sum()), rmse=table["rmse"].copy(),
                                 iters_per_start=table["iters"].copy()))
        return self._select(table, draw)

    def _scaled_targets(self, target, scales):
        """[target * s for s in scales] (s of shape (1, 3)) as consecutive views
        of one contiguous block that is reused across calls: the products are
        taken column by column, elementwise as the broadcast product (the
        broadcast over rows of 3 and fresh 1.2 MB allocations cost ~1 ms per
        50k-point candidate; this ~0.1 ms).  An optimizer keeping a reference
        to a target past its call must copy it (ours key their caches on the
        content)."""
        target = np.asarray(target, dtype=np.float64)
        shape = (len(scales),) + target.shape
        buf = getattr(self, "_scaled_buf", None)
        if buf is None or buf.shape[1:] != target.shape or buf.shape[0] < len(scales):
            buf = self._scaled_buf = np.empty((max(len(scales), 6),) + target.shape)
        out = buf[: shape[0]]
        for k, s in enumerate(scales):
            s = np.asarray(s, dtype=np.float64).reshape(-1)
            for c in range(target.shape[1]):
                np.multiply(target[:, c], s[c], out=out[k, :, c])
        return [out[k] for k in range(len(scales))]

    class _Tape:
        """The reference's RNG stream as consecutive multistart blocks.

        Every multistart the reference evaluates draws the next ``attempts``
        starts (Aligner.py:178-186), whichever compass candidate it belongs
        to: block 0 is the initial multistart (:245), a compass iteration at
        block position p draws blocks p .. p+5 for +x, -x, +y, -y, +z, -z
        (:270-297) as far as it gets; accepting candidate k moves the position
        to p+k+1, failing all six to p+6.  Blocks are drawn once, in stream
        order, by the native replay of numpy's legacy generator
        (_native.LegacyDraws) from the global state at align() entry;
        ``state_after`` gives the global state the reference leaves after a
        block."""

        def __init__(self, aligner):
            self._al = aligner
            self._rs = _native.LegacyDraws(np.random.get_state())
            self._states = [self._rs.state()]  # [j]: the state before block j
            self._blocks = []

        def _extend(self, j):
            while len(self._blocks) <= j:
                self._blocks.append(self._al._draw_block(self._al._attempts, self._rs))
                self._states.append(self._rs.state())

        def draw(self, j):
            """Block j as _draw_starts returns it: (R0s, t0s, per-attempt states)."""
            self._extend(j)
            R0s, t0s = self._blocks[j]
            return R0s, t0s, Aligner._BlockStates(self._al, self._states[j], self._states[j + 1], self._al._attempts)

        def state_after(self, j):
            self._extend(j)
            return self._states[j + 1]

    def _compass_steps(self, delta):
        """The candidate steps of one compass iteration in the reference's order
        +x, -x, +y, -y, +z, -z (Aligner.py:270-291: delta * e_axis, -delta * e_axis)."""
        directions = np.eye(3)
        return [sign * delta * directions[:, axis] for axis in range(3) for sign in (1.0, -1.0)]

    def _depth(self, n_points):
        if self._speculative_depth is not None:
            return max(1, int(self._speculative_depth))
        _, ws = parallel.world()
        return 2 if 6 * self._attempts * n_points <= 96 * 50_000 * ws else 1

    def _plan(self, pos, scale_factors, delta, iteration, depth, initial):
        """The multistarts (block, target scale) the reference may evaluate
        next from this state: the initial multistart if pending, then `depth`
        compass iterations along the fail path (delta halving, scale factors
        unchanged) while the reference's loop condition holds."""
        items = [(0, np.ones((1, 3)))] if initial else []
        for _ in range(depth):
            if not (delta >= self._eps and iteration <= self._max_iter):  # Aligner.py:262
                break
            items.extend((pos + k, scale_factors + step) for k, step in enumerate(self._compass_steps(delta)))
            pos, iteration, delta = pos + 6, iteration + 1, delta / 2
        return items

    def _align_speculative(self, source, target):
        """Aligner.py:245-298 (initial multistart + compass search) over planned
        device batches.  Returns (T, metric, scale factors, errors) and leaves
        np.random and delta exactly where the reference leaves them."""
        tape = Aligner._Tape(self)
        depth = self._depth(len(source))
        done = {}  # (block, scale bytes) -> (table, seconds)
        used = set()

        def run(items):
            draws = [tape.draw(b) for b, _ in items]
            t_start = time.perf_counter()
            tables = self._run_tables(
                source, lambda ks: self._scaled_targets(target, [items[k][1] for k in ks]), draws,
                keys=[(b, sc.tobytes()) for b, sc in items])
            sec = (time.perf_counter() - t_start) / len(items)
            for (b, sc), tb in zip(items, tables):
                done[(b, sc.tobytes())] = (tb, sec)

        def select(block, scale):
            key = (block, scale.tobytes())
            table, sec = done[key]
            used.add(key)
            self.history.append(dict(B=self._attempts, seconds=sec, iters=int(table["iters"].sum()),
                                     rmse=table["rmse"].copy(), iters_per_start=table["iters"].copy()))
            return self._select(table, tape.draw(block))

        scale_factors = np.ones((1, 3))
        iteration, pos = 0, 1
        try:
            run(self._plan(1, scale_factors, self._delta, iteration, depth, initial=True))
            start = time.time()
            transformation, metric = select(0, np.ones((1, 3)))
            self._LOG.info(f"Multi-start registration time: {time.time() - start}")
            errors = [metric]
            while self._delta >= self._eps and iteration <= self._max_iter:
                iteration += 1
                steps = self._compass_steps(self._delta)
                if any((pos + k, (scale_factors + st).tobytes()) not in done for k, st in enumerate(steps)):
                    run(self._plan(pos, scale_factors, self._delta, iteration - 1, depth, initial=False))
                for k, step in enumerate(steps):
                    new_transformation, new_metric = select(pos + k, scale_factors + step)
                    if new_metric <= metric:  # Aligner.py:273,287
                        metric, transformation = new_metric, new_transformation
                        scale_factors += step
                        errors.append(new_metric)
                        pos += k + 1
                        break
                else:
                    pos += 6
                if new_metric > metric:  # Aligner.py:296-297
                    self._delta = self._delta / 2
            np.random.set_state(tape.state_after(pos - 1))
        finally:
            self.speculative_history.extend(dict(B=self._attempts, iters=int(tb["iters"].sum()))
                                            for key, (tb, _) in done.items() if key not in used)
        return transformation, metric, scale_factors, errors

    # -------------------------------------------------------------- compass
    def compass_step(self, source, target, scale_factors, delta):
        """Aligner.py:206-226."""
        new_scale_factors = scale_factors + delta
        target_scaled = target * new_scale_factors
        current_rotation, current_metric = self.multistart_registration(source, target_scaled)
        return new_scale_factors, current_rotation, current_metric

    def align(self, source: np.ndarray, target: np.ndarray, refine_registration: bool = True,
              icp_type: str = "PointToPlane") -> Tuple[np.ndarray, float, np.ndarray, List[float]]:
        """Aligner.py:228-317."""
        source = self._source_preprocessor.preprocess(source)
        target = self._target_preprocessor.preprocess(target)
        # speculation needs an optimizer whose result is a pure function of its
        # inputs and that can run several targets at once (optimize_batch_multi)
        if self._speculative_compass and hasattr(self._optimizer, "optimize_batch_multi"):
            optimal_transformation, optimal_metric, optimal_scale_factors, errors = self._align_speculative(
                source, target)
            return self._finish(source, target, optimal_transformation, optimal_metric, optimal_scale_factors,
                                errors, refine_registration, icp_type)
        iteration = 0
        optimal_scale_factors = np.ones((1, 3))
        start = time.time()
        optimal_transformation, optimal_metric = self.multistart_registration(source, target)
        self._LOG.info(f"Multi-start registration time: {time.time() - start}")
        errors = [optimal_metric]
        directions = np.eye(3)
        while self._delta >= self._eps and iteration <= self._max_iter:
            iteration += 1
            for axis in range(3):
                scale_plus = self._delta * directions[:, axis]
                new_scale_factors, new_rotation, new_metric = self.compass_step(
                    source, target, optimal_scale_factors, scale_plus)
                if new_metric <= optimal_metric:
                    optimal_metric = new_metric
                    optimal_transformation = new_rotation
                    optimal_scale_factors += scale_plus
                    errors.append(new_metric)
                    break
                scale_neg = -self._delta * directions[:, axis]
                new_scale_factors, new_rotation, new_metric = self.compass_step(
                    source, target, optimal_scale_factors, scale_neg)
                if new_metric <= optimal_metric:
                    optimal_metric = new_metric
                    optimal_transformation = new_rotation
                    optimal_scale_factors += scale_neg
                    errors.append(new_metric)
                    break
            if new_metric > optimal_metric:
                self._delta = self._delta / 2
        return self._finish(source, target, optimal_transformation, optimal_metric, optimal_scale_factors, errors,
                            refine_registration, icp_type)

    def _finish(self, source, target, optimal_transformation, optimal_metric, optimal_scale_factors, errors,
                refine_registration, icp_type):
        """Aligner.py:299-317."""
        if refine_registration:
            target = target * optimal_scale_factors
            optimal_transformation, optimal_metric = self.refine_registration(
                source=source, target=target, initial_transform=optimal_transformation, icp_type=icp_type)
            errors.append(optimal_metric)
        self.transfromation = optimal_transformation
        self.scale_factors = optimal_scale_factors
        return optimal_transformation, optimal_metric, optimal_scale_factors, errors

    def refine_registration(self, source, target, initial_transform, max_iteration: int = __REFINER_MAX_ITER__,
                            distance_threshold: float = __REFINER_DISTANCE_THRESHOLD__, icp_type: str = "PointToPoint"):
        """Aligner.py:319-364 on the MI355X kernels (orpcd_icp_p2p_batch).

        As in the reference, ``initial_transform`` (the row-convention T that
        align() composes) is handed to registration_icp, which applies it in
        its own column convention, and Open3D's column-convention result is
        returned (Q5).  ``PointToPlane`` raises as Open3D 0.18 does: the
        target cloud built by create_cloud carries no normals."""
        if icp_type == "PointToPlane":
            raise RuntimeError("TransformationEstimationPointToPlane and TransformationEstimationColoredICP "
                               "require pre-computed normal vectors for target PointCloud.")
        if icp_type != "PointToPoint":
            raise TypeError(f"registration_icp(): incompatible estimation_method {icp_type!r}")
        if distance_threshold <= 0:
            raise RuntimeError("Invalid max_correspondence_distance.")
        ctx = getattr(self._optimizer, "context", None)
        if ctx is None or not hasattr(ctx, "icp_p2p_batch"):
            if self._refine_ctx is None:
                self._refine_ctx = _native.default_context(None)
            ctx = self._refine_ctx
        ctx.set_target_points(np.asarray(target, dtype=np.float64))
        ctx.set_source_points(np.asarray(source, dtype=np.float64))
        r = ctx.icp_p2p_batch(np.asarray(initial_transform, dtype=np.float64)[None],
                              max_correspondence_distance=distance_threshold, max_iteration=max_iteration)
        self.last_refine = dict(fitness=float(r["fitness"][0]), iters=int(r["iters"][0]), ncorr=int(r["ncorr"][0]))
        return r["T"][0].copy(), float(r["rmse"][0])

    def transfrom(self, source: np.ndarray) -> np.ndarray:
        """Aligner.py:367-394."""
        for block in self._source_preprocessor.preprocessor_blocks:
            if issubclass(block.__class__, BaseScaler):
                source_mean, source_distance = block.mean, block.scale
        for block in self._target_preprocessor.preprocessor_blocks:
            if issubclass(block.__class__, BaseScaler):
                target_mean, target_distance = block.mean, block.scale
        source = (source - source_mean) / source_distance
        source = np.dot(source, self.transfromation[:3, :3]) + self.transfromation[:3, 3]
        source = source / self.scale_factors
        return source * target_distance + target_mean

    def __repr__(self):
        return (f"{self.__class__.__name__}(source_preprocessor={self._source_preprocessor}, "
                f"target_preprocessor={self._target_preprocessor}, optimizer={self._optimizer}, "
                f"attempts={self._attempts}, deg={self._deg}, mu={self._mu}, std={self._std}, "
                f"delta={self._delta}, max_iter={self._max_iter}, eps={self._eps})")
