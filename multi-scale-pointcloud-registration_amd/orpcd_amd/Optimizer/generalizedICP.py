"""GeneralizedICP plugin on the MI355X kernels.

Reference: or_pcd/Optimizer/generalizedICP.py:15-83 (wraps Open3D 0.18's
``registration_generalized_icp``).  Same constructor, defaults, validation
(warn + fall back to the default) and the same return convention: the 4x4
comes back with R transposed (row-vector convention, :72-74) and a
``ValueError`` is raised when the inlier RMSE is 0 (:77-81).

``optimize_batch`` is the batched entry the build's ``Aligner`` uses: all
multistart attempts of one target scale run as ONE device batch
(``orpcd_gicp_batch``) instead of ``attempts`` sequential calls.
"""
import time
from typing import Optional, Tuple

import numpy as np

from .. import _native
from ..utils.constants import (
    __ALIGNER_DEG__,
    __ALIGNER_MU__,
    __ALIGNER_STD__,
    __GICP_EPSILON__,
    __ICP_RELATIVE_FITNESS__,
    __ICP_RELATIVE_RMSE__,
    __MAX_ITERATIONS__,
    __MAXIMUM_CORRESPONDENCE_DISTANCE__,
)
from ..utils.logger_factory import LoggerFactory
from .iOptimizer import IOptimizer

_ZERO_RMSE_MSG = """Optimization failed with loss = 0. Parameters are not well set.
        Probably due to maximum_correspondence_distance set too low."""


class GeneralizedICP(IOptimizer):
    def __init__(
        self,
        max_correspondence_distance: float = __MAXIMUM_CORRESPONDENCE_DISTANCE__,
        max_iterations: int = __MAX_ITERATIONS__,
        *,
        epsilon: float = __GICP_EPSILON__,
        relative_fitness: float = __ICP_RELATIVE_FITNESS__,
        relative_rmse: float = __ICP_RELATIVE_RMSE__,
        device: Optional[int] = None,
        exact_nn: bool = True,
        rigid_cache: bool = True,
        speculate: int = 29,
        draw_model: Tuple[float, float, float] = (__ALIGNER_DEG__, __ALIGNER_MU__, __ALIGNER_STD__),
    ):
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)
        if max_correspondence_distance <= 0:
            self._LOG.warning(f"max correspondence distance cannot be 0 or less. Provided: {max_correspondence_distance}")
            self._max_correspondence_distance = __MAXIMUM_CORRESPONDENCE_DISTANCE__
        else:
            self._max_correspondence_distance = max_correspondence_distance
        if max_iterations <= 0:
            self._LOG.warning(f"max iterations cannot be 0 or less. Provided: {max_iterations}")
            self._max_iterations = __MAX_ITERATIONS__
        else:
            self._max_iterations = max_iterations
        self._epsilon = float(epsilon)
        self._relative_fitness = float(relative_fitness)
        self._relative_rmse = float(relative_rmse)
        self._device = device
        # exact_nn (default): every correspondence is the fp64 nearest target,
        # as Open3D's KD-tree (SearchHybrid, generalizedICP.py:59-70) and the
        # oracle find it (fp32 search + fp64 re-search of the queries whose
        # runner-up is within the fp32 error band).  False: the
        # fp32 search's answer (near-ties within 2^-17 resolved by position).
        self._exact_nn = bool(exact_nn)
        # the drop-in path (one optimize() per attempt, as the reference's
        # Aligner calls it): recognise a rigid image of the last cloud and
        # reuse its device layout and covariances (_rigid_image)
        self._rigid_cache = bool(rigid_cache)
        # ... and run the caller's next attempts ahead as one batch (at most
        # `speculate` of them; _speculate_next; 0: off).  draw_model: the (deg, mu, std) of the
        # Aligner whose initialize_rotation draws are predicted.
        self._speculate = max(0, int(speculate)) if rigid_cache else 0
        self._draw_model = tuple(float(x) for x in draw_model)
        self._spec = None  # predicted attempts: dict(base, target key, rows)
        self._spec_prev = None  # the RNG state after the last optimize() call's draw
        self._chain = None  # consecutive calls whose draws the model predicts (_speculate_next)
        self._learned = None  # the caller's attempts per multistart, once seen (_count_call)
        self._calls_key, self._calls, self._calls_ok = None, 0, False
        self._ended = None  # how the last confirmed chain ended: "switch" (new cloud / target) or "miss"
        self.spec_stats = dict(served=0, batches=0, missed=0, batch_s=0.0, serve_s=0.0, tie_reruns=0)
        self._tie_gaps_seen = 0  # context tie_gaps already reported (_note_tie_gaps)
        self._base = None
        self._tie_rows = None  # (base, rows of its KNN-20 boundary ties or None): _base_ties
        self._ctx = None
        self.last_result = None

    # the device context is created lazily (so the object can be built on a
    # host without a GPU, as the reference's can be without running Open3D)
    @property
    def context(self) -> _native.Context:
        if self._ctx is None:
            self._ctx = _native.default_context(self._device)
        # the process-wide context is shared: this optimizer's search mode every time
        self._ctx.set_option("exact_nn", 1 if self._exact_nn else 0)
        return self._ctx

    def _params(self):
        return dict(max_correspondence_distance=self._max_correspondence_distance,
                    max_iteration=self._max_iterations, relative_fitness=self._relative_fitness,
                    relative_rmse=self._relative_rmse, epsilon=self._epsilon)

    def _rigid_image(self, source: np.ndarray):
        """(R, t) with source == base @ R + t to round-off, when the base cloud
        cached by an earlier call is a rigid image of `source` -- what the
        reference's Aligner passes attempt after attempt (source_initialized =
        source @ R0 + t0, Aligner.py:183-190).  None otherwise.

        R, t come from a least-squares fit on 64 spread points and are then
        verified on EVERY point (|source - (base @ R + t)| <= 1e-12 relative to
        the cloud's extent, R orthonormal to 1e-12): a start is then run on the
        cached base with pose (R, t), so its KNN-20 covariances are the base's
        rotated (rigid invariance) instead of being recomputed
        on the posed copy."""
        base = self._base
        if base is None or base.shape != source.shape or len(source) < 4:
            return None
        idx = np.linspace(0, len(source) - 1, num=min(64, len(source))).astype(np.int64)
        A = np.c_[base[idx], np.ones(len(idx))]
        M, *_ = np.linalg.lstsq(A, source[idx], rcond=None)
        R, t = M[:3], M[3]
        if not np.all(np.isfinite(M)) or np.abs(R.T @ R - np.eye(3)).max() > 1e-12:
            return None
        res, mag = _native.rigid_residual(base, source, R, t)  # every point, one native pass
        if not res <= 1e-12 * (1.0 + mag):
            return None
        return R, t

    def _note_tie_gaps(self, ctx):
        """Warn about starts whose source boundary ties could not all be
        re-decided from their posed copy (orpcd_stats [19]); their covariances
        keep the rotated unposed ones (parity unpinned there).  One warning per
        source cloud (a source whose tie table overflowed would otherwise warn
        on every multistart); later gaps of the same source are logged at
        debug level and still counted in spec_stats["tie_gaps"]."""
        stats = getattr(ctx, "stats", None)  # a stand-in context (tests) may not count
        if stats is None:
            return
        g = int(stats().get("tie_gaps", 0))
        if g < self._tie_gaps_seen:  # the context's statistics were reset
            self._tie_gaps_seen = 0
        if g > self._tie_gaps_seen:
            new = g - self._tie_gaps_seen
            self.spec_stats["tie_gaps"] = self.spec_stats.get("tie_gaps", 0) + new
            source = getattr(ctx, "_source_key", None)
            msg = (f"{new} GICP start(s) with source KNN-20 boundary ties not re-decided per pose "
                   "(tie table full or pose far outside the cloud's extent)")
            if source is None or source != getattr(self, "_tie_gap_source", None):
                self._LOG.warning(msg + "; further gaps of this source are logged at debug level")
                self._tie_gap_source = source
            else:
                self._LOG.debug(msg)
        self._tie_gaps_seen = g

    def _base_ties(self, ctx):
        """Rows of the base cloud's KNN-20 boundary ties (orpcd_source_ties;
        None when it has none).  The device re-decides those points' neighbour
        sets per start from posed coordinates; on this path a call's own
        coordinates are the ones Open3D would use (the posed copy the caller
        formed), so they are handed over (orpcd_set_posed_tie_rows)."""
        if self._tie_rows is None or self._tie_rows[0] is not self._base:
            t = ctx.source_ties()
            self._tie_rows = (self._base, t["rows"] if t["n_ties"] else None)
        return self._tie_rows[1]

    def _run_alone(self, ctx, src, pose):
        """One start on the cached base with pose (R, t), the call's own
        posed coordinates deciding the boundary ties."""
        rows = self._base_ties(ctx)
        if rows is not None:
            ctx.set_posed_tie_rows(src[rows][None])
        r = ctx.gicp_batch(pose[0][None], pose[1][None], **self._params())
        self._note_tie_gaps(ctx)
        self.last_result = r
        return r["T"][0], float(r["rmse"][0])

    def optimize(self, source: np.ndarray, target: np.ndarray, **kwargs) -> Tuple[np.ndarray, float]:
        ctx = self.context
        ctx.set_target(target, self._epsilon)
        src = np.ascontiguousarray(source, dtype=np.float64)
        state = np.random.get_state() if self._speculate else None  # after this attempt's draw
        # a predicted attempt (checked on every point) needs no device work
        row = self._speculated(src, ctx._target_key) if self._spec is not None else None
        if row is None:
            pose = self._rigid_image(src) if self._rigid_cache else None
            if pose is None:  # a new cloud: it becomes the base (layout and KNN-20 covariances once)
                self._base = src.copy()
                ctx.set_source(self._base)
                pose = (np.eye(3), np.zeros(3))
            else:
                ctx.set_source(self._base)  # cached on the device (content key)
            if self._speculate:
                row = self._speculate_next(ctx, pose, state, src)
        else:
            self._count_call(ctx._target_key)
        self._spec_prev = state
        if row is None:
            T, rmse = self._run_alone(ctx, src, pose)
        else:
            T, rmse = row
        roto_translation = np.copy(T)
        roto_translation[:3, :3] = roto_translation[:3, :3].T
        if rmse == 0:
            self._LOG.error(_ZERO_RMSE_MSG)
            raise ValueError(_ZERO_RMSE_MSG)
        return roto_translation, rmse

    # ------------------------------------------------------------------
    # Speculative attempts on the drop-in path.  The reference's Aligner calls
    # optimize() once per attempt with source_initialized = source @ R0 + t0,
    # (R0, t0) = initialize_rotation() drawn from np.random just before the
    # call (Aligner.py:178-190).  The draw of a call is predicted from the RNG
    # state seen by the previous call (read, never advanced: a private replay
    # of the legacy MT19937 stream, draw_block); with the call's pose (R, t)
    # relative to the cached base (base = S Rb + tb, source = S R0 + t0 =
    # base R + t) it fixes the base's own pose Rb = R0 R^T, tb = (t0 - t) R^T.
    # Two consecutive calls that agree on (Rb, tb) confirm the model (a
    # chain); the next call's draws are then predicted and this call's start
    # and the predicted ones run as ONE device batch.  A predicted result is
    # returned only for a call whose source IS that predicted pose of the base
    # (every point checked to 1e-12 of the extent, as _rigid_image), so a
    # wrong prediction costs wasted device work, never a different answer;
    # each start's result does not depend on its batch mates
    # (tests/test_gpu_sched.py).  The batch covers the rest of the caller's
    # multistart as learned from a chain that ended on a new cloud (a
    # multistart's attempts; `speculate` ahead until one has been seen).
    # ------------------------------------------------------------------
    def _speculated(self, src: np.ndarray, tkey):
        t_0 = time.perf_counter()
        r = self._speculated_row(src, tkey)
        if r is not None:
            self.spec_stats["serve_s"] += time.perf_counter() - t_0
        return r

    def _speculated_row(self, src: np.ndarray, tkey):
        sp, ch = self._spec, self._chain
        if sp["base"] is not self._base or sp["tkey"] != tkey or not sp["rows"]:
            self._spec = None
            return None
        R, t, T, rmse, sets = sp["rows"].pop(0)
        res, mag = _native.rigid_residual(self._base, src, R, t) if src.shape == self._base.shape else (1.0, 0.0)
        if not res <= 1e-12 * (1.0 + mag):
            # not the predicted attempt (the caller re-seeded, or draws
            # differently): the chain ends here
            self._spec = None
            if self._rigid_image(src) is None:  # another cloud (the next multistart's): not a miss
                self._end_chain("switch")
            else:
                self._end_chain("miss")
                self.spec_stats["missed"] += 1
            return None
        ch["n"] += 1
        ctx = self.context
        rows = self._base_ties(ctx)
        if rows is not None:
            ctx.set_source(self._base)  # the tie table is the device source's (cached: no upload)
        if rows is not None and not np.array_equal(np.sort(sets, axis=1),
                                                   np.sort(ctx.tie_sets(posed_rows=src[rows]), axis=1)):
            # the predicted start decided a boundary tie from the base's posing,
            # the caller's own posed copy decides it otherwise: this call alone
            # (the order within a set only rounds the covariance's sums differently)
            self.spec_stats["tie_reruns"] += 1
            return self._run_alone(ctx, src, (R, t))
        self.spec_stats["served"] += 1
        return T, rmse

    def _end_chain(self, why):
        ch = self._chain
        if ch is None:
            return
        self._ended = why if ch["n"] >= 2 else None
        self._chain = None

    def _count_call(self, tkey):
        """Calls on the current (cloud, target): a confirmed run of them that
        ends on a new cloud or target is one multistart of the caller, whose
        length (its attempts) sizes later speculation."""
        key = (id(self._base), tkey)
        if key != self._calls_key:
            if self._calls_key is not None and self._calls_ok and self._calls >= 2:
                self._learned = self._calls
            self._calls_key, self._calls, self._calls_ok = key, 0, False
        self._calls += 1
        return self._calls

    def _speculate_next(self, ctx, pose, state, src):
        """Extend or start the chain with this call; once confirmed, run this
        call's start plus the predicted next attempts as one batch and return
        this call's (T, rmse)."""
        from ..Aligner.Aligner import draw_block

        c = self._count_call(ctx._target_key)  # this call's position on its cloud and target
        if self._spec_prev is None:
            return None
        deg, mu, std = self._draw_model
        (R0,), (t0,) = draw_block(1, deg, mu, std, _native.LegacyDraws(self._spec_prev))
        R, t = pose
        Rb, tb = R0 @ R.T, (t0 - t) @ R.T
        ch = self._chain
        same = ch is not None and ch["base"] is self._base and ch["tkey"] == ctx._target_key
        if same and np.abs(ch["Rb"] - Rb).max() <= 1e-9 and np.abs(ch["tb"] - tb).max() <= 1e-9:
            ch["n"] += 1
        else:
            # a confirmed chain that ended on a new cloud or target (the next
            # multistart of an align(): its draws continue the same stream) is
            # followed at once; after a re-seed (a miss) or a disagreement,
            # the new chain waits for a second call's confirmation
            self._end_chain("switch" if ch is not None and not same else "miss")
            self._chain = ch = dict(base=self._base, tkey=ctx._target_key, Rb=Rb, tb=tb, n=1)
            if self._ended != "switch":
                return None
            self._ended = None
        # the rest of the caller's multistart when its length is known (a
        # chain that ended on a new cloud or target: an align()'s multistarts),
        # else `speculate` ahead; predictions left over past a multistart's end
        # stay valid while the stream continues on the same cloud and target
        self._calls_ok = True
        A = self._learned
        ahead = self._speculate if A is None else min(self._speculate, (A - c % A) % A)
        if ahead < 1:
            return None
        Rb, tb = ch["Rb"], ch["tb"]
        Rn, tn = draw_block(ahead, deg, mu, std, _native.LegacyDraws(state))
        Rs = [R] + [Rb.T @ Rk for Rk in Rn]
        ts = [t] + [tk - tb @ Rr for tk, Rr in zip(tn, Rs[1:])]
        t_0 = time.perf_counter()
        rows = self._base_ties(ctx)
        if rows is not None:  # this call's own posed rows; the predicted ones are posed from the base
            posed = np.full((len(Rs), len(rows), 3), np.nan)
            posed[0] = src[rows]
            ctx.set_posed_tie_rows(posed)
        r = ctx.gicp_batch(np.array(Rs), np.array(ts), **self._params())
        self._note_tie_gaps(ctx)
        sets = [None if rows is None else ctx.tie_sets(k) for k in range(len(Rs))]
        self.spec_stats["batch_s"] += time.perf_counter() - t_0
        self.last_result = r
        self.spec_stats["batches"] += 1
        self._spec = dict(base=self._base, tkey=ctx._target_key,
                          rows=[(Rs[k], ts[k], r["T"][k], float(r["rmse"][k]), sets[k]) for k in range(1, len(Rs))])
        return r["T"][0], float(r["rmse"][0])

    def optimize_batch(self, source: np.ndarray, target: np.ndarray, R0: np.ndarray, t0: np.ndarray) -> dict:
        """GICP for every start ``source @ R0[b] + t0[b]`` (Aligner.py:183-190).

        Returns per-start ``T`` (R transposed, as ``optimize``), ``rmse``,
        ``fitness``, ``iters`` and ``ncorr``.  Does not raise on rmse == 0:
        the caller applies the reference's per-attempt error order."""
        ctx = self.context
        ctx.set_target(target, self._epsilon)
        ctx.set_source(source)
        r = ctx.gicp_batch(R0, t0, **self._params())
        self._note_tie_gaps(ctx)
        T = r["T"].copy()
        T[:, :3, :3] = np.transpose(T[:, :3, :3], (0, 2, 1))
        r["T"] = T
        self.last_result = r
        return r

    def optimize_batch_multi(self, source: np.ndarray, targets, R0s, t0s) -> list:
        """``optimize_batch`` for several targets at once (the speculative
        compass of ``Aligner``): up to 16 targets run as ONE device batch
        (orpcd_set_targets + orpcd_gicp_batch_targets), start (k, b) being
        ``source @ R0s[k][b] + t0s[k][b]`` against ``targets[k]``; more targets
        run in groups of 16.  Returns the per-target result dicts."""
        ctx = self.context
        out = []
        for g in range(0, len(targets), 16):
            tg, Rg, tg0 = targets[g:g + 16], R0s[g:g + 16], t0s[g:g + 16]
            ctx.set_targets(tg, self._epsilon)
            ctx.set_source(source)
            sizes = [len(r) for r in Rg]
            tids = np.repeat(np.arange(len(tg), dtype=np.int32), sizes)
            r = ctx.gicp_batch_targets(np.concatenate([np.asarray(x).reshape(-1, 3, 3) for x in Rg]),
                                       np.concatenate([np.asarray(x).reshape(-1, 3) for x in tg0]), tids,
                                       **self._params())
            self._note_tie_gaps(ctx)
            T = r["T"].copy()
            T[:, :3, :3] = np.transpose(T[:, :3, :3], (0, 2, 1))
            lo = 0
            for n in sizes:
                out.append({k: (T if k == "T" else v)[lo:lo + n] for k, v in r.items()})
                lo += n
        self.last_result = out[-1]
        return out

    zero_rmse_message = _ZERO_RMSE_MSG

    def batch_error(self, table: dict, n: int):
        """The exception optimize() would have raised for attempt n of a
        batched table (generalizedICP.py:77-81), or None."""
        if float(table["rmse"][n]) == 0:
            self._LOG.error(_ZERO_RMSE_MSG)
            return ValueError(_ZERO_RMSE_MSG)
        return None

    def __repr__(self):
        return f"""{self.__class__.__name__}
            (max_correspondence_distance={self._max_correspondence_distance},
            max_iterations={self._max_iterations})
        """
