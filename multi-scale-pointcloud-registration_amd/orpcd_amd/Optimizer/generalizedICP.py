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
from typing import Optional, Tuple

import numpy as np

from .. import _native
from ..utils.constants import (
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
        self._ctx = None
        self._pool = []          # device contexts of optimize_batch_multi (the first is self.context)
        self._executor = None
        self.last_result = None

    # the device context is created lazily (so the object can be built on a
    # host without a GPU, as the reference's can be without running Open3D)
    @property
    def context(self) -> _native.Context:
        if self._ctx is None:
            self._ctx = _native.default_context(self._device)
        return self._ctx

    def _params(self):
        return dict(max_correspondence_distance=self._max_correspondence_distance,
                    max_iteration=self._max_iterations, relative_fitness=self._relative_fitness,
                    relative_rmse=self._relative_rmse, epsilon=self._epsilon)

    def optimize(self, source: np.ndarray, target: np.ndarray, **kwargs) -> Tuple[np.ndarray, float]:
        ctx = self.context
        ctx.set_target(target, self._epsilon)
        ctx.set_source(source)
        r = ctx.gicp_batch(np.eye(3)[None], np.zeros((1, 3)), **self._params())
        self.last_result = r
        roto_translation = np.copy(r["T"][0])
        roto_translation[:3, :3] = roto_translation[:3, :3].T
        rmse = float(r["rmse"][0])
        if rmse == 0:
            self._LOG.error(_ZERO_RMSE_MSG)
            raise ValueError(_ZERO_RMSE_MSG)
        return roto_translation, rmse

    def optimize_batch(self, source: np.ndarray, target: np.ndarray, R0: np.ndarray, t0: np.ndarray) -> dict:
        """GICP for every start ``source @ R0[b] + t0[b]`` (Aligner.py:183-190).

        Returns per-start ``T`` (R transposed, as ``optimize``), ``rmse``,
        ``fitness``, ``iters`` and ``ncorr``.  Does not raise on rmse == 0:
        the caller applies the reference's per-attempt error order."""
        ctx = self.context
        ctx.set_target(target, self._epsilon)
        ctx.set_source(source)
        r = ctx.gicp_batch(R0, t0, **self._params())
        T = r["T"].copy()
        T[:, :3, :3] = np.transpose(T[:, :3, :3], (0, 2, 1))
        r["T"] = T
        self.last_result = r
        return r

    def optimize_batch_multi(self, source: np.ndarray, targets, R0s, t0s) -> list:
        """``optimize_batch`` for several targets at once: batch k runs on its
        own device context (own stream) from its own host thread, so the
        batches execute concurrently on the GPU (the speculative compass of
        ``Aligner``).  Returns the per-target result dicts."""
        from concurrent.futures import ThreadPoolExecutor

        n = len(targets)
        while len(self._pool) < n:
            self._pool.append(self.context if not self._pool else _native.Context(self.context.device))
        # the concurrent batches share the GPU: each splits its search over a
        # share of the waves one batch alone would use
        waves = max(4096, self.search_waves // n)
        for ctx in self._pool[:n]:
            ctx.set_option("search_waves", waves)
        if self._executor is None or self._executor._max_workers < n:
            self._executor = ThreadPoolExecutor(max_workers=n)

        def run(k):
            ctx = self._pool[k]
            ctx.set_target(targets[k], self._epsilon)
            ctx.set_source(source)
            r = ctx.gicp_batch(R0s[k], t0s[k], **self._params())
            T = r["T"].copy()
            T[:, :3, :3] = np.transpose(T[:, :3, :3], (0, 2, 1))
            r["T"] = T
            return r

        try:
            out = list(self._executor.map(run, range(n)))  # ctypes releases the GIL during each call
        finally:
            self.context.set_option("search_waves", self.search_waves)  # single batches: the full target
        self.last_result = out[-1]
        return out

    search_waves = 32768  # split target of one batch alone (orpcd_set_option "search_waves" default)

    zero_rmse_message = _ZERO_RMSE_MSG

    def __repr__(self):
        return f"""{self.__class__.__name__}
            (max_correspondence_distance={self._max_correspondence_distance},
            max_iterations={self._max_iterations})
        """
