"""FastGlobalOptimizer plugin on the MI355X kernels.

Reference: or_pcd/Optimizer/fastGlobalOptimizer.py:22-203 (wraps Open3D 0.18's
``estimate_normals`` + ``compute_fpfh_feature`` + ``registration_fgr_based_on_
feature_matching``).  Same constructor, defaults, validation (log + fall back
to the default), R-transposed return (:176-178) and ``Warning`` raised when
the evaluation finds no correspondence (:181-188).

One call = one ``orpcd_fgr_optimize``: FPFH of both clouds, the mutual
feature matching, the tuple test, the GNC IRLS and the evaluation all run
against device-resident clouds.  The tuple test's mt19937 word stream is
generated on the host; every trial is evaluated and the accepted tuples
selected on the device.  Matching: with each cloud's own features it is the
fp64-MFMA 33-D nearest-row search in both directions; under Q4 on equal-size
clouds the two feature sets are the same rows, so every row's nearest row is
the lowest index of its exact duplicates and the mutual pairs come from the
dedup pass alone (no search).

Quirk Q4 (fastGlobalOptimizer.py:137-142): the reference computes the TARGET
features from the SOURCE cloud.  ``target_features_from_source=True`` (the
default) reproduces that; it needs ``len(target) <= len(source)`` — the
reference would index past the source's features otherwise, so this build
raises ``ValueError`` there.  Set it to False for the evidently intended
behaviour (features of each cloud).

``optimize_batch`` / ``optimize_batch_multi`` are the batched entries the
build's ``Aligner`` uses (as for GeneralizedICP): all attempts of a
multistart, or of the speculative compass's candidate scales, run as ONE
``orpcd_fgr_optimize_batch`` call -- per start the same normals, FPFH,
matching, tuple test, IRLS and evaluation as ``optimize`` on the posed copy
``source @ R0 + t0``, bit for bit, with the tuple tests of all starts and
the IRLS problems of all starts each in one device launch.

``seed`` seeds the tuple test's mt19937.  Open3D draws it from its global
engine, which is not seeded by the reference, so the reference's FGR result
varies run to run; here it is reproducible.
"""
from typing import Optional, Tuple

import numpy as np

from .. import _native
from ..utils.constants import (
    __DECREASE_MU__,
    __DIVISION_FACTOR__,
    __FGR_MAXIMUM_TUPLE_COUNT__,
    __FPFH_KNN__,
    __FPFH_RADIUS__,
    __ITERATION_NUMBER__,
    __MAXIMUM_CORRESPONDENCE_DISTANCE__,
    __NORMAL_ESTIMATE_KNN__,
    __NORMAL_ESTIMATE_RADIUS__,
    __TUPLE_SCALE__,
)
from ..utils.logger_factory import LoggerFactory
from .iOptimizer import IOptimizer

_NO_CORR_MSG = """No correspondences detected from the optimizer. Parameters are not well set.
        Probably due to:
        -   maximum_correspondence_distance set too low
        -   tuple_scale set too high
        """


class FastGlobalOptimizer(IOptimizer):
    def __init__(
        self,
        division_factor: float = __DIVISION_FACTOR__,
        tuple_scale: float = __TUPLE_SCALE__,
        maximum_correspondence_distance: float = __MAXIMUM_CORRESPONDENCE_DISTANCE__,
        iteration_number: int = __ITERATION_NUMBER__,
        decrease_mu: bool = __DECREASE_MU__,
        normal_estimate_radius: float = __NORMAL_ESTIMATE_RADIUS__,
        normal_estimate_knn: int = __NORMAL_ESTIMATE_KNN__,
        fpfh_radius: float = __FPFH_RADIUS__,
        fpfh_knn: int = __FPFH_KNN__,
        *,
        target_features_from_source: bool = True,
        maximum_tuple_count: int = __FGR_MAXIMUM_TUPLE_COUNT__,
        seed: int = 0,
        device: Optional[int] = None,
    ):
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)

        def positive(value, default, what):
            if value <= 0:
                self._LOG.error(f"{what} cannot be 0 or less. Provided: {value}")
                return default
            return value

        self._division_factor = positive(division_factor, __DIVISION_FACTOR__,
                                         "division factor")
        self._tuple_scale = positive(tuple_scale, __TUPLE_SCALE__, "tuple scale")
        self._maximum_correspondence_distance = positive(maximum_correspondence_distance,
            __MAXIMUM_CORRESPONDENCE_DISTANCE__, "maximum correspondence distance")
        self._iteration_number = positive(iteration_number, __ITERATION_NUMBER__,
                                          "iteration number")
        self._decrease_mu = decrease_mu
        self._fpfh_radius = positive(fpfh_radius, __FPFH_RADIUS__, "fpfh radius")
        self._fpfh_knn = positive(fpfh_knn, __FPFH_KNN__, "fpfh knn")
        self._normal_estimate_radius = positive(normal_estimate_radius,
                                                __NORMAL_ESTIMATE_RADIUS__, "normal estimate radius")
        self._normal_estimate_knn = positive(normal_estimate_knn, __NORMAL_ESTIMATE_KNN__,
                                             "normal estimate knn")
        if not (int(self._fpfh_knn) <= 1024 and int(self._normal_estimate_knn) <= 1024):
            # the device KNN keeps up to 16 sorted chunks of 64 per query (knn_wave_multi_kernel)
            raise ValueError("this build supports neighbourhoods of at most 1024 points (knn <= 1024)")
        self._target_features_from_source = bool(target_features_from_source)
        self._maximum_tuple_count = int(maximum_tuple_count)
        self._seed = int(seed)
        self._device = device
        self._ctx = None
        self.last_result = None
        self._LOG.debug(msg=f"initialized optimizer: {self}")

    @property
    def context(self) -> _native.Context:
        if self._ctx is None:
            self._ctx = _native.default_context(self._device)
        return self._ctx

    def get_fpfh_features(self, source_point_cloud: np.ndarray, target_point_cloud: np.ndarray):
        """(source features, target features), each (N, 33) — fastGlobalOptimizer.py:109-144,
        including Q4 when ``target_features_from_source``."""
        ctx = self.context
        args = (self._normal_estimate_radius, self._normal_estimate_knn, self._fpfh_radius, self._fpfh_knn)
        _, fs = ctx.fpfh(source_point_cloud, *args)
        ft = fs.copy() if self._target_features_from_source else ctx.fpfh(target_point_cloud, *args)[1]
        return fs, ft

    def optimize(self, source: np.ndarray, target: np.ndarray, **kwargs) -> Tuple[np.ndarray, float]:
        r = self.context.fgr_optimize(
            source, target, normal_radius=self._normal_estimate_radius, normal_knn=self._normal_estimate_knn,
            fpfh_radius=self._fpfh_radius, fpfh_knn=self._fpfh_knn,
            target_features_from_source=self._target_features_from_source,
            division_factor=self._division_factor, tuple_scale=self._tuple_scale,
            maximum_correspondence_distance=self._maximum_correspondence_distance,
            iteration_number=self._iteration_number, decrease_mu=self._decrease_mu,
            maximum_tuple_count=self._maximum_tuple_count, seed=self._seed)
        self.last_result = r
        roto_translation = np.copy(r["T"])
        roto_translation[:3, :3] = roto_translation[:3, :3].T
        if r["ncorr"] == 0:
            self._LOG.error(_NO_CORR_MSG)
            raise Warning(_NO_CORR_MSG)
        return roto_translation, r["rmse"]

    def _kw(self):
        return dict(normal_radius=self._normal_estimate_radius, normal_knn=self._normal_estimate_knn,
                    fpfh_radius=self._fpfh_radius, fpfh_knn=self._fpfh_knn,
                    target_features_from_source=self._target_features_from_source,
                    division_factor=self._division_factor, tuple_scale=self._tuple_scale,
                    maximum_correspondence_distance=self._maximum_correspondence_distance,
                    iteration_number=self._iteration_number, decrease_mu=self._decrease_mu,
                    maximum_tuple_count=self._maximum_tuple_count, seed=self._seed)

    def _table(self, r):
        """Per-start records in the Aligner's table form (T with R transposed,
        as optimize returns it; iters = the IRLS iterations run, 0 when
        fewer than 10 tuple correspondences leave T at the identity)."""
        T = r["T"].copy()
        T[:, :3, :3] = np.transpose(T[:, :3, :3], (0, 2, 1))
        iters = np.where(r["n_tuple_corr"] >= 10, self._iteration_number, 0).astype(np.int64)
        return dict(T=T, rmse=r["rmse"], fitness=r["fitness"], iters=iters, ncorr=r["ncorr"],
                    n_mutual=r["n_mutual"], n_tuple_corr=r["n_tuple_corr"])

    def optimize_batch(self, source: np.ndarray, target: np.ndarray, R0: np.ndarray, t0: np.ndarray) -> dict:
        """``optimize(source @ R0[b] + t0[b], target)`` for every start b as one
        device call.  Does not raise on a start without correspondences: the
        caller replays the reference's per-attempt error order (batch_error)."""
        r = self._table(self.context.fgr_optimize_batch(source, [target], R0, t0, **self._kw()))
        self.last_result = r
        return r

    def optimize_batch_multi(self, source: np.ndarray, targets, R0s, t0s) -> list:
        """``optimize_batch`` for several targets (the speculative compass's
        candidate scales) as one call per 16 targets."""
        out = []
        for g in range(0, len(targets), 16):
            tg, Rg, tg0 = targets[g:g + 16], R0s[g:g + 16], t0s[g:g + 16]
            sizes = [len(np.asarray(x).reshape(-1, 9)) for x in Rg]
            tids = np.repeat(np.arange(len(tg), dtype=np.int32), sizes)
            r = self._table(self.context.fgr_optimize_batch(
                source, tg, np.concatenate([np.asarray(x).reshape(-1, 3, 3) for x in Rg]),
                np.concatenate([np.asarray(x).reshape(-1, 3) for x in tg0]), target_of_start=tids, **self._kw()))
            lo = 0
            for k in sizes:
                out.append({key: v[lo:lo + k] for key, v in r.items()})
                lo += k
        self.last_result = out[-1]
        return out

    def batch_error(self, table: dict, n: int):
        """The exception optimize() would have raised for attempt n of a
        batched table (fastGlobalOptimizer.py:181-188), or None."""
        if int(table["ncorr"][n]) == 0:
            self._LOG.error(_NO_CORR_MSG)
            return Warning(_NO_CORR_MSG)
        return None

    def __repr__(self):
        return f"""{self.__class__.__name__}
            (division_factor={self._division_factor},
            tuple_scale={self._tuple_scale},
            maximum_correspondence_distance={self._maximum_correspondence_distance},
            iteration_number={self._iteration_number},
            decrease_mu={self._decrease_mu},
            normal_estimate_radius={self._normal_estimate_radius},
            normal_estimate_knn={self._normal_estimate_knn},
            fpfh_radius={self._fpfh_radius},
            fpfh_knn={self._fpfh_knn})"
        """
