"""VoxelDownsampler on the MI355X kernels.

Reference: or_pcd/Preprocessor/Downsamplers/voxelDownsampler.py:14-136 — a
compass search over the voxel size until |target_points - n_points| stops
improving, each step an Open3D ``voxel_down_sample``.  Same validation, the
same search (including the stateful ``_delta``, which the reference halves
in place across calls), each step's count from ``orpcd_voxel_down_sample``
(device sort + run-length encoding) and the averaged points of the chosen
size from the same call.  Voxels come out in (ix, iy, iz) order (Open3D's
order is its unordered_map's, unspecified).
"""
import numpy as np

from ... import _native
from ...utils.constants import __BASE_VOXEL_SIZE__, __DELTA__, __EPS__, __MIN_VOXEL_SIZE__
from ...utils.logger_factory import LoggerFactory
from ..iProcessBlock import IProcessBlock


class VoxelDownsampler(IProcessBlock):
    def __init__(self, target_points: int, base_voxel_size: float = __BASE_VOXEL_SIZE__,
                 min_voxel_size: float = __MIN_VOXEL_SIZE__, delta: float = __DELTA__, eps: float = __EPS__, *,
                 device=None):
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)
        if target_points <= 0:
            msg = f"target points cannot be 0 or less. Provided: {target_points}"
            self._LOG.error(msg)
            raise ValueError(msg)
        self._target_points = target_points
        checks = [("min voxel size", min_voxel_size, __MIN_VOXEL_SIZE__),
                  ("base voxel size", base_voxel_size, __BASE_VOXEL_SIZE__),
                  ("delta", delta, __DELTA__), ("eps", eps, __EPS__)]
        vals = []
        for name, v, default in checks:  # voxelDownsampler.py:45-72
            if v <= 0:
                self._LOG.warning(f"{name} cannot be 0 or less. Provided: {v}. Using default value: {default}")
                v = default
            vals.append(v)
        self._min_voxel_size, self._base_voxel_size, self._delta, self._eps = vals
        self._device = device
        self.voxel_size = None  # instrumentation: the size chosen by the last process()

    def _count(self, ctx, cloud, voxel_size):
        return ctx.voxel_down_sample(cloud, voxel_size, count_only=True)

    def compass_step(self, delta: float, ctx, cloud: np.ndarray, current_voxel_size: float):
        """voxelDownsampler.py:77-85 (returns the size and metric; the cloud is
        materialised once, for the size finally chosen)."""
        new_voxel_size = current_voxel_size + delta
        if new_voxel_size <= self._min_voxel_size:
            new_voxel_size = self._min_voxel_size
        metric = np.abs(self._target_points - self._count(ctx, cloud, new_voxel_size))
        return new_voxel_size, metric

    def process(self, cloud: np.ndarray) -> np.ndarray:
        """voxelDownsampler.py:87-125."""
        ctx = _native.default_context(self._device)
        cloud = np.asarray(cloud, dtype=np.float64)
        current_voxel_size = self._base_voxel_size
        best_size = current_voxel_size
        metric = np.abs(self._target_points - self._count(ctx, cloud, current_voxel_size))
        while self._delta >= self._eps:
            new_voxel_size, obtained_metric = self.compass_step(self._delta, ctx, cloud, current_voxel_size)
            if obtained_metric < metric:
                current_voxel_size = new_voxel_size
                metric = obtained_metric
                best_size = new_voxel_size
                continue
            new_voxel_size, obtained_metric = self.compass_step(-self._delta, ctx, cloud, current_voxel_size)
            if obtained_metric < metric:
                current_voxel_size = new_voxel_size
                metric = obtained_metric
                best_size = new_voxel_size
                continue
            self._delta = self._delta / 2
        self._LOG.debug(msg=f"Voxel size: {current_voxel_size}, Metric: {metric}")
        self.voxel_size = best_size
        return ctx.voxel_down_sample(cloud, best_size)

    def __repr__(self):
        return (f"{self.__class__.__name__}(target_points={self._target_points}, "
                f"base_voxel_size={self._base_voxel_size}, min_voxel_size={self._min_voxel_size}, "
                f"delta={self._delta}, eps={self._eps})")
