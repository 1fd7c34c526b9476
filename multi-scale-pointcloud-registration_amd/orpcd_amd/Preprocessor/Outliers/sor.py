"""SOR — statistical outlier removal on the MI355X kernels.

Reference: or_pcd/Preprocessor/Outliers/sor.py:13-102, which calls Open3D
0.18's ``remove_statistical_outlier(nb_neighbors, std_ratio)`` and keeps the
inliers.  Here: ``orpcd_sor`` (exact KNN-k on device, the mean KNN distance
per point, the cloud statistics folded in index order as Open3D does, and a
device compaction of the kept indices); the inliers come back in input order.
"""
import numpy as np

from ... import _native
from ...utils.constants import __NB_NEIGHBOURS__, __STD_RATIO__
from ...utils.logger_factory import LoggerFactory
from ..iProcessBlock import IProcessBlock


class SOR(IProcessBlock):
    def __init__(self, nb_neighbours: int = __NB_NEIGHBOURS__, std_ratio: float = __STD_RATIO__, *, device=None):
        super().__init__()
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)
        self._nb_neighbours = nb_neighbours
        self._std_ratio = std_ratio
        self._device = device

    def process(self, cloud: np.ndarray) -> np.ndarray:
        ctx = _native.default_context(self._device)
        try:
            kept = ctx.sor(np.asarray(cloud, dtype=np.float64), self._nb_neighbours, self._std_ratio)
        except ValueError as e:  # Open3D raises RuntimeError on illegal parameters
            raise RuntimeError(str(e)) from None
        inliers = np.asarray(cloud, dtype=np.float64)[kept]
        self._LOG.debug(msg=f"Cloud before SOR had {int(cloud.shape[0])} points. "
                            f"After SOR has {inliers.shape[0]} points!")
        return inliers

    @property
    def nb_neighbours(self) -> int:
        return self._nb_neighbours

    @property
    def std_ratio(self) -> float:
        return self._std_ratio

    def __repr__(self):
        return f"{self.__class__.__name__}(nb_neighbours={self._nb_neighbours}, std_ratio={self._std_ratio})"
