"""FarthestDownsampler on the MI355X kernels.

Reference: or_pcd/Preprocessor/Downsamplers/farthestDownsampler.py:10-57 (a
Python loop of ``sample_size - 1`` scipy ``cdist`` calls).  Here the first
index is drawn exactly as the reference draws it (``np.random.randint``,
:35, global legacy RNG, Q7) and all steps run in ONE cooperative device
launch (``orpcd_farthest_downsample``): same distances (cdist's Euclidean,
correctly rounded), same elementwise minimum, same first-index argmax, so the
chosen points are the reference's bit for bit.
"""
import numpy as np

from ... import _native
from ...utils.constants import __SAMPLE_SIZE__
from ...utils.logger_factory import LoggerFactory
from ..iProcessBlock import IProcessBlock


class FarthestDownsampler(IProcessBlock):
    def __init__(self, sample_size: int = __SAMPLE_SIZE__, *, device=None):
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)
        if sample_size <= 0:
            self._LOG.warning(f"sample size cannot be 0 or less. Provided: {sample_size}. "
                              f"Using default value: {__SAMPLE_SIZE__}")
            self._sample_size = __SAMPLE_SIZE__
        else:
            self._sample_size = sample_size
        self._device = device

    def process(self, cloud: np.ndarray) -> np.ndarray:
        cloud = np.asarray(cloud)
        first = np.random.randint(low=0, high=cloud.shape[0])
        idx = _native.default_context(self._device).farthest_downsample(cloud.astype(np.float64, copy=False),
                                                                      self._sample_size, first)
        return cloud[idx]

    def __repr__(self):
        return f"{self.__class__.__name__}(sample_size={self._sample_size})"
