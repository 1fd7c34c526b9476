"""RandomDownsampler (reference: or_pcd/Preprocessor/Downsamplers/randomDownsampler.py:9-40).
Uses the global legacy numpy RNG exactly like the reference (Q7)."""
import numpy as np

from ...utils.constants import __SAMPLE_SIZE__
from ...utils.logger_factory import LoggerFactory
from ..iProcessBlock import IProcessBlock


class RandomDownsampler(IProcessBlock):
    def __init__(self, sample_size: int = __SAMPLE_SIZE__, replace: bool = False):
        self._LOG = LoggerFactory.get_logger(log_name=self.__class__.__name__)
        if sample_size <= 0:
            self._LOG.warning(f"sample size cannot be 0 or less. Provided: {sample_size}. "
                              f"Using default value: {__SAMPLE_SIZE__}")
            self._sample_size = __SAMPLE_SIZE__
        else:
            self._sample_size = sample_size
        self._replace = replace

    def process(self, cloud: np.ndarray) -> np.ndarray:
        return cloud[np.random.choice(cloud.shape[0], self._sample_size, replace=self._replace)]

    def __repr__(self):
        return f"{self.__class__.__name__}(sample_size={self._sample_size}, replace={self._replace})"
