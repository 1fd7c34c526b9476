"""Preprocessor (reference: or_pcd/Preprocessor/preprocessor.py:11-31).
Auto-inserts a RadiusScaler at index 0 when no scaler is present."""
from typing import List

import numpy as np

from ..utils.logger_factory import LoggerFactory
from .iProcessBlock import IProcessBlock
from .Scalers import BaseScaler, RadiusScaler


class Preprocessor:
    def __init__(self, preprocessor_blocks: List[IProcessBlock]):
        self._LOG = LoggerFactory.get_logger(self.__class__.__name__)
        if not any(issubclass(block.__class__, BaseScaler) for block in preprocessor_blocks):
            self._LOG.warning("Scalers block is not present in the preprocessor blocks --> "
                              "Adding Scalers block to the preprocessor blocks")
            preprocessor_blocks.insert(0, RadiusScaler())
        self.preprocessor_blocks = preprocessor_blocks

    def preprocess(self, cloud: np.ndarray) -> np.ndarray:
        for block in self.preprocessor_blocks:
            cloud = block.process(cloud)
        return cloud
