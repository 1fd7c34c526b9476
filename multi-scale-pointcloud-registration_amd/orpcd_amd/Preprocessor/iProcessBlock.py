"""IProcessBlock (reference: or_pcd/Preprocessor/iProcessBlock.py:6-12)."""
from abc import ABC, abstractmethod

import numpy as np


class IProcessBlock(ABC):
    @abstractmethod
    def process(self, cloud: np.ndarray) -> np.ndarray:
        """Processing function of the input cloud array."""
