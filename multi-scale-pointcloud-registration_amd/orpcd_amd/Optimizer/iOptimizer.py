"""IOptimizer — the plugin boundary (reference: or_pcd/Optimizer/iOptimizer.py:7-20)."""
from abc import ABC, abstractmethod
from typing import Tuple

import numpy as np


class IOptimizer(ABC):
    @abstractmethod
    def optimize(self, source: np.ndarray, target: np.ndarray, **kwargs) -> Tuple[np.ndarray, float]:
        """Run the inner block optimizer.

        Returns (4x4 roto-translation with R TRANSPOSED — row-vector convention —,
        inlier RMSE), exactly as the reference plugins do (generalizedICP.py:72-83)."""
