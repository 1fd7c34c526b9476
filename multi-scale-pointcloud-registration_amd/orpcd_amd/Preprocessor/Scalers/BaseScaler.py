"""BaseScaler (reference: or_pcd/Preprocessor/Scalers/BaseScaler.py)."""
import numpy as np

from ..iProcessBlock import IProcessBlock


class BaseScaler(IProcessBlock):
    mean: np.ndarray = np.zeros((1, 3))
    scale: float = 1.0
