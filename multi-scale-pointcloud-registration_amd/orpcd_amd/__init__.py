"""orpcd_amd — MI355X-native inner registration loop of OR-PCD.

Drop-in for the reference's plugin API (or_pcd.Optimizer / or_pcd.Aligner):

    from orpcd_amd.Optimizer import GeneralizedICP
    from orpcd_amd.Aligner import Aligner
    from orpcd_amd.Preprocessor import Preprocessor

Compute runs in liborpcd_hip.so (hand-written gfx950 kernels) through a
ctypes C-ABI (include/orpcd.h).  There is no CPU fallback.
"""
__version__ = "0.1.0"

from .Aligner import Aligner  # noqa: F401,E402
from .Optimizer import FastGlobalOptimizer, GeneralizedICP, IOptimizer  # noqa: F401,E402
from .Preprocessor import Preprocessor  # noqa: F401,E402
