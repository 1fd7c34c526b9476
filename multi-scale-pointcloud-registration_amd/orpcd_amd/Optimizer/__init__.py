from .iOptimizer import IOptimizer  # noqa: F401
from .generalizedICP import GeneralizedICP  # noqa: F401
