from .iOptimizer import IOptimizer  # noqa: F401
from .generalizedICP import GeneralizedICP  # noqa: F401
from .fastGlobalOptimizer import FastGlobalOptimizer  # noqa: F401
