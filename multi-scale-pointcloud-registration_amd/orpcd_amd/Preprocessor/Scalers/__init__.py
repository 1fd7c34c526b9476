from .BaseScaler import BaseScaler  # noqa: F401
from .radiusScaler import RadiusScaler  # noqa: F401
