from .farthestDownsampler import FarthestDownsampler  # noqa: F401
from .randomDownsampler import RandomDownsampler  # noqa: F401
from .voxelDownsampler import VoxelDownsampler  # noqa: F401
