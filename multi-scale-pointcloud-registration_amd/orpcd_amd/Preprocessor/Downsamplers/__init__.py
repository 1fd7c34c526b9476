from .randomDownsampler import RandomDownsampler  # noqa: F401
