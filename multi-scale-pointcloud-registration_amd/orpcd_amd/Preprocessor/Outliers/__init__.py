from .sor import SOR  # noqa: F401
