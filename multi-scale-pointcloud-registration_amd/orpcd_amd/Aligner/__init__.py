from .Aligner import Aligner  # noqa: F401
