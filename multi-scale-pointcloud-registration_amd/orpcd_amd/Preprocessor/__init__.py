from .preprocessor import Preprocessor  # noqa: F401
