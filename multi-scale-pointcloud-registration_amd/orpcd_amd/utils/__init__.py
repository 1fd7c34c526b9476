from .logger_factory import LoggerFactory  # noqa: F401
