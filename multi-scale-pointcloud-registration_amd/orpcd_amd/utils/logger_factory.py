"""Minimal logger factory (reference: or_pcd/utils/logger_factory.py:18-100).

Unlike the reference it never writes files under <cwd>/../logs and adds a
single console handler per logger, so repeated construction does not
duplicate lines.  Level defaults to WARNING (ORPCD_LOG_LEVEL overrides)."""
import logging
import os
import sys

_FMT = "%(asctime)s | %(name)s | %(levelname)s : %(message)s"


class LoggerFactory:
    @staticmethod
    def get_logger(log_name: str = "orpcd_amd", log_on_file: bool = False, **_) -> logging.Logger:
        logger = logging.getLogger(f"orpcd_amd.{log_name}")
        if not logger.handlers:
            h = logging.StreamHandler(stream=sys.stderr)
            h.setFormatter(logging.Formatter(_FMT))
            logger.addHandler(h)
            logger.setLevel(os.environ.get("ORPCD_LOG_LEVEL", "WARNING").upper())
            logger.propagate = False
        return logger
