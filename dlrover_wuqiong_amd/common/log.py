"""One logger for the whole framework.

Parity: reference ``dlrover/python/common/log.py:22-45`` (format
``[time] [level] [file:line:func] msg``).
"""

import logging
import os
import sys

_FMT = "[%(asctime)s] [%(levelname)s] [%(filename)s:%(lineno)d:%(funcName)s] %(message)s"


def get_logger(name: str = "dwamd", level=None) -> logging.Logger:
    logger = logging.getLogger(name)
    if not logger.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter(_FMT))
        logger.addHandler(h)
        logger.propagate = False
    lv = level or os.getenv("DWAMD_LOG_LEVEL", "INFO")
    logger.setLevel(lv)
    return logger


default_logger = get_logger()
logger = default_logger
