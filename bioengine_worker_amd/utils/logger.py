"""Logging helpers (reference: bioengine/utils/logger.py:10-31).

Colored console output plus an optional plain-text file handler; loggers do not propagate to the
root logger so app replicas and the worker can each own their log files.
"""
from __future__ import annotations

import logging
from pathlib import Path

stream_logging_format = "\033[36m%(asctime)s\033[0m - \033[32m%(name)s\033[0m - \033[1;33m%(levelname)s\033[0m - %(message)s"
file_logging_format = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"
date_format = "%Y-%m-%d %H:%M:%S %Z"


def create_logger(name: str, level: int = logging.INFO, log_file: str | Path | None = None) -> logging.Logger:
    log = logging.getLogger(name)
    log.setLevel(level)
    log.propagate = False
    have_stream = any(isinstance(h, logging.StreamHandler) and not isinstance(h, logging.FileHandler) for h in log.handlers)
    if not have_stream:
        sh = logging.StreamHandler()
        sh.setFormatter(logging.Formatter(stream_logging_format, date_format))
        log.addHandler(sh)
    if log_file and str(log_file).lower() != "off":
        p = Path(log_file).resolve()
        p.parent.mkdir(parents=True, exist_ok=True)
        if not any(isinstance(h, logging.FileHandler) and Path(h.baseFilename) == p for h in log.handlers):
            fh = logging.FileHandler(p)
            fh.setFormatter(logging.Formatter(file_logging_format, date_format))
            log.addHandler(fh)
    return log
