"""Logging in the reference format.

Reference: src/federation/server.py:93-105, client.py:66-73,245-257 -- file +
stdout handlers, format ``%(asctime)s [%(threadName)-12.12s] [%(levelname)-5.5s]
%(message)s``, files ``{logs_server}/logs_{YYYYMMDD}.txt`` and
``{logs_client}{id}/logs_{YYYYMMDD}.txt``.  Structured JSONL metrics (docs/s,
round latency split, loss) go to a separate ``metrics_{...}.jsonl`` next to the
log so the text log stays scraper-compatible.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Optional

from ..eval.export import date_stamp

LOG_FORMAT = "%(asctime)s [%(threadName)-12.12s] [%(levelname)-5.5s]  %(message)s"


def setup_logger(name: str, log_dir: Optional[str] = None, stamp: Optional[str] = None,
                 level=logging.INFO, stdout: bool = True) -> logging.Logger:
    logger = logging.getLogger(name)
    logger.setLevel(level)
    logger.propagate = False
    for h in list(logger.handlers):
        logger.removeHandler(h)
        h.close()
    fmt = logging.Formatter(LOG_FORMAT)
    if log_dir is not None:
        os.makedirs(log_dir, exist_ok=True)
        fh = logging.FileHandler(os.path.join(log_dir, f"logs_{stamp or date_stamp()}.txt"))
        fh.setFormatter(fmt)
        logger.addHandler(fh)
    if stdout:
        sh = logging.StreamHandler(sys.stdout)
        sh.setFormatter(fmt)
        logger.addHandler(sh)
    return logger


class MetricsWriter:
    """Append-only JSONL metrics (one object per line, wall-clock stamped)."""

    def __init__(self, path: Optional[str]):
        self.path = path
        if path:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)

    def write(self, **kv):
        if not self.path:
            return
        kv.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kv, default=float) + "\n")
