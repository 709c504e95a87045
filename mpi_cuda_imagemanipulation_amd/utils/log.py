"""Rank-prefixed logging (the reference prints from rank 0 with std::cout)."""
from __future__ import annotations

import logging
import os
import sys


def get_logger(name: str = "stripe", rank: int | None = None) -> logging.Logger:
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    log = logging.getLogger(f"{name}.r{rank}")
    if not log.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter(f"[r{rank} %(asctime)s %(levelname)s] %(message)s", "%H:%M:%S"))
        log.addHandler(h)
        log.setLevel(os.environ.get("STRIPE_LOG", "WARNING").upper())
        log.propagate = False
    return log
