"""Seeded synthetic random-pixel frames (counter-based: any rank can generate any
rows independently; identical bytes on host (C++) and device (HIP))."""
from __future__ import annotations

import numpy as np

from .._native import C


def synthetic_image(seed: int, width: int, height: int, channels: int = 3) -> np.ndarray:
    return C.synth_image(int(seed), int(width), int(height), int(channels))


def synthetic_rows(seed: int, width: int, channels: int, row0: int, rows: int) -> np.ndarray:
    return C.synth_rows(int(seed), int(width), int(channels), int(row0), int(rows))
