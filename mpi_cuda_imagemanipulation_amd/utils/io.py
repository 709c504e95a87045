"""PPM (P6, RGB) / PGM (P5, gray) I/O, maxval 255; ASCII P2/P3 accepted on read.

Reference I/O was OpenCV JPEG with hard-coded paths (kernel.cu:110,236); this is
lossless and path-parameterised.  Parsing/encoding is native (csrc/core/image.cpp);
writes are atomic (temp file + rename).  Arrays are HxW (gray) or HxWx3 (RGB) uint8.
"""
from __future__ import annotations

import numpy as np

from .._native import C


def read_image(path: str) -> np.ndarray:
    return C.read_pnm(str(path))


def write_image(path: str, img) -> None:
    if hasattr(img, "detach"):
        img = img.detach().cpu().numpy()
    C.write_pnm(str(path), np.ascontiguousarray(img, dtype=np.uint8))


def decode_pnm(data: bytes) -> np.ndarray:
    return C.decode_pnm(data)


def encode_pnm(img) -> bytes:
    return C.encode_pnm(np.ascontiguousarray(img, dtype=np.uint8))
