"""Image I/O.  PPM (P6, RGB) / PGM (P5, gray), maxval 255, ASCII P2/P3 on read:
native (csrc/core/image.cpp), atomic writes (temp file + rename).  Other formats
(JPEG, PNG, BMP, TIFF - the reference reads JPEG via cv::imread, kernel.cu:110,
and writes JPEG, kernel.cu:236) go through Pillow when it is installed.
Arrays are HxW (gray) or HxWx3 (RGB order) uint8.
"""
from __future__ import annotations

import os

import numpy as np

from .._native import C

PNM_EXT = {".ppm", ".pgm", ".pnm"}


def _is_pnm(path) -> bool:
    return os.path.splitext(str(path))[1].lower() in PNM_EXT


def read_image(path: str) -> np.ndarray:
    if _is_pnm(path):
        return C.read_pnm(str(path))
    try:
        from PIL import Image
    except ImportError as e:  # pragma: no cover - Pillow is optional
        raise RuntimeError(f"reading {path} needs Pillow (or use .ppm/.pgm)") from e
    with Image.open(str(path)) as im:
        if im.mode in ("L", "I;16", "I", "F", "1"):
            return np.asarray(im.convert("L"), dtype=np.uint8).copy()
        return np.asarray(im.convert("RGB"), dtype=np.uint8).copy()


def write_image(path: str, img, quality: int = 95) -> None:
    if hasattr(img, "detach"):
        img = img.detach().cpu().numpy()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if _is_pnm(path):
        C.write_pnm(str(path), img)
        return
    try:
        from PIL import Image
    except ImportError as e:  # pragma: no cover
        raise RuntimeError(f"writing {path} needs Pillow (or use .ppm/.pgm)") from e
    tmp = f"{path}.tmp{os.getpid()}{os.path.splitext(str(path))[1]}"
    Image.fromarray(img).save(tmp, quality=quality) if str(path).lower().endswith((".jpg", ".jpeg")) \
        else Image.fromarray(img).save(tmp)
    os.replace(tmp, str(path))


def decode_pnm(data: bytes) -> np.ndarray:
    return C.decode_pnm(data)


def encode_pnm(img) -> bytes:
    return C.encode_pnm(np.ascontiguousarray(img, dtype=np.uint8))
