"""Image I/O.  PPM (P6, RGB) / PGM (P5, gray), maxval 255, ASCII P2/P3 on read,
and baseline JPEG (the reference's format: cv::imread, kernel.cu:110;
imwrite, kernel.cu:236): native (csrc/core/image.cpp, csrc/core/jpeg.cpp),
atomic writes (temp file + rename).  Other formats (PNG, BMP, TIFF,
progressive JPEG) go through Pillow when it is installed.
Arrays are HxW (gray) or HxWx3 (RGB order) uint8.
"""
from __future__ import annotations

import os

import numpy as np

from .._native import C

PNM_EXT = {".ppm", ".pgm", ".pnm"}
JPEG_EXT = {".jpg", ".jpeg", ".jfif"}


def _is_pnm(path) -> bool:
    return os.path.splitext(str(path))[1].lower() in PNM_EXT


def _is_jpeg(path) -> bool:
    return os.path.splitext(str(path))[1].lower() in JPEG_EXT


def read_image(path: str) -> np.ndarray:
    if _is_pnm(path):
        return C.read_pnm(str(path))
    if _is_jpeg(path):
        try:
            return C.read_image(str(path))
        except RuntimeError as e:  # progressive / arithmetic-coded: Pillow, if present
            if "not supported" not in str(e):
                raise
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
    if _is_jpeg(path):
        C.write_image(str(path), img, quality)
        return
    try:
        from PIL import Image
    except ImportError as e:  # pragma: no cover
        raise RuntimeError(f"writing {path} needs Pillow (or use .ppm/.pgm)") from e
    tmp = f"{path}.tmp{os.getpid()}{os.path.splitext(str(path))[1]}"
    Image.fromarray(img).save(tmp)
    os.replace(tmp, str(path))


def decode_pnm(data: bytes) -> np.ndarray:
    return C.decode_pnm(data)


def encode_pnm(img) -> bytes:
    return C.encode_pnm(np.ascontiguousarray(img, dtype=np.uint8))


def decode_jpeg(data: bytes) -> np.ndarray:
    return C.decode_jpeg(data)


def encode_jpeg(img, quality: int = 95, subsample: bool = True, restart_interval: int = -1) -> bytes:
    """restart_interval: MCUs per interval (-1: one MCU row, coded in parallel; 0: none)"""
    return C.encode_jpeg(np.ascontiguousarray(img, dtype=np.uint8), quality, subsample, restart_interval)
