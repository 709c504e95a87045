"""Image I/O.  PPM (P6, RGB) / PGM (P5, gray), maxval 255, ASCII P2/P3 on read,
and JPEG (the reference's format: cv::imread, kernel.cu:110; imwrite,
kernel.cu:236): native (csrc/core/image.cpp, csrc/core/jpeg.cpp: sequential
and progressive decode, baseline encode), atomic writes (temp file + rename).
Other formats (PNG, BMP, TIFF; lossless / arithmetic-coded JPEG) go through
Pillow when it is installed.
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
        except RuntimeError as e:  # lossless / arithmetic-coded: Pillow, if present
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


def read_image_device(path: str, device=None):
    """Decode an image straight into a CUDA uint8 tensor (HxW or HxWx3).
    Baseline JPEG: Huffman decoding on the host, IDCT + upsampling + colour on
    the GPU (csrc/hip/jpeg_dev.hip) -- only the coefficients cross the link.
    Other formats: host decode, then one upload."""
    import torch

    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    data = open(str(path), "rb").read()
    if data[:2] != b"\xff\xd8":
        return torch.from_numpy(read_image(path)).to(dev)
    jc = C.jpeg_entropy_decode(data)
    shape = (jc.H, jc.W) if jc.C == 1 else (jc.H, jc.W, jc.C)
    out = torch.empty(shape, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        jc.to_device(out.data_ptr(), jc.W * jc.C, torch.cuda.current_stream(dev).cuda_stream)
    return out


def write_image_device(path: str, img, quality: int = 95) -> None:
    """Write a CUDA uint8 tensor: JPEG paths encode with colour conversion,
    DCT and quantisation on the GPU and Huffman coding on the host (restart
    interval per MCU row, coded in parallel); other formats via the host."""
    import torch

    if not _is_jpeg(path) or not (hasattr(img, "is_cuda") and img.is_cuda):
        write_image(path, img, quality)
        return
    x = img.contiguous()
    H, W = int(x.shape[0]), int(x.shape[1])
    Cc = 1 if x.dim() == 2 else int(x.shape[2])
    with torch.cuda.device(x.device):
        data = C.jpeg_encode_device(x.data_ptr(), W * Cc, W, H, Cc, quality, True, -1,
                                    torch.cuda.current_stream(x.device).cuda_stream)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, str(path))
