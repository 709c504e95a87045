"""Filter operations on single images.

* torch CUDA (ROCm) uint8 tensors run on the HIP kernels (csrc/hip/*.hip) on
  torch's current stream;
* numpy arrays / CPU tensors run on the threaded host executor
  (csrc/core/cpu_exec.cpp, bit-identical to the C++ golden path).

Images are HxW (gray) or HxWx3 (RGB, PPM channel order) uint8; a batch of
frames is BxHxWxC (C = 1 or 3) and runs frame by frame through one cached
engine (same kernels, no per-frame setup).  A chain is a
comma-separated filter list, e.g. "gray:ref,contrast:3.5,emboss3" (see
`FILTERS`); consecutive pointwise ops are fused into the neighbouring stencil
kernel.  Reference kernels: grayscaleKernel / contrastKernel / embossKernel
(kernel.cu:31-94) and the OpenCV CPU chain (kern.cpp:58-77).
"""
from __future__ import annotations

import collections
import threading

import numpy as np

from .._native import C

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

FILTERS = {
    # pointwise
    "gray[:ref|bt601]": "grayscale (ref: kernel.cu:31-44 weights/truncation; bt601: OpenCV, kern.cpp:73)",
    "contrast:F[:cv]": "trunc(clamp(F*(p-128)+128)) (kernel.cu:49-58); ':cv' = OpenCV rounding (kern.cpp:74)",
    "invert": "255 - p",
    "brightness:D": "sat(p + D)",
    "threshold:T": "p >= T ? 255 : 0",
    "expand": "gray -> 3 identical channels (GRAY2BGR, kernel.cu:210)",
    # stencils
    "emboss3 / emboss5": "kernel.cu:64-94 filters (3x3 and diagonal 5x5)",
    "gaussian3/5/7": "binomial Gaussian, integer, rounded",
    "box3 / box5": "box mean, rounded",
    "sharpen": "[[0,-1,0],[-1,5,-1],[0,-1,0]]",
    "laplace": "[[0,1,0],[1,-4,1],[0,1,0]]",
    "sobel": "sat(|Gx| + |Gy|)",
    "sobel_l2 / magnitude": "sat(round(sqrt(Gx^2 + Gy^2))), exact integer rounding",
    "blur:K[:sigma][:lsb]": "KxK float Gaussian (separable MFMA path), K <= 33; :lsb = every output within 1 LSB, "
                            "2.5x fewer MFMAs",
    "conv:K:w0;w1;...[:lsb]": "generic KxK float correlation (MFMA path); :lsb = within 1 LSB, 2/3 of the MFMAs",
    "sepconv:K:h..:v..[:lsb]": "rank-one KxK float correlation v (x) h (separable MFMA path)",
    "...@border": "per-stencil border: reflect101 | replicate | constant | skip",
}

_cache_lock = threading.Lock()
_engines: "collections.OrderedDict" = collections.OrderedDict()
_MAX_ENGINES = 8


def _is_tensor(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor)


def _shape(x):
    if x.ndim == 2:
        return x.shape[1], x.shape[0], 1
    if x.ndim == 3 and x.shape[2] in (1, 3):
        return x.shape[1], x.shape[0], x.shape[2]
    raise ValueError(f"image must be HxW or HxWx3 uint8, got shape {tuple(x.shape)}")


def _engine(W, H, Cc, chain, border, fuse, device_index, halo=True):
    key = (W, H, Cc, chain, border, fuse, device_index, halo)
    with _cache_lock:
        eng = _engines.get(key)
        if eng is not None:
            _engines.move_to_end(key)
            return eng
        cfg = C.EngineConfig()
        cfg.W, cfg.H, cfg.C = int(W), int(H), int(Cc)
        cfg.chain = chain
        cfg.border = C.parse_border(border)
        cfg.fuse = bool(fuse)
        cfg.halo = bool(halo)
        cfg.device = int(device_index)
        cfg.backend = C.Backend.device
        eng = C.Engine(cfg)
        eng._stream = None
        # one call at a time per engine: the C++ calls release the GIL and the
        # engine's ping-pong buffers are shared by every call with this key
        eng._lock = threading.Lock()
        _engines[key] = eng
        while len(_engines) > _MAX_ENGINES:
            _engines.popitem(last=False)
        return eng


def apply(image, chain: str, border: str = "reflect101", fuse: bool = True):
    """Apply a filter chain to one image (tensor on GPU -> HIP kernels; numpy / CPU
    tensor -> the threaded host executor, bit-identical to the golden path).
    A 4-D BxHxWxC input is a batch of frames; the result stacks the frames."""
    if image.ndim == 4:
        if image.shape[3] not in (1, 3):
            raise ValueError(f"a batch must be BxHxWxC with C in (1, 3), got {tuple(image.shape)}")
        outs = [apply(image[b], chain, border, fuse) for b in range(image.shape[0])]
        if _is_tensor(image):
            return torch.stack(outs) if outs else image.new_empty((0,) + tuple(image.shape[1:]))
        return np.stack(outs) if outs else np.empty((0,) + tuple(image.shape[1:]), np.uint8)
    if _is_tensor(image) and image.is_cuda:
        if image.dtype != torch.uint8:
            raise TypeError("image tensor must be uint8")
        x = image.contiguous()
        W, H, Cc = _shape(x)
        if Cc == 1 and x.ndim == 3:
            x = x.reshape(H, W)
        eng = _engine(W, H, Cc, chain, border, fuse, x.device.index)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        cout = eng.out_channels
        out = torch.empty((H, W) if cout == 1 else (H, W, cout), dtype=torch.uint8, device=x.device)
        with eng._lock:
            if eng._stream != stream:
                # the new stream waits for the work still queued on the old one
                eng.use_external_stream(stream)
                eng._stream = stream
            eng.load_packed_ptr(x.data_ptr(), True)
            eng.run(1)
            eng.store_packed_ptr(out.data_ptr(), True)
        # keep x alive until the stream has consumed it
        x.record_stream(torch.cuda.current_stream(x.device))
        return out
    was_tensor = _is_tensor(image)
    arr = image.numpy() if was_tensor else np.asarray(image)
    if arr.dtype != np.uint8:
        raise TypeError("image must be uint8")
    if arr.ndim == 3 and arr.shape[2] == 1:
        arr = arr[:, :, 0]
    out = C.cpu_apply(np.ascontiguousarray(arr), chain, border, fuse)
    return torch.from_numpy(out) if was_tensor else out


def reference(image, chain: str, border: str = "reflect101"):
    """Golden CPU result of `chain`, applied op by op (no fusion)."""
    arr = image.detach().cpu().numpy() if _is_tensor(image) else np.asarray(image)
    return C.golden_apply_unfused(np.ascontiguousarray(arr), chain, border)


# ---- named convenience wrappers -------------------------------------------------
def grayscale(x, mode: str = "bt601"):
    return apply(x, f"gray:{mode}")


def contrast(x, factor: float = 3.5, rounding: str = "ref"):
    return apply(x, f"contrast:{factor}:{rounding}")


def invert(x):
    return apply(x, "invert")


def brightness(x, delta: int):
    return apply(x, f"brightness:{int(delta)}")


def threshold(x, t: int = 128):
    return apply(x, f"threshold:{int(t)}")


def gaussian_blur(x, ksize: int = 5, border: str = "reflect101"):
    if ksize in (3, 5, 7):
        return apply(x, f"gaussian{ksize}", border)
    return apply(x, f"blur:{ksize}", border)


def box_blur(x, ksize: int = 3, border: str = "reflect101"):
    return apply(x, f"box{ksize}", border)


def sobel(x, border: str = "reflect101"):
    return apply(x, "sobel", border)


def sharpen(x, border: str = "reflect101"):
    return apply(x, "sharpen", border)


def laplace(x, border: str = "reflect101"):
    return apply(x, "laplace", border)


def emboss(x, size: int = 3, border: str = "reflect101"):
    return apply(x, f"emboss{size}", border)


def conv2d(x, weights, border: str = "reflect101"):
    """Generic KxK float correlation on the MFMA path (weights: KxK array)."""
    w = np.asarray(weights, dtype=np.float64)
    K = w.shape[0]
    if w.shape != (K, K) or K % 2 == 0:
        raise ValueError("weights must be an odd KxK matrix")
    spec = ";".join(repr(float(v)) for v in w.reshape(-1))
    return apply(x, f"conv:{K}:{spec}", border)


def sep_conv2d(x, h, v, border: str = "reflect101"):
    """Rank-one KxK correlation, weights[dy][dx] = v[dy] * h[dx] (separable MFMA path)."""
    h = np.asarray(h, dtype=np.float64).reshape(-1)
    v = np.asarray(v, dtype=np.float64).reshape(-1)
    K = h.shape[0]
    if v.shape[0] != K or K % 2 == 0:
        raise ValueError("h and v must have the same odd length")
    hs = ";".join(repr(float(t)) for t in h)
    vs = ";".join(repr(float(t)) for t in v)
    return apply(x, f"sepconv:{K}:{hs}:{vs}", border)


def large_blur(x, ksize: int = 31, sigma: float = 0.0, border: str = "reflect101"):
    return apply(x, f"blur:{ksize}:{sigma}" if sigma > 0 else f"blur:{ksize}", border)


def clear_cache() -> None:
    with _cache_lock:
        _engines.clear()


__all__ = [
    "FILTERS", "apply", "reference", "grayscale", "contrast", "invert", "brightness", "threshold",
    "gaussian_blur", "box_blur", "sobel", "sharpen", "laplace", "emboss", "conv2d", "sep_conv2d", "large_blur", "clear_cache",
]
