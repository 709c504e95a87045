"""Independent float oracles for the conv / blur filters.

The spec (golden.cpp): out = sat(rne(sum_{dy,dx} w32[dy,dx] *
in[y+dy-R, x+dx-R])) with the weights rounded to f32 first and the sum exact
(f64).  These oracles compute that sum with third-party code -- scipy.ndimage
and torch.nn.functional.conv2d in float64 -- so the C++ golden path and the HIP
kernels are not only checked against each other.

Comparisons are tie-aware: a float path may round a sum that lies within
`band` of k + 1/2 either way, so `compare` reports the mismatches OUTSIDE that
band (must be 0) separately from all mismatches (at most 1 LSB, inside the band).
"""
from __future__ import annotations

import numpy as np


def f32_weights(w) -> np.ndarray:
    return np.asarray(w, dtype=np.float64).astype(np.float32).astype(np.float64)


def blur_weights(C, K: int) -> np.ndarray:
    g = np.asarray(C.gaussian_1d(K), dtype=np.float64)
    return np.outer(g, g).astype(np.float32).astype(np.float64)


def _planes(img):
    return [img.astype(np.float64)] if img.ndim == 2 else [img[..., c].astype(np.float64) for c in range(img.shape[2])]


def _stack(planes, like):
    return planes[0] if like.ndim == 2 else np.stack(planes, axis=-1)


def scipy_sums(img: np.ndarray, w: np.ndarray, border: str) -> np.ndarray:
    from scipy import ndimage

    mode = {"reflect101": "mirror", "constant": "constant", "replicate": "nearest"}[border]
    return _stack([ndimage.correlate(p, w, mode=mode, cval=0.0) for p in _planes(img)], img)


def torch_sums(img: np.ndarray, w: np.ndarray, border: str, device: str = "cpu") -> np.ndarray:
    import torch
    import torch.nn.functional as F

    K = w.shape[0]
    R = K // 2
    mode = {"reflect101": "reflect", "constant": "constant", "replicate": "replicate"}[border]
    wt = torch.from_numpy(np.ascontiguousarray(w)).to(device=device, dtype=torch.float64).view(1, 1, K, K)
    out = []
    for p in _planes(img):
        x = torch.from_numpy(np.ascontiguousarray(p)).to(device=device).view(1, 1, *p.shape)
        H, W = p.shape
        if border == "reflect101" and (H <= R or W <= R):
            # torch's reflect pad needs pad < size: pad in steps (reflect101 is periodic)
            x = _reflect101_pad(x, R)
        else:
            x = F.pad(x, (R, R, R, R), mode=mode)
        out.append(F.conv2d(x, wt).view(H, W).cpu().numpy())  # conv2d is a correlation
    return _stack(out, img)


def _reflect101_pad(x, R):
    import torch

    H, W = x.shape[-2:]

    def idx(n):
        i = np.arange(-R, n + R)
        if n == 1:
            return np.zeros_like(i)
        per = 2 * (n - 1)
        j = np.mod(i, per)
        return np.where(j < n, j, per - j)

    return x[..., torch.from_numpy(idx(H))[:, None], torch.from_numpy(idx(W))[None, :]]


def finish(sums: np.ndarray) -> np.ndarray:
    """sat(rne(s)) as uint8 (np.rint rounds half to even)."""
    return np.clip(np.rint(sums), 0, 255).astype(np.uint8)


def compare(got: np.ndarray, sums: np.ndarray, band: float) -> dict:
    ref = finish(sums)
    d = np.abs(got.astype(np.int32) - ref.astype(np.int32))
    frac = np.abs(sums - np.floor(sums) - 0.5)
    in_band = (frac < band) & (sums > -0.5) & (sums < 255.5)
    return {
        "max_diff": int(d.max()) if d.size else 0,
        "mismatch": int((d != 0).sum()),
        "mismatch_outside_ties": int(((d != 0) & ~in_band).sum()),
        "tie_band_px": int(in_band.sum()),
        "n": int(d.size),
    }
