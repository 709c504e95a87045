"""Independent numpy mirror of the filter spec.

Written directly from the spec, not from the C++ code, so the golden path is
checked against a second implementation.  Images: HxW or HxWx3 uint8, RGB.
"""
from __future__ import annotations

import numpy as np

_PAD = {"reflect101": "reflect", "replicate": "edge", "constant": "constant"}

STENCILS = {
    "emboss3": (np.array([[-2, -1, 0], [-1, 1, 1], [0, 1, 2]]), 1),
    "emboss5": (np.diag([4, 4, 1, -4, -4]), 1),
    "sharpen": (np.array([[0, -1, 0], [-1, 5, -1], [0, -1, 0]]), 1),
    "laplace": (np.array([[0, 1, 0], [1, -4, 1], [0, 1, 0]]), 1),
    "gaussian3": (np.outer([1, 2, 1], [1, 2, 1]), 16),
    "gaussian5": (np.outer([1, 4, 6, 4, 1], [1, 4, 6, 4, 1]), 256),
    "gaussian7": (np.outer([1, 6, 15, 20, 15, 6, 1], [1, 6, 15, 20, 15, 6, 1]), 4096),
    "box3": (np.ones((3, 3), int), 9),
    "box5": (np.ones((5, 5), int), 25),
}
SOBEL_X = np.outer([1, 2, 1], [-1, 0, 1])


def gray_ref(img):
    f = img.astype(np.float32).astype(np.float64)
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    return (np.trunc(b * 0.11) + np.trunc(g * 0.59) + np.trunc(r * 0.3)).astype(np.uint8)


def gray_bt601(img):
    x = img.astype(np.int64)
    return ((x[..., 0] * 4899 + x[..., 1] * 9617 + x[..., 2] * 1868 + 8192) >> 14).astype(np.uint8)


def contrast_ref(x, f=3.5):
    v = np.float32(f) * (x.astype(np.int32) - 128).astype(np.float32) + np.float32(128)
    return np.clip(v, 0, 255).astype(np.float32).astype(np.uint8)


def contrast_cv(x, f=3.0):
    v = x.astype(np.float32) * np.float32(f) + np.float32(128 - 128 * f)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def invert(x):
    return (255 - x.astype(np.int32)).astype(np.uint8)


def brightness(x, d):
    return np.clip(x.astype(np.int32) + d, 0, 255).astype(np.uint8)


def _pad(ch, R, border):
    return np.pad(ch, R, mode=_PAD[border])


def _correlate(ch, w, border):
    K = w.shape[0]
    R = K // 2
    H, W = ch.shape
    p = _pad(ch.astype(np.int64), R, border)
    s = np.zeros((H, W), np.int64)
    for dy in range(K):
        for dx in range(K):
            if w[dy, dx]:
                s += int(w[dy, dx]) * p[dy:dy + H, dx:dx + W]
    return s


def _per_channel(img, fn):
    if img.ndim == 2:
        return fn(img)
    return np.stack([fn(img[..., c]) for c in range(img.shape[2])], axis=-1)


def stencil(img, name, border="reflect101"):
    skip = border == "skip"
    b = "reflect101" if skip else border

    def one(ch):
        if name in ("sobel", "sobel_l2"):
            gx = _correlate(ch, SOBEL_X, b)
            gy = _correlate(ch, SOBEL_X.T, b)
            if name == "sobel":
                out = np.clip(np.abs(gx) + np.abs(gy), 0, 255)
            else:  # double sqrt is correctly rounded and never lands on a half-integer
                out = np.clip(np.rint(np.sqrt((gx.astype(np.int64) ** 2 + gy.astype(np.int64) ** 2).astype(np.float64))), 0, 255)
            R = 1
        else:
            w, div = STENCILS[name]
            R = w.shape[0] // 2
            s = _correlate(ch, w, b)
            out = np.clip((s + div // 2) // div if div > 1 else s, 0, 255)
        out = out.astype(np.uint8)
        if skip:
            # kernel.cu:83 bounds minus its wrap/OOB column W-R and row H-R
            # (deliberate deviation, README "Parity"): those keep the input too
            H, W = ch.shape
            yy, xx = np.mgrid[0:H, 0:W]
            m = (xx <= R) | (yy <= R) | (xx >= W - R) | (yy >= H - R)
            out[m] = ch[m]
        return out

    return _per_channel(img, one)


def gaussian_1d(K, sigma=0.0):
    if sigma <= 0:
        sigma = 0.3 * ((K - 1) * 0.5 - 1) + 0.8
    x = np.arange(K) - K // 2
    g = np.exp(-(x * x) / (2 * sigma * sigma))
    return g / g.sum()


def blur(img, K, border="reflect101"):
    g = gaussian_1d(K)
    w = np.outer(g, g).astype(np.float32).astype(np.float64)
    R = K // 2

    def one(ch):
        H, W = ch.shape
        p = _pad(ch.astype(np.float64), R, border)
        s = np.zeros((H, W))
        for dy in range(K):
            for dx in range(K):
                s += w[dy, dx] * p[dy:dy + H, dx:dx + W]
        return np.clip(np.rint(s), 0, 255).astype(np.uint8)

    return _per_channel(img, one)


def expand(g):
    return np.repeat(g[..., None], 3, axis=-1)
