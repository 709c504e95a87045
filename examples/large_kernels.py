#!/usr/bin/env python3
"""Large-window filters (SURVEY config 5) through the Python API: a 31x31
Gaussian on the separable MFMA kernel (exact and `:lsb`), an asymmetric
rank-one `sepconv`, and an arbitrary (non-separable) 31x31 correlation on the
i8-digit Toeplitz MFMA kernel -- each checked against the golden CPU path on
the same image (outputs agree within 1 LSB, at ties only) and timed.

    python examples/large_kernels.py [--shape WxHxC] [--iters N]

On a GPU box the image is a device tensor and the HIP kernels run; without a
GPU the same calls run the host executor (bit-identical to the golden path).
The reference has no large-window filter (its only stencil is the 3x3/5x5
emboss, kernel.cu:64-94); these are the framework's MFMA showcase.
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096x2048x3", help="WxHxC, C in 1 or 3")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import mpi_cuda_imagemanipulation_amd as m
    from mpi_cuda_imagemanipulation_amd import ops

    W, H, Cc = (int(v) for v in a.shape.split("x"))
    rng = np.random.default_rng(a.seed)
    img = rng.integers(0, 256, size=(H, W, Cc) if Cc == 3 else (H, W), dtype=np.uint8)
    try:
        import torch

        gpu = torch.cuda.is_available()
    except ImportError:  # pragma: no cover - torch is part of the image
        torch, gpu = None, False
    x = torch.from_numpy(img).cuda() if gpu else img
    where = "on GPU" if gpu else "on host"

    K = 31
    g = np.exp(-((np.arange(K) - K // 2) ** 2) / (2 * 5.0**2))
    g /= g.sum()
    h = rng.uniform(-0.25, 1.0, K)
    h /= h.sum()
    w = rng.uniform(-1.0, 1.0, (K, K)) / (K * K / 4)
    cases = [
        ("blur:31 (separable MFMA, exact)", lambda t: ops.apply(t, "blur:31"), "blur:31"),
        ("blur:31:lsb (separable MFMA, within 1 LSB)", lambda t: ops.apply(t, "blur:31:lsb"), "blur:31"),
        ("sepconv:31 asymmetric (separable MFMA)", lambda t: ops.sep_conv2d(t, h, g),
         "sepconv:31:" + ";".join(repr(float(v)) for v in h) + ":" + ";".join(repr(float(v)) for v in g)),
        ("conv:31 arbitrary weights (i8-digit Toeplitz MFMA)", lambda t: ops.conv2d(t, w),
         "conv:31:" + ";".join(repr(float(v)) for v in w.reshape(-1))),
    ]
    print(f"{W}x{H}x{Cc} {where}" + ("" if gpu else " (host executor: the kernels named below are the GPU paths)"))
    for name, fn, golden_chain in cases:
        out = fn(x)
        if gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            out = fn(x)
        if gpu:
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.iters
        got = out.cpu().numpy() if gpu else out
        ref = m._C.golden_apply(img, golden_chain, "reflect101", True)
        d = np.abs(got.astype(int) - ref.astype(int))
        print(f"{name}: {ms:.3f} ms ({W * H / ms / 1e3:.1f} Mpx/s), max |diff| vs golden {d.max()}, "
              f"{(d != 0).mean() * 100:.3f} % off by one")
        if d.max() > 1:
            raise SystemExit(f"{name}: off by {d.max()} LSB")


if __name__ == "__main__":
    main()
