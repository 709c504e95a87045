#!/usr/bin/env python3
"""Device copy bandwidth reference (torch.Tensor.copy_, ping-pong) for the
working-set sizes of the stencil benchmarks: the practical streaming ceiling the
kernels are compared against (full 16K RGB frame, one N=8 stripe, ...)."""
import sys

import torch

sizes = [int(s) for s in (sys.argv[1:] or [16384 * 16384 * 3, 16384 * 2048 * 3, 16384 * 4096 * 3, 8192 * 8192])]
for n in sizes:
    x = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    for _ in range(5):
        y.copy_(x)
        x.copy_(y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 100
    e0.record()
    for _ in range(it // 2):
        y.copy_(x)
        x.copy_(y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"copy {n / 2**20:8.1f} MiB: {ms:.4f} ms  {2 * n / ms / 1e9:.2f} TB/s (read + write)")
