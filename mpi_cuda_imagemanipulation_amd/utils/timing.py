"""Timing helpers: host wall clock and device (HIP event) timers.

Reference timing: std::chrono::high_resolution_clock around kernels + D2H +
GRAY2BGR + MPI_Gather, printed by rank 0 only (kernel.cu:190,226-232)."""
from __future__ import annotations

import contextlib
import time


class Timer:
    def __init__(self) -> None:
        self.elapsed_ms = 0.0

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.elapsed_ms = (time.perf_counter() - self._t0) * 1e3
        return False


@contextlib.contextmanager
def cuda_timer(result: dict, key: str = "ms"):
    import torch

    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    e.synchronize()
    result[key] = s.elapsed_time(e)
