#!/usr/bin/env python3
"""Host-side cost of enqueuing one step, measured while the GPU is busy.

A long torch kernel queue keeps the GPU occupied, then N steps are enqueued
and the host clock measures the enqueue alone (the GPU cannot have caught up):
  run1       N x engine.run(1) from Python (frames rotated, like bench.py)
  runN       one engine.run(N) (the C++ loop)
  run1+ev    run(1) plus a torch event per step (bench.py's per-step timing)
Then the same steps are timed on the GPU (events) to compare with the kernel
time, so a host-bound step (GPU idle between kernels) shows as host >= device.

    python tools/hostbench.py --shape 16384x2048x3 --chain gaussian5
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", default="gaussian5")
    ap.add_argument("--shape", default="16384x2048x3")
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--n", type=int, default=200)
    a = ap.parse_args()
    import torch

    from mpi_cuda_imagemanipulation_amd._native import C
    from mpi_cuda_imagemanipulation_amd.models import Pipeline

    W, H, Cc = (int(v) for v in a.shape.split("x"))
    s = torch.cuda.Stream()
    engines = []
    for f in range(a.frames):
        e = C.Engine(Pipeline(a.chain).config(W, H, Cc, "device", device=0))
        e.use_external_stream(s.cuda_stream)
        e.load_synthetic(1 + f)
        engines.append(e)
    big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def busy(ms=60.0):
        # ~0.35 ms per 1 GiB fill: queue `ms` of GPU work on the stream
        with torch.cuda.stream(s):
            for _ in range(int(ms / 0.35)):
                big.fill_(1)

    out = {}
    for name in ("run1", "runN", "run1+ev"):
        for rep in range(2):
            torch.cuda.synchronize()
            busy()
            t0 = time.perf_counter()
            if name == "runN":
                engines[0].run(a.n)
            else:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.n)] if name == "run1+ev" else None
                for i in range(a.n):
                    engines[i % a.frames].run(1)
                    if ev:
                        ev[i].record(s)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
        out[name + "_host_us_per_step"] = round((t1 - t0) / a.n * 1e6, 2)
    # device time per step with and without a host-bound gap
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for i in range(a.n):
        engines[i % a.frames].run(1)
    e1.record(s)
    e1.synchronize()
    out["run1_device_us_per_step"] = round(e0.elapsed_time(e1) / a.n * 1e3, 2)
    busy()
    e0.record(s)
    for i in range(a.n):
        engines[i % a.frames].run(1)
    e1.record(s)
    e1.synchronize()
    out["run1_device_us_per_step_queued"] = round(e0.elapsed_time(e1) / a.n * 1e3, 2)
    out.update({"shape": a.shape, "chain": a.chain, "frames": a.frames})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
