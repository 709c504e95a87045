"""Frame-stream step time with the frames' two streams from PyTorch's stream
pool (plain HIP streams, which share the GPU_MAX_HW_QUEUES hardware queues
round-robin) against two streams with hardware queues of their own
(C.stream_create: CU-masked streams), one rank, alternating rounds.

    python tools/stream_probe.py [--shape 16384x2048x3] [--chain gaussian5] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mpi_cuda_imagemanipulation_amd as m  # noqa: E402
from mpi_cuda_imagemanipulation_amd import parallel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16384x2048x3")
    ap.add_argument("--chain", default="gaussian5")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pre", default="", help="comma list run first, as bench.py does: roofline, ring")
    a = ap.parse_args()
    W, H, Cc = (int(v) for v in a.shape.split("x"))
    C = m._C
    ctx = parallel.init("auto")
    pre = [p for p in a.pre.split(",") if p]
    if "ring" in pre:
        parallel.ring_check(ctx, nbytes=2 * W * Cc * 2, iters=200)
    if "roofline" in pre:
        C.copy_roofline(0, W * H * Cc, 4, 20)
    fs = parallel.FrameStream(ctx, m.models.Pipeline(a.chain, halo_depth=1), W, H, Cc)
    fs.load_synthetic(1)
    fs.tune()
    pool = list(fs.streams)
    handles = [C.stream_create(0, True) for _ in range(2)]
    dedicated = [torch.cuda.ExternalStream(h) for h in handles]

    def timed(streams, n):
        fs.streams = streams
        fs.set_streams(n)
        for i in range(2 * len(fs.frames)):
            fs.step(i)
        fs.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            fs.step(i)
        fs.synchronize()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.steps

    res = {"pool@1": [], "pool@2": [], "dedicated@2": []}
    for _ in range(a.rounds):
        res["pool@1"].append(round(timed(pool, 1), 5))
        res["pool@2"].append(round(timed(pool, 2), 5))
        res["dedicated@2"].append(round(timed(dedicated, 2), 5))
    fs.streams = pool
    fs.set_streams(1)
    fs.synchronize()
    for h in handles:
        C.stream_destroy(h)
    print(json.dumps({"shape": a.shape, "chain": a.chain, "pre": pre, "frames": len(fs.frames), "cache": fs.cache,
                      "ms_per_step": res}))


if __name__ == "__main__":
    main()
