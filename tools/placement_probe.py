"""Does the frames' memory placement decide the two-stream gain of the
headline frame stream?  One process builds the 16384^2 RGB gaussian5 frame
stream several times, each after holding a different amount of device memory
(which shifts where the frames' buffers land), and times one and two streams
on each layout (profiles/r5/streams/README.md).

    python tools/placement_probe.py [--layouts 4] [--steps 100]
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
    ap.add_argument("--shape", default="16384x16384x3")
    ap.add_argument("--layouts", type=int, default=4)
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    W, H, Cc = (int(v) for v in a.shape.split("x"))
    ctx = parallel.init("auto")
    out = []
    tuning = None
    for k in range(a.layouts):
        hold = torch.empty((k * 384 + 64) << 20, dtype=torch.uint8, device="cuda")  # shifts later allocations
        fs = parallel.FrameStream(ctx, m.models.Pipeline("gaussian5", halo_depth=1), W, H, Cc, autotune=tuning is None)
        fs.load_synthetic(1)
        if tuning is None:
            fs.tune()
            e = fs.head.engine
            tuning = (e.bands, e.caps, e.policies, e.orders)
        for f in fs.frames:
            f.engine.set_tuning(*tuning)
        row = {"layout": k, "held_mib": hold.numel() >> 20}
        for rep in range(2):
            for n in (1, 2):
                fs.set_streams(n)
                for i in range(2 * len(fs.frames)):
                    fs.step(i)
                fs.synchronize()
                t0 = time.perf_counter()
                for i in range(a.steps):
                    fs.step(i)
                fs.synchronize()
                row.setdefault(f"s{n}", []).append(round((time.perf_counter() - t0) * 1e3 / a.steps, 5))
        out.append(row)
        print(json.dumps(row), flush=True)
        del fs, hold
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
