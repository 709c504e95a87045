"""e2e scope (pinned host stripe -> H2D -> filter -> D2H -> pinned host) against
the row-chunk count of Engine.run_e2e: the pipeline's fill and drain cost
about one chunk's transfer each, so more chunks approach the host link's
both-directions floor until per-chunk launch overhead takes over.

    python tools/e2e_chunks.py [--shape 16384x16384x3] [--chain gaussian5] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mpi_cuda_imagemanipulation_amd as m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16384x16384x3")
    ap.add_argument("--chain", default="gaussian5")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--chunks", default="4,8,16,32,64")
    a = ap.parse_args()
    W, H, Cc = (int(v) for v in a.shape.split("x"))
    C = m._C
    e = C.Engine(m.models.Pipeline(a.chain).config(W, H, Cc, "device", device=0))
    e.alloc_host_io()
    e.host_input()[...] = C.synth_rows(1, W, Cc, 0, H)
    ref = None
    res = {}
    for rnd in range(2):
        for n in [int(v) for v in a.chunks.split(",")]:
            e.run_e2e(n)
            e.synchronize()
            out = e.host_output().copy()
            if ref is None:
                ref = out
            assert (out == ref).all(), f"chunks={n}: output differs"
            t0 = time.perf_counter()
            for _ in range(a.steps):
                e.run_e2e(n)
            e.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            res.setdefault(n, []).append(round(ms, 3))
    print(json.dumps({"shape": a.shape, "chain": a.chain, "ms_by_chunks": res}))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
