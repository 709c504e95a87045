#!/usr/bin/env python3
"""Single-GPU kernel benchmark: time `iters` resident passes of each chain.

    python tools/kbench.py --chains gaussian5,sobel --shape 16384x16384x3 --iters 50

Reports ms per pass, Mpixels/s and the effective HBM bandwidth (input + output
bytes of every pass, counted once).  Used for tuning and under rocprofv3.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", default="gaussian5")
    ap.add_argument("--shape", default="16384x16384x3")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bands", default="0", help="comma list of stencil band heights (0 = static heuristic, -1 = engine autotune)")
    ap.add_argument("--no-fuse", action="store_true")
    ap.add_argument("--graphs", action="store_true", help="replay iterations from a captured hipGraph")
    a = ap.parse_args()
    import torch

    from mpi_cuda_imagemanipulation_amd._native import C
    from mpi_cuda_imagemanipulation_amd.models import Pipeline

    W, H, Cc = (int(v) for v in a.shape.split("x"))
    for chain, band in [(c, int(b)) for c in (a.chains.split("|") if "|" in a.chains else a.chains.split(";")) if c for b in a.bands.split(",")]:
        pipe = Pipeline(chain, fuse=not a.no_fuse)
        cfg = pipe.config(W, H, Cc, "device", device=0)
        cfg.band = max(band, 0)
        cfg.autotune = band < 0
        cfg.graphs = a.graphs
        e = C.Engine(cfg)
        info = C.plan_info(chain, Cc)
        e.load_synthetic(1)
        iters = a.iters if info["cout"] == info["cin"] else 1
        e.run(a.warmup if iters > 1 else 1)
        e.synchronize()
        t_ramp = time.perf_counter()  # clock ramp: ~50 ms of this chain before timing
        while time.perf_counter() - t_ramp < 0.05:
            e.rewind()
            e.run(1)
            e.synchronize()
        e.rewind()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(max(1, a.iters // iters)):
            if iters == 1:
                e.rewind()
            e.run(iters)
        e.synchronize()
        t1 = time.perf_counter()
        n = iters * max(1, a.iters // iters)
        ms = (t1 - t0) * 1e3 / n
        byts = sum(W * H * (p["cin"] + p["cout"]) for p in info["passes"])
        print(json.dumps({"chain": chain if len(chain) <= 48 else chain[:40] + "...", "band": band, "shape": a.shape, "ms": round(ms, 4),
                          "mpx_s": round(W * H / ms / 1e3, 1), "GBps": round(byts / ms / 1e6, 1),
                          "passes": len(info["passes"]), "graphs": e.graph_launches > 0,
                          "bands": e.bands, "caps": e.caps}), flush=True)
        del e


if __name__ == "__main__":
    main()
