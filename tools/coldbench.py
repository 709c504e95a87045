#!/usr/bin/env python3
"""Cache-cold stencil sweep: one rank's share of the N=8 headline (16384x2048 RGB
gaussian5 by default) filtered from HBM every step.

`--frames` engines (independent stripe copies, each with its own ping-pong
pair) share one HIP stream and are stepped round-robin, so a step's input was
last touched frames-1 steps earlier: with frames * (in + out) > 2 x 256 MiB the
Infinity Cache holds none of it.  Every (band, cap, store policy) candidate is
timed as the median of per-step device events over `--steps` steps.

    python tools/coldbench.py --shape 16384x2048x3 --chain gaussian5 --frames 4
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", default="gaussian5")
    ap.add_argument("--shape", default="16384x2048x3")
    ap.add_argument("--frames", type=int, default=4, help="stripe copies rotated over (1: cache-warm)")
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--bands", default="4,8,12,16,20,24,32,48,64")
    ap.add_argument("--caps", default="-1,0,1,2,3,4")
    ap.add_argument("--nt", default="0,1", help="store policies to try (STRIPE_NT)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from mpi_cuda_imagemanipulation_amd._native import C
    from mpi_cuda_imagemanipulation_amd.models import Pipeline

    W, H, Cc = (int(v) for v in a.shape.split("x"))
    pipe = Pipeline(a.chain)
    stream = torch.cuda.Stream()
    engines = []
    for f in range(a.frames):
        e = C.Engine(pipe.config(W, H, Cc, "device", device=0))
        e.use_external_stream(stream.cuda_stream)
        e.load_synthetic(1 + f)
        engines.append(e)
    torch.cuda.synchronize()
    npass = len(engines[0].bands)

    def timed(steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        with torch.cuda.stream(stream):
            ev[0].record(stream)
            for i in range(steps):
                engines[i % a.frames].run(1)
                ev[i + 1].record(stream)
        ev[-1].synchronize()
        t = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
        return t[len(t) // 2], t[0]

    # clock ramp
    for e in engines:
        e.set_tuning([16] * npass, [-1] * npass)
    for _ in range(20):
        timed(a.steps)
    rows = []
    for nt in [int(x) for x in a.nt.split(",")]:
        os.environ["STRIPE_NT"] = str(nt)
        for band in [int(x) for x in a.bands.split(",")]:
            for cap in [int(x) for x in a.caps.split(",")]:
                for e in engines:
                    e.set_tuning([band] * npass, [cap] * npass)
                timed(a.frames * 2)
                med, mn = timed(a.steps)
                rows.append({"nt": nt, "band": band, "cap": cap, "median_ms": round(med, 5), "min_ms": round(mn, 5)})
                print(f"nt {nt} band {band:3d} cap {cap:2d}: median {med:.5f} ms  min {mn:.5f}", flush=True)
    best = min(rows, key=lambda r: r["median_ms"])
    nbytes = W * H * Cc * 2
    print(json.dumps({"shape": a.shape, "chain": a.chain, "frames": a.frames, "xcd": os.environ.get("STRIPE_XCD", "auto"),
                      "best": best, "gb_s_best": round(nbytes / (best["median_ms"] * 1e-3) / 1e9, 1)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "best": best}, f, indent=1)


if __name__ == "__main__":
    main()
