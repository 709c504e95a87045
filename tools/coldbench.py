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
    ap.add_argument("--frames", type=int, default=0,
                    help="stripe copies rotated over (0: enough for 3 x 256 MiB; 1: cache-warm)")
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--bands", default="4,8,12,16,20,24,32,48,64")
    ap.add_argument("--caps", default="-1,0,1,2,3,4")
    ap.add_argument("--nt", default="0,1", help="store policies to try (STRIPE_NT)")
    ap.add_argument("--streams", type=int, default=1, help="streams the frames alternate over")
    ap.add_argument("--stage-timing", type=int, default=1, help="engine device-event stage timing (0: off)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from mpi_cuda_imagemanipulation_amd._native import C
    from mpi_cuda_imagemanipulation_amd.models import Pipeline

    W, H, Cc = (int(v) for v in a.shape.split("x"))
    if a.frames <= 0:
        a.frames = max(2, -(-3 * (256 << 20) // (2 * W * H * Cc)))
    pipe = Pipeline(a.chain)
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    engines = []
    for f in range(a.frames):
        e = C.Engine(pipe.config(W, H, Cc, "device", device=0))
        e.use_external_stream(streams[f % a.streams].cuda_stream)
        e.stage_timing = bool(a.stage_timing)
        e.load_synthetic(1 + f)
        engines.append(e)
    torch.cuda.synchronize()
    npass = len(engines[0].bands)

    def timed(steps):
        # end of step i on its frame's stream; step time = end(i) - end(i - 1)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        torch.cuda.synchronize()
        ev[0].record(streams[0])
        for st in streams[1:]:
            st.wait_event(ev[0])
        for i in range(steps):
            engines[i % a.frames].run(1)
            ev[i + 1].record(streams[(i % a.frames) % a.streams])
        torch.cuda.synchronize()
        t = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
        # the same steps with events at the two ends only (a timestamped event
        # between dependent kernels costs the GPU several microseconds)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        for st in streams[1:]:
            st.wait_event(e0)
        for i in range(steps):
            engines[i % a.frames].run(1)
        for st in streams[1:]:
            streams[0].wait_stream(st)
        e1.record(streams[0])
        torch.cuda.synchronize()
        return t[len(t) // 2], e0.elapsed_time(e1) / steps

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
                rows.append({"nt": nt, "band": band, "cap": cap, "median_ms": round(med, 5), "mean_ms": round(mn, 5)})
                print(f"nt {nt} band {band:3d} cap {cap:2d}: median {med:.5f} ms  mean {mn:.5f}", flush=True)
    best = min(rows, key=lambda r: r["mean_ms"])
    nbytes = W * H * Cc * 2
    print(json.dumps({"shape": a.shape, "chain": a.chain, "frames": a.frames, "streams": a.streams,
                      "stage_timing": a.stage_timing, "xcd": os.environ.get("STRIPE_XCD", "auto"),
                      "best": best, "gb_s_best": round(nbytes / (best["mean_ms"] * 1e-3) / 1e9, 1)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "best": best}, f, indent=1)


if __name__ == "__main__":
    main()
