#!/usr/bin/env python3
"""A stream of independent frames through the distributed pipeline -- the
throughput mode behind bench.py's headline: one process per GPU, each frame
row-partitioned with the halo exchanged every step, frames stepped
round-robin over alternating streams, the halo schedule measured on the real
transport first.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/frame_stream.py --frames 64
    python examples/frame_stream.py --backend gloo          # CPU, one rank

Prints rank 0's frames per second and the schedule it chose.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chain", default="gaussian5")
    ap.add_argument("--shape", default="4096x4096x3")
    ap.add_argument("--frames", type=int, default=32, help="frames to push through")
    ap.add_argument("--backend", default="auto", choices=["auto", "rccl", "gloo", "gloo-gpu"])
    a = ap.parse_args()

    import mpi_cuda_imagemanipulation_amd as m
    from mpi_cuda_imagemanipulation_amd import parallel

    W, H, Cc = (int(v) for v in a.shape.split("x"))
    ctx = parallel.init(a.backend)
    fs = parallel.FrameStream(ctx, m.models.Pipeline(a.chain, halo_depth=1), W, H, Cc)
    fs.load_synthetic(seed=1)
    fs.tune()
    reduce_max, barrier = (lambda v: v), (lambda: None)
    if ctx.world > 1:
        import torch
        import torch.distributed as dist

        dev = "cuda" if ctx.transport == "rccl" else "cpu"

        def reduce_max(v):
            t = torch.tensor([v], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())

        barrier = dist.barrier
    sched = fs.pick_schedule(reduce_max, barrier)
    fs.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        fs.step()
    fs.synchronize()
    barrier()
    dt = reduce_max(time.perf_counter() - t0)
    if ctx.rank == 0:
        print(f"{a.frames} frames of {a.shape} {a.chain} on {ctx.world} rank(s) ({ctx.transport or 'host'}): "
              f"{a.frames / dt:.1f} frames/s, {W * H * a.frames / dt / 1e6:.0f} Mpx/s; "
              f"{len(fs)} frame buffers, schedule {sched['chosen']} on {sched['streams']} stream(s)")


if __name__ == "__main__":
    main()
