"""Process exit under rocprofv3 with a one-rank RCCL communicator: `keep`
leaves the communicator to interpreter teardown, `release` drops it (and
synchronises) before returning.  Used to find which object a profiled
bench.py run crashed on at exit (profiles/r5/bench/README.md)."""
import gc
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mpi_cuda_imagemanipulation_amd import parallel  # noqa: E402


def main(mode):
    ctx = parallel.init("rccl")
    x = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    print("comm ready", ctx.transport, float(x.sum()), flush=True)
    if mode == "dedicated":  # a CU-masked stream of the process-wide pool, used by torch
        from mpi_cuda_imagemanipulation_amd._native import C
        s = torch.cuda.ExternalStream(C.dedicated_stream(0, 0))
        with torch.cuda.stream(s):
            x.mul_(2)
        torch.cuda.synchronize()
    if mode == "frames":  # the headline's frame stream on a small frame
        import mpi_cuda_imagemanipulation_amd as m
        fs = parallel.FrameStream(ctx, m.models.Pipeline("gaussian5", halo_depth=1), 4096, 512, 3)
        fs.load_synthetic(1)
        for i in range(8):
            fs.step(i)
        fs.synchronize()
        print("frames", len(fs), fs.queues, flush=True)
    if mode == "release":
        ctx.comm = None
        del ctx
        gc.collect()
        torch.cuda.synchronize()
    return ctx if mode == "keep" else None


if __name__ == "__main__":
    keep = main(sys.argv[1] if len(sys.argv) > 1 else "keep")
    print("exit", flush=True)
