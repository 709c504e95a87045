"""`python -m mpi_cuda_imagemanipulation_amd` - Python front end of the native
engine for any image format Pillow reads (the native `bin/stripe` CLI is
PNM-only).  The reference's single command (kernel.cu main: load, distribute,
gray -> contrast -> emboss, gather, write) is `run --preset ref-gpu`.

  python -m mpi_cuda_imagemanipulation_amd run --input in.jpg --output out.png \\
      --chain gray:ref,contrast:3.5,emboss3 --ranks 4 --backend local
  python -m mpi_cuda_imagemanipulation_amd convert in.jpg out.ppm
  python -m mpi_cuda_imagemanipulation_amd filters

One process per rank, like the reference's `mpiexec -n N kernel.exe`
(kernel.cu:104-137 Init/Bcast/Scatter, :223-225 Gather): under torchrun,
`--backend rccl` (one GPU per process, RCCL over xGMI) or `--backend gloo`
(CPU golden engine) - rank 0 reads the image, broadcasts its shape (the
reference's 4-int metadata Bcast), scatters the stripes, every rank filters
its stripe with halo exchange, rank 0 gathers and writes:

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m mpi_cuda_imagemanipulation_amd \\
      run --input in.jpg --output out.png --preset ref-gpu --backend rccl
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def main(argv=None) -> int:
    from . import models, ops, utils
    from ._native import C

    ap = argparse.ArgumentParser(prog="python -m mpi_cuda_imagemanipulation_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run", help="filter an image (distributed over in-process ranks)")
    r.add_argument("--input", required=True)
    r.add_argument("--output", required=True)
    r.add_argument("--chain", default=None)
    r.add_argument("--preset", default=None, choices=sorted(models.PRESETS))
    r.add_argument("--ranks", type=int, default=1)
    r.add_argument("--backend", default="auto", choices=["auto", "local", "host", "rccl", "gloo", "gloo-gpu"],
                   help="local: N logical ranks on this process's GPU; host: CPU golden engine; "
                        "rccl / gloo / gloo-gpu: one process per rank under torchrun (RANK / WORLD_SIZE env; "
                        "gloo-gpu: GPU engines sharing GPUs, gloo transport through pinned host memory)")
    r.add_argument("--border", default=None)
    r.add_argument("--iterations", type=int, default=1)
    r.add_argument("--dist-chunks", type=int, default=0,
                   help="> 1 ranks, one iteration, single-pass chains: ship / filter / gather the "
                        "stripes in this many overlapped row chunks (bit-identical)")
    r.add_argument("--row-weights", default=None,
                   help="comma list, one share per rank (weighted split, e.g. a larger root share for "
                        "--dist-chunks); default: even rows")
    r.add_argument("--verbose", "-v", action="store_true", help="rank-prefixed progress log on stderr")
    c = sub.add_parser("convert", help="convert between image formats")
    c.add_argument("src")
    c.add_argument("dst")
    sub.add_parser("filters", help="list the filter syntax")
    a = ap.parse_args(argv)

    if a.cmd == "filters":
        for k, v in ops.FILTERS.items():
            print(f"{k:24s} {v}")
        return 0
    if a.cmd == "convert":
        utils.write_image(a.dst, utils.read_image(a.src))
        return 0
    if a.preset:
        pipe = models.Pipeline.preset(a.preset)
    else:
        pipe = models.Pipeline(a.chain or "gaussian5", border=a.border or "reflect101")
    pipe.dist_chunks = a.dist_chunks
    weights = [float(v) for v in a.row_weights.split(",")] if a.row_weights else None
    if a.verbose:
        import os

        os.environ["STRIPE_LOG"] = "INFO"
    if a.backend in ("rccl", "gloo", "gloo-gpu"):
        return _run_per_process(a, pipe)
    img = utils.read_image(a.input)
    backend = a.backend
    if backend == "auto":
        import torch

        backend = "local" if torch.cuda.is_available() else "host"
    t0 = time.perf_counter()
    log = utils.get_logger("cli", 0)
    log.info("run %s on %s, %d ranks (%s)", pipe.spec.chain, img.shape, a.ranks, backend)
    out = pipe.run_distributed(img, a.ranks, backend=backend, iterations=a.iterations, row_weights=weights)
    ms = (time.perf_counter() - t0) * 1e3
    utils.write_image(a.output, out)
    print(json.dumps({"cmd": "run", "input": a.input, "output": a.output, "shape": list(img.shape),
                      "chain": pipe.spec.chain, "ranks": a.ranks, "backend": backend, "wall_ms": round(ms, 3)}))
    return 0


def _run_per_process(a, pipe) -> int:
    """One rank per process (torchrun env): root load -> metadata broadcast ->
    scatter -> per-stripe chain with halo exchange -> gather -> root write."""
    import numpy as np
    import torch.distributed as dist

    from . import parallel, utils

    ctx = parallel.init(a.backend)
    log = utils.get_logger("cli", ctx.rank)
    img = utils.read_image(a.input) if ctx.rank == 0 else None
    meta = [None if img is None else tuple(img.shape)]
    if ctx.world > 1:
        dist.broadcast_object_list(meta, src=0)
    shape = meta[0]
    H, W = shape[:2]
    Cc = 1 if len(shape) == 2 else shape[2]
    weights = [float(v) for v in a.row_weights.split(",")] if a.row_weights else None
    dp = parallel.DistributedPipeline(ctx, pipe, W, H, Cc, root_buffers=True, row_weights=weights)
    log.info("stripe rows %s of %dx%dx%d, chain %s", dp.stripe, W, H, Cc, pipe.spec.chain)
    dp.load_root(img)
    if ctx.world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if a.iterations == 1 and dp.engine.dist_chunks(a.dist_chunks) > 0:
        dp.engine.run_dist(a.dist_chunks)
    else:
        dp.scatter()
        dp.run(a.iterations)
        dp.gather()
    dp.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    log.info("dist step %.3f ms", ms)
    if ctx.rank == 0:
        out = dp.result_root()
        utils.write_image(a.output, np.ascontiguousarray(out))
        print(json.dumps({"cmd": "run", "input": a.input, "output": a.output, "shape": list(shape),
                          "chain": pipe.spec.chain, "ranks": ctx.world, "backend": a.backend,
                          "stripe_rows": dp.stripe[1], "dist_ms": round(ms, 3)}))
    if ctx.world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
