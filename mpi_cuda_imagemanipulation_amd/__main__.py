"""`python -m mpi_cuda_imagemanipulation_amd` - Python front end of the native
engine for any image format Pillow reads (the native `bin/stripe` CLI is
PNM-only).  The reference's single command (kernel.cu main: load, distribute,
gray -> contrast -> emboss, gather, write) is `run --preset ref-gpu`.

  python -m mpi_cuda_imagemanipulation_amd run --input in.jpg --output out.png \\
      --chain gray:ref,contrast:3.5,emboss3 --ranks 4 --backend local
  python -m mpi_cuda_imagemanipulation_amd convert in.jpg out.ppm
  python -m mpi_cuda_imagemanipulation_amd filters
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
    r.add_argument("--backend", default="auto", choices=["auto", "local", "host"],
                   help="local: N logical ranks on this process's GPU; host: CPU golden engine")
    r.add_argument("--border", default=None)
    r.add_argument("--iterations", type=int, default=1)
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
    img = utils.read_image(a.input)
    if a.preset:
        pipe = models.Pipeline.preset(a.preset)
    else:
        pipe = models.Pipeline(a.chain or "gaussian5", border=a.border or "reflect101")
    backend = a.backend
    if backend == "auto":
        import torch

        backend = "local" if torch.cuda.is_available() else "host"
    t0 = time.perf_counter()
    out = pipe.run_distributed(img, a.ranks, backend=backend, iterations=a.iterations)
    ms = (time.perf_counter() - t0) * 1e3
    utils.write_image(a.output, out)
    print(json.dumps({"cmd": "run", "input": a.input, "output": a.output, "shape": list(img.shape),
                      "chain": pipe.spec.chain, "ranks": a.ranks, "backend": backend, "wall_ms": round(ms, 3)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
