#!/usr/bin/env python3
"""The reference program's flow (kernel.cu:96-254) on this framework:
read a JPEG, gray (0.11 B + 0.59 G + 0.30 R, truncated) -> contrast 3.5 ->
3x3 emboss, expand back to 3 channels, write a JPEG -- on the GPU when one is
present (JPEG pixels made and encoded on the device, the chain as one fused
HIP kernel), else on the host executor (bit-identical to the golden path).

    python examples/reference_flow.py in.jpg out.jpg [--chain CHAIN] [--ranks N]

--ranks N > 1 runs the reference's row partition over N in-process ranks
(stripes filtered independently, remainder rows dropped: the `ref-gpu` preset
semantics) through the native CLI engine.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF_CHAIN = "gray:ref,contrast:3.5,emboss3@skip,expand"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("--chain", default=REF_CHAIN)
    ap.add_argument("--quality", type=int, default=95)
    ap.add_argument("--ranks", type=int, default=1)
    a = ap.parse_args()

    import mpi_cuda_imagemanipulation_amd as m

    gpu = False
    try:
        import torch

        gpu = torch.cuda.is_available()
    except ImportError:
        torch = None
    t0 = time.perf_counter()
    if a.ranks > 1:
        img = m.utils.read_image(a.input)
        pipe = m.models.Pipeline.preset("ref-gpu") if a.chain == REF_CHAIN else m.models.Pipeline(a.chain)
        out = pipe.run_distributed(img, a.ranks, "local" if gpu else "host", 1)
        m.utils.write_image(a.output, out, a.quality)
        where = f"{a.ranks} ranks ({'local GPU' if gpu else 'host'})"
    elif gpu:
        x = m.utils.read_image_device(a.input)          # Huffman on the host, pixels on the GPU
        y = m.ops.apply(x, a.chain)                     # one fused HIP kernel for the chain
        m.utils.write_image_device(a.output, y, a.quality)
        torch.cuda.synchronize()
        where = "GPU"
    else:
        y = m.ops.apply(m.utils.read_image(a.input), a.chain)
        m.utils.write_image(a.output, y, a.quality)
        where = "host"
    print(f"{a.input} -> {a.output}: {a.chain} on {where} in {(time.perf_counter() - t0) * 1e3:.1f} ms")


if __name__ == "__main__":
    main()
