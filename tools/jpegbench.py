#!/usr/bin/env python3
"""JPEG I/O throughput on one MI355X: host codec (csrc/core/jpeg.cpp), the
split codec with pixel stages on the GPU (csrc/hip/jpeg_dev.hip), and Pillow
(libjpeg-turbo) as the library baseline.  Synthetic smooth RGB frame; with
Pillow also the same frame saved progressive by libjpeg (decode only: the
native encoder writes baseline).  Prints one JSON line.  python tools/jpegbench.py [--size 8192] [--quality 90]"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from mpi_cuda_imagemanipulation_amd._native import C

    n = a.size
    y, x = np.mgrid[0:n, 0:n].astype(np.float32)
    img = np.stack([128 + 100 * np.sin(x / 37 + k) * np.cos(y / 53 - k) for k in range(3)], -1).astype(np.uint8)
    del x, y
    data = C.encode_jpeg(img, a.quality, True, -1)

    def best(fn):
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(min(ts) * 1e3, 1)

    dev = torch.from_numpy(img).cuda()
    out = torch.empty_like(dev)
    stream = torch.cuda.current_stream().cuda_stream

    def dev_decode():
        jc = C.jpeg_entropy_decode(data)
        jc.to_device(out.data_ptr(), n * 3, stream)
        torch.cuda.synchronize()

    def dev_encode():
        C.jpeg_encode_device(dev.data_ptr(), n * 3, n, n, 3, a.quality, True, -1, stream)

    rec = {"size": f"{n}x{n}x3", "quality": a.quality, "jpeg_bytes": len(data),
           "decode_ms": {"host": best(lambda: C.decode_jpeg(data)),
                         "entropy_only": best(lambda: C.jpeg_entropy_decode(data)),
                         "entropy_host_pixels_gpu": best(dev_decode)},
           "encode_ms": {"host": best(lambda: C.encode_jpeg(img, a.quality, True, -1)),
                         "pixels_gpu_entropy_host": best(dev_encode)}}
    try:
        from PIL import Image

        rec["decode_ms"]["pillow"] = best(lambda: np.asarray(Image.open(io.BytesIO(data)).convert("RGB")))

        def pil_enc():
            b = io.BytesIO()
            Image.fromarray(img).save(b, "JPEG", quality=a.quality)

        rec["encode_ms"]["pillow"] = best(pil_enc)
    except ImportError:
        pass
    try:
        import tempfile

        from PIL import Image

        with tempfile.TemporaryDirectory() as td:  # (Pillow's progressive writer wants a real file)
            f = os.path.join(td, "p.jpg")
            Image.fromarray(img).save(f, "JPEG", quality=a.quality, progressive=True)
            prog = open(f, "rb").read()
            # libjpeg's own sequential save: no restart markers, so the native
            # decoder's speculative parallel entropy stage is what runs
            Image.fromarray(img).save(f, "JPEG", quality=a.quality)
            lib = open(f, "rb").read()

        def dev_decode_prog():
            jc = C.jpeg_entropy_decode(prog)
            jc.to_device(out.data_ptr(), n * 3, stream)
            torch.cuda.synchronize()

        def dev_decode_lib():
            jc = C.jpeg_entropy_decode(lib)
            jc.to_device(out.data_ptr(), n * 3, stream)
            torch.cuda.synchronize()

        rec["libjpeg_sequential"] = {
            "jpeg_bytes": len(lib),
            "decode_ms": {"host": best(lambda: C.decode_jpeg(lib)),
                          "entropy_only": best(lambda: C.jpeg_entropy_decode(lib)),
                          "entropy_host_pixels_gpu": best(dev_decode_lib),
                          "pillow": best(lambda: np.asarray(Image.open(io.BytesIO(lib)).convert("RGB")))},
            "host_vs_pillow_max_diff": int(np.abs(C.decode_jpeg(lib).astype(int)
                                                  - np.asarray(Image.open(io.BytesIO(lib)).convert("RGB")).astype(int)).max())}
        ref = np.asarray(Image.open(io.BytesIO(prog)).convert("RGB"))
        rec["progressive"] = {
            "jpeg_bytes": len(prog),
            "decode_ms": {"host": best(lambda: C.decode_jpeg(prog)),
                          "entropy_only": best(lambda: C.jpeg_entropy_decode(prog)),
                          "entropy_host_pixels_gpu": best(dev_decode_prog),
                          "pillow": best(lambda: np.asarray(Image.open(io.BytesIO(prog)).convert("RGB")))},
            "host_vs_pillow_max_diff": int(np.abs(C.decode_jpeg(prog).astype(int) - ref.astype(int)).max())}
    except ImportError:
        pass
    dev_decode()
    rec["gpu_vs_host_max_diff"] = int(np.abs(out.cpu().numpy().astype(int) - C.decode_jpeg(data).astype(int)).max())
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
