#!/usr/bin/env python3
"""run_e2e chunk-count sweep on one GPU (pinned H2D -> filter -> D2H, 16384^2 RGB gaussian5)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from mpi_cuda_imagemanipulation_amd._native import C  # noqa: E402
from mpi_cuda_imagemanipulation_amd.models import Pipeline  # noqa: E402

W = H = 16384
cfg = Pipeline("gaussian5").config(W, H, 3, "device", device=0)
e = C.Engine(cfg)
e.alloc_host_io()
e.host_input()[...] = C.synth_rows(1, W, 3, 0, H)
for chunks in (4, 8, 16, 32, 64):
    e.run_e2e(chunks)
    e.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        e.run_e2e(chunks)
    e.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 4
    print(json.dumps({"chunks": chunks, "ms": round(ms, 3), "mpx_s": round(W * H / ms / 1e3, 1)}), flush=True)
