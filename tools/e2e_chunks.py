import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from mpi_cuda_imagemanipulation_amd._native import C
from mpi_cuda_imagemanipulation_amd.models import Pipeline
W, H, Cc = 16384, 16384, 3
cfg = Pipeline("gaussian5").config(W, H, Cc, "device", device=0)
e = C.Engine(cfg)
e.alloc_host_io()
e.host_input()[...] = C.synth_rows(1, W, Cc, 0, H)
for ch in (4, 8, 16, 32, 64):
    e.run_e2e(ch); e.synchronize()
    t0 = time.perf_counter()
    for _ in range(3): e.run_e2e(ch)
    e.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 3
    print(f"chunks={ch:3d} e2e {ms:.2f} ms  {W*H/ms/1e3:.0f} Mpx/s", flush=True)
