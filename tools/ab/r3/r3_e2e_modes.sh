#!/bin/bash
# e2e scope (pinned host -> H2D -> filter -> D2H -> pinned host), 16K RGB gaussian5, per transfer mode
set -o pipefail
for m in 2d staged zerocopy; do
  echo "mode=$m"; STRIPE_E2E_MODE=$m timeout -k 10 200 python3 -c "
import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from mpi_cuda_imagemanipulation_amd._native import C
from mpi_cuda_imagemanipulation_amd.models import Pipeline
W, H, Cc = 16384, 16384, 3
e = C.Engine(Pipeline('gaussian5').config(W, H, Cc, 'device', device=0))
e.alloc_host_io()
e.host_input()[...] = C.synth_rows(1, W, Cc, 0, H)
for ch in (8, 32):
    e.run_e2e(ch); e.synchronize()
    t0 = time.perf_counter()
    for _ in range(3): e.run_e2e(ch)
    e.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 3
    t = e.times.as_dict()
    print(f'  chunks={ch:3d} e2e {ms:.2f} ms  h2d {t[\"h2d\"]:.2f} d2h {t[\"d2h\"]:.2f} compute {t[\"compute\"]:.2f}', flush=True)
" || exit 1
done
python3 - <<'PY'
import torch, time
n = 805306368
h = torch.empty(n, dtype=torch.uint8, pin_memory=True); h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d = torch.empty(n, dtype=torch.uint8, device='cuda'); d2 = torch.empty(n, dtype=torch.uint8, device='cuda')
s1 = torch.cuda.Stream(); s2 = torch.cuda.Stream()
for _ in range(2):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize(); t3 = time.perf_counter()
    print(f"torch copy_ 805 MB: h2d {1e3*(t1-t0):.2f} ms, d2h {1e3*(t2-t1):.2f} ms, both at once {1e3*(t3-t2):.2f} ms")
PY
