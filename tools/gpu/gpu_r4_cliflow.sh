#!/bin/bash
# The reference program's flow end to end through the native CLI on one
# MI355X: read (PPM / JPEG) -> scatter -> filter -> gather -> write, 16384^2 RGB.
set -o pipefail
O=gpurun_out/r4/cliflow
mkdir -p $O
T=$(mktemp -d)
S=bin/stripe
# a smooth photo-like frame (random bytes would make a worst-case JPEG)
timeout -k 10 300 python3 -c "
import sys, numpy as np
sys.path.insert(0, '.')
from mpi_cuda_imagemanipulation_amd._native import C
n = 16384
y = np.arange(n, dtype=np.float32)[:, None]
img = np.empty((n, n, 3), np.uint8)
for k in range(3):
    x = np.arange(n, dtype=np.float32)[None, :]
    img[..., k] = (128 + 100 * np.sin(x / 37 + k) * np.cos(y / 53 - k)).astype(np.uint8)
C.write_pnm('$T/in.ppm', img)
" > $O/gen.log 2>&1 || exit 1
timeout -k 10 120 $S convert --input $T/in.ppm --output $T/in.jpg --quality 90 >> $O/gen.log 2>&1 || exit 1
ls -la $T >> $O/gen.log
: > $O/flow.txt
for rep in 1 2; do
  echo "== ppm -> gaussian5 -> ppm (rep $rep)" >> $O/flow.txt
  timeout -k 10 120 $S run --input $T/in.ppm --output $T/out.ppm --chain gaussian5 >> $O/flow.txt 2>&1 || exit 1
  echo "== jpg -> ref-gpu -> jpg (rep $rep)" >> $O/flow.txt
  timeout -k 10 120 $S run --input $T/in.jpg --output $T/out.jpg --preset ref-gpu >> $O/flow.txt 2>&1 || exit 1
  echo "== ppm -> ref-gpu -> ppm (rep $rep)" >> $O/flow.txt
  timeout -k 10 120 $S run --input $T/in.ppm --output $T/out2.ppm --preset ref-gpu >> $O/flow.txt 2>&1 || exit 1
done
rm -rf $T
echo done
