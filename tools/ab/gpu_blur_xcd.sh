#!/bin/bash
# blur:31 (separable MFMA) with / without the XCD-contiguous remap
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for x in 0 8; do
    STRIPE_XCD=$x timeout -k 10 200 python tools/kbench.py --chains "blur:31" --shape 16384x2048x3 --iters 50 --warmup 5 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
    STRIPE_XCD=$x timeout -k 10 200 python tools/kbench.py --chains "blur:31" --shape 16384x16384x3 --iters 10 --warmup 3 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
  done
done
