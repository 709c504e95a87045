#!/bin/bash
# N=8 stripe (16384x2048 RGB, MALL-resident) gaussian5: XCD remap x band height
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for x in 0 8; do
    STRIPE_XCD=$x timeout -k 10 200 python tools/kbench.py --chains "gaussian5" --shape 16384x2048x3 --bands 8,12,16,24 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
  done
done
