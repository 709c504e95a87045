#!/bin/bash
# Streaming flat pointwise passes (invert, brightness) on the 16K RGB frame:
# resident workgroups per CU capped by an LDS reservation (STRIPE_PW_WGS).
set -o pipefail
O=gpurun_out/pw_wgs
mkdir -p $O
for rep in 1 2; do
for w in 0 1 2 3 4 6 8; do
  STRIPE_PW_WGS=$w timeout -k 10 150 python tools/kbench.py --shape 16384x16384x3 --chains "invert|brightness:20" --iters 30 --warmup 5 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
done; done
echo done
