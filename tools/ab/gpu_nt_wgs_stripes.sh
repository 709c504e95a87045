#!/bin/bash
# nt occupancy cap on the N=2 / N=4 per-rank stripes of the 16K RGB frame (nt launches)
set -o pipefail
O=gpurun_out/nt_wgs_stripes
mkdir -p $O
for rep in 1 2; do
for w in 0 2 3 4; do
  for sh in 16384x8192x3 16384x4096x3; do
    STRIPE_NT_WGS=$w timeout -k 10 150 python tools/kbench.py --shape $sh --chains "gaussian5|sobel" --iters 30 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
  done
done; done
echo done
