#!/bin/bash
# nt-store threshold sweep: default policy vs nt stores per working-set size.
set -o pipefail
mkdir -p gpurun_out
for shape in 16384x16384x3 16384x4096x3 16384x2048x3 8192x8192x1 4096x4096x3; do
  for nt in 0 1 auto; do
    if [ $nt = auto ]; then unset STRIPE_NT; else export STRIPE_NT=$nt; fi
    timeout -k 10 120 python tools/kbench.py --chains "gaussian5;sobel;gray:ref,contrast:3.5,emboss3" --shape $shape --iters 40 2>&1 | grep -v amdgpu | sed "s#^#nt=$nt #" || exit 1
  done
done
