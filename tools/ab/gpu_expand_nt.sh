#!/bin/bash
# nt vs default store policy for the fused-expand reference chain (16K RGB)
set -o pipefail
mkdir -p gpurun_out
for nt in 0 1; do
  STRIPE_NT=$nt timeout -k 10 200 python -u tools/kbench.py --shape 16384x16384x3 --iters 30 \
    --chains "gray:ref,contrast:3.5,emboss3@skip,expand|gray,gaussian5,expand" > gpurun_out/expand_nt$nt.log 2>&1 \
    || { tail -20 gpurun_out/expand_nt$nt.log; exit 1; }
  echo "STRIPE_NT=$nt"; grep chain gpurun_out/expand_nt$nt.log
done
