#!/bin/bash
# HBM-streaming separable launches: occupancy cap by reserved LDS (STRIPE_NT_LDS)
# vs the previous build (ab_old: runtime hdpp branch, 96 VGPRs = 5 waves/SIMD).
set -o pipefail
O=gpurun_out/nt_lds
mkdir -p $O
for rep in 1 2; do
for v in old 0 28672 36864 46080; do
  K=tools/kbench.py; [ $v = old ] && K=ab_old/tools/kbench.py
  L=$v; [ $v = old ] && L=0
  STRIPE_NT_LDS=$L STRIPE_SEP_DPP=1 timeout -k 10 120 python $K --shape 16384x16384x3 --chains "gaussian5|sobel" --iters 30 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$v /" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
