#!/bin/bash
# Separable MFMA blur: band height (32-row groups per wave task) sweep vs the launch cost model (band 0).
set -o pipefail
O=gpurun_out/blur_band
mkdir -p $O
timeout -k 10 200 python tools/kbench.py --shape 16384x2048x3 --chains "blur:31" --iters 30 --warmup 3 --bands 0,128,192,224,256,320,352,384,416,512,704,1024 2>&1 | grep chain >> $O/sweep.txt || exit 1
timeout -k 10 200 python tools/kbench.py --shape 8192x2048x1 --chains "blur:31" --iters 30 --warmup 3 --bands 0,128,192,256,352,416,512,1024 2>&1 | grep chain >> $O/sweep.txt || exit 1
timeout -k 10 200 python tools/kbench.py --shape 16384x16384x3 --chains "blur:31" --iters 10 --warmup 2 --bands 0,256,384,512,1024 2>&1 | grep chain >> $O/sweep.txt || exit 1
cat $O/sweep.txt
