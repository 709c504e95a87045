#!/bin/bash
# Filter sweep on one MI355X: every stencil / pointwise / conv family on the
# full 16K RGB frame (HBM-bound) and on one N=8 stripe (Infinity-Cache resident).
# Output: gpurun_out/sweep_r2/{full,stripe}.jsonl
set -o pipefail
O=gpurun_out/sweep_r2
mkdir -p $O
CH="invert|contrast:3.5|gray|gray,expand|gaussian3|gaussian5|gaussian7|box3|box5|emboss3|emboss5|sharpen|laplace|sobel|sobel_l2|gray:ref,contrast:3.5,emboss3|gray:ref,contrast:3.5,emboss3@skip,expand|gray,gaussian5,expand|conv:3:1;2;1;2;4;2;1;2;1|blur:9|blur:15|blur:31"
timeout -k 10 400 python tools/kbench.py --shape 16384x16384x3 --chains "$CH" --iters 20 --warmup 3 2>&1 | grep chain > $O/full.jsonl || exit 1
echo full done
timeout -k 10 400 python tools/kbench.py --shape 16384x2048x3 --chains "$CH" --iters 100 --warmup 10 2>&1 | grep chain > $O/stripe.jsonl || exit 1
echo stripe done
