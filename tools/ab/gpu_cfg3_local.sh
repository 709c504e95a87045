#!/bin/bash
# config 3 with 4 local ranks on one GPU: XCD remap default vs off, two reps
set -o pipefail
for rep in 1 2; do
  for x in def 0; do
    if [ $x = def ]; then unset STRIPE_XCD; else export STRIPE_XCD=0; fi
    timeout -k 10 200 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 50 --warmup 10 --scope resident --backend local 2>&1 | grep metric | sed "s#^#xcd=$x #" || exit 1
    timeout -k 10 200 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 1 --iters 50 --warmup 10 --scope resident --backend local 2>&1 | grep metric | sed "s#^#xcd=$x #" || exit 1
  done
done
