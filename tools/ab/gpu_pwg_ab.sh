#!/bin/bash
set -o pipefail
O=gpurun_out/pwg
mkdir -p $O
for rep in 1 2; do for w in 0 2 3 4 6; do
  STRIPE_PWG_WGS=$w timeout -k 10 150 python tools/kbench.py --shape 16384x16384x3 --chains "gray:ref|gray:bt601|gray:ref,contrast:3.5" --iters 30 --warmup 5 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
  STRIPE_PWG_WGS=$w timeout -k 10 150 python tools/kbench.py --shape 16384x16384x1 --chains "expand" --iters 30 --warmup 5 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
done; done
echo done
