#!/bin/bash
# 8-wave shared-window blur: band height (rows per workgroup task) x XCD remap
set -o pipefail
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1|" --shape $2 --iters 20 --warmup 3 --bands $3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for mode in blur:31 blur:31:lsb; do
  for shape in 16384x16384x3 16384x2048x3; do
    for x in 0 8; do
      for b in 0 256 512 1024 2048; do
        echo "$mode $shape xcd=$x band=$b $(STRIPE_XCD=$x kb $mode $shape $b) $(STRIPE_XCD=$x kb $mode $shape $b)" || exit 1
      done
    done
  done
done
