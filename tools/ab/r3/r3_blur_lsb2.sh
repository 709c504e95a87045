#!/bin/bash
# blur:31 strip width / prefetch depth A/B (STRIPE_BLUR_XCFG), lsb and exact modes
set -o pipefail
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1" --shape $2 --iters 20 --warmup 3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x3 16384x2048x3; do
  for mode in blur:31:lsb blur:31; do
    echo "$shape $mode default $(kb "$mode|" $shape) $(kb "$mode|" $shape)" || exit 1
    for x in 0 1 2 3; do
      echo "  xcfg=$x $(STRIPE_BLUR_XCFG=$x kb "$mode|" $shape) $(STRIPE_BLUR_XCFG=$x kb "$mode|" $shape)" || exit 1
    done
  done
done
