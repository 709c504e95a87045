#!/bin/bash
# RGB blur:31:lsb strip width / prefetch depth A/B (STRIPE_BLUR_XCFG)
set -o pipefail
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1" --shape $2 --iters 20 --warmup 3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x3 16384x2048x3 4096x4096x3; do
  echo "$shape exact $(kb 'blur:31|' $shape)  lsb $(kb 'blur:31:lsb|' $shape) $(kb 'blur:31:lsb|' $shape)" || exit 1
  for x in 0 1 2 3; do
    echo "  xcfg=$x $(STRIPE_BLUR_XCFG=$x kb 'blur:31:lsb|' $shape) $(STRIPE_BLUR_XCFG=$x kb 'blur:31:lsb|' $shape) $(STRIPE_BLUR_XCFG=$x kb 'blur:31:lsb|' $shape)" || exit 1
  done
done
