#!/bin/bash
# blur:31:lsb 16K RGB: XCD remap and band height (32-row groups per task)
set -o pipefail
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "blur:31:lsb|" --shape $1 --iters 20 --warmup 3 --bands $2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x3 16384x2048x3; do
  for x in 0 8; do
    for b in 0 128 256 512 1024; do
      echo "$shape xcd=$x band=$b $(STRIPE_XCD=$x kb $shape $b) $(STRIPE_XCD=$x kb $shape $b)" || exit 1
    done
  done
done
