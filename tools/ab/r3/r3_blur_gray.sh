#!/bin/bash
# gray blur on 8-wave shared windows (STRIPE_BLUR_NW = 0..3): correctness, kbench
set -o pipefail
O=gpurun_out/r3blurgray; mkdir -p $O
for x in 0 1 2 3; do
  STRIPE_BLUR_NW=$x timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_kernels.py tests/test_n8.py -m gpu -x -q -k "blur or sep" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_$x.txt 2>&1 || { echo "tests failed nw=$x"; tail -30 $O/tests_$x.txt; exit 1; }
  echo "nw=$x $(tail -1 $O/tests_$x.txt)"
done
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1|" --shape $2 --iters 20 --warmup 3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x1 16384x2048x1; do
  echo "$shape base $(kb blur:31 $shape) $(kb blur:31 $shape)" || exit 1
  for x in 0 1 2 3; do echo "  nw=$x $(STRIPE_BLUR_NW=$x kb blur:31 $shape) $(STRIPE_BLUR_NW=$x kb blur:31 $shape)" || exit 1; done
done
