#!/bin/bash
# three 32-row pairs in flight on the 8-wave windows (STRIPE_BLUR_NW=0): correctness, kbench
set -o pipefail
O=gpurun_out/r3blurpfd3; mkdir -p $O
STRIPE_BLUR_NW=0 timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_kernels.py tests/test_n8.py -m gpu -x -q -k "blur or sep" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1|" --shape $2 --iters 20 --warmup 3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for rep in 1 2; do for mode in blur:31 blur:31:lsb; do for shape in 16384x16384x3 16384x2048x3; do
  echo "$mode $shape base $(kb $mode $shape)  pfd3 $(STRIPE_BLUR_NW=0 kb $mode $shape)" || exit 1
done; done; done
