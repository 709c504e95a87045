#!/bin/bash
# shared-window blur as the RGB default: full GPU suite, then kbench
set -o pipefail
O=gpurun_out/r3blurnw2; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1" --shape $2 --iters 20 --warmup 3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x3 16384x2048x3 4096x4096x3 16383x4099x3; do
  for mode in blur:31 blur:31:lsb blur:9; do
    echo "$shape $mode $(kb "$mode|" $shape) $(kb "$mode|" $shape) $(kb "$mode|" $shape)" || exit 1
  done
done
