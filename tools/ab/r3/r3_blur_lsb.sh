#!/bin/bash
# blur:K:lsb (centred single-f16 MFMA blur): oracle tests, then exact vs lsb and
# the LSB configuration A/B (STRIPE_BLUR_XCFG) on 16K RGB / 16K gray / N=8 stripe
set -o pipefail
O=gpurun_out/r3blurlsb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_kernels.py -m gpu -x -q -s -k "blur or sep" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; grep "off by one" $O/tests.txt | head -30
[ $rc -ne 0 ] && exit $rc
kb() { timeout -k 10 120 python3 tools/kbench.py --chains "$1" --shape $2 --iters 20 --warmup 3 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x3 16384x2048x3 16384x16384x1; do
  echo "$shape exact $(kb 'blur:31|' $shape) $(kb 'blur:31|' $shape)  lsb $(kb 'blur:31:lsb|' $shape) $(kb 'blur:31:lsb|' $shape)" || exit 1
  for x in 0 1 2 3; do
    echo "  xcfg=$x $(STRIPE_BLUR_XCFG=$x kb 'blur:31:lsb|' $shape) $(STRIPE_BLUR_XCFG=$x kb 'blur:31:lsb|' $shape)" || exit 1
  done
done
