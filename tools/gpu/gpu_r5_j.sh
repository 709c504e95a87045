#!/bin/bash
# Round 5: blur lsb on a cache-resident stripe with late staging (default now)
# vs early (variant 0 forced through STRIPE_BLUR_VARIANT is the early kernel
# only on streaming passes, so the stripe numbers show the new default);
# conv:31:lsb at 4 m-tiles (STRIPE_CONV_MT=4) vs 3; conv / blur GPU tests.
#   bash tools/gpu/gpu_r5_j.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
STRIPE_CONV_MT=4 timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py -m gpu -q -k "conv" --timeout 120 --timeout-method thread > $O/tests_mt4.txt 2>&1 || exit 2
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --chains "blur:31:lsb|blur:31" --shape 16384x2048x3 --iters 60 >> $O/blur_stripe.txt 2>&1 || exit 3
  timeout -k 10 120 python tools/kbench.py --chains "blur:31:lsb|blur:31" --shape 16384x16384x3 --iters 20 >> $O/blur_16k.txt 2>&1 || exit 3
  for mt in 3 4; do
    STRIPE_CONV_MT=$mt timeout -k 10 200 python tools/kbench.py --chains "$C31:lsb|" --shape 16384x16384x3 --iters 6 >> $O/conv_lsb_16k_mt$mt.txt 2>&1 || exit 4
    STRIPE_CONV_MT=$mt timeout -k 10 200 python tools/kbench.py --chains "$C31:lsb|" --shape 16384x2048x3 --iters 20 >> $O/conv_lsb_stripe_mt$mt.txt 2>&1 || exit 4
  done
done
echo done
