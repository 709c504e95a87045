#!/bin/bash
# Round 5: conv:31 with single-buffered A fragments (STRIPE_CONV_A1=1) at 3 / 4
# / 5 m-tiles (STRIPE_CONV_MT) against the defaults, exact and :lsb, 16K frame
# and N=8 stripe, alternating; conv GPU tests under the variants.
#   bash tools/gpu/gpu_r5_k.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-k}
mkdir -p $O
export TMPDIR=/tmp
for mt in 4 5; do
  STRIPE_CONV_A1=1 STRIPE_CONV_MT=$mt timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py -m gpu -q -k conv --timeout 120 --timeout-method thread > $O/tests_a1_mt$mt.txt 2>&1 || exit 2
done
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
for r in 1 2; do
  for v in d a3 a4 a5; do
    case $v in d) E="";; a3) E="STRIPE_CONV_A1=1 STRIPE_CONV_MT=3";; a4) E="STRIPE_CONV_A1=1 STRIPE_CONV_MT=4";; a5) E="STRIPE_CONV_A1=1 STRIPE_CONV_MT=5";; esac
    env $E timeout -k 10 200 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x16384x3 --iters 6 >> $O/conv_16k_$v.txt 2>&1 || exit 3
    env $E timeout -k 10 200 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x2048x3 --iters 20 >> $O/conv_stripe_$v.txt 2>&1 || exit 3
  done
done
echo done
