#!/bin/bash
# sobel_l2 f32 rounding: exactness tests + timing; gray-prologue chain on the stripe: bands x XCD remap
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "sobel or chains or skip" > gpurun_out/l2_pytest.log 2>&1 || { tail -30 gpurun_out/l2_pytest.log; exit 1; }
tail -1 gpurun_out/l2_pytest.log
timeout -k 10 200 python tools/kbench.py --chains "sobel_l2|sobel" --shape 16384x16384x3 --iters 20 --warmup 3 2>&1 | grep chain || exit 1
timeout -k 10 200 python tools/kbench.py --chains "sobel_l2" --shape 16384x2048x3 --iters 100 --warmup 10 2>&1 | grep chain || exit 1
for x in def 0; do
  if [ $x = def ]; then unset STRIPE_XCD; else export STRIPE_XCD=0; fi
  timeout -k 10 200 python tools/kbench.py --chains "gray:ref,contrast:3.5,emboss3|gray,gaussian5" --shape 16384x2048x3 --bands 4,8,12,16 --iters 100 --warmup 10 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
done
