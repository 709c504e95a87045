#!/bin/bash
# Round 5: blur:31 with the next pair staged inside the current step's MFMAs
# (EARLY, the default) against round 4's staging between barrier and MFMAs
# (STRIPE_BLUR_VARIANT=3), exact and :lsb, 16K frame and N=8 stripe,
# alternating; the blur / conv GPU tests; config 3 on 4 `local` ranks at halo
# depth 1 / 8 (spinning local hub).
#   bash tools/gpu/gpu_r5_blur.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-blur}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
for v in 0 3 0 3; do
  STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/v${v}_16k.txt 2>&1 || exit 3
  STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/v${v}_stripe.txt 2>&1 || exit 3
done
for d in 1 8 1 8; do
  timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 48 --warmup 8 --scope resident --backend local --halo-depth $d >> $O/cfg3_local_depth.txt 2>&1 || exit 4
done
echo done
