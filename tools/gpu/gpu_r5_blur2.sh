#!/bin/bash
# Round 5: blur:31:lsb with three pairs in flight (STRIPE_BLUR_VARIANT=4)
# against the default (two), alternating, 16K frame and N=8 stripe; the blur
# GPU tests under the variant; config 3 local ranks auto vs 21 (repeat) with
# the engine's depth log line.
#   bash tools/gpu/gpu_r5_blur2.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-blur2}
mkdir -p $O
export TMPDIR=/tmp
STRIPE_BLUR_VARIANT=4 timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests_v4.txt 2>&1 || exit 2
for v in 0 4 0 4 0 4; do
  STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31:lsb|" --shape 16384x16384x3 --iters 30 >> $O/v${v}_16k.txt 2>&1 || exit 3
  STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31:lsb|" --shape 16384x2048x3 --iters 60 >> $O/v${v}_stripe.txt 2>&1 || exit 3
done
STRIPE_LOG=debug timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 5 --warmup 1 --scope resident --backend local 2>&1 | grep -i "depth" > $O/cfg3_depthlog.txt
for d in 0 21 0 21 0 21; do
  echo "depth $d" >> $O/cfg3_auto.txt
  timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 50 --warmup 10 --scope resident --backend local --halo-depth $d 2>&1 | grep -v amdgpu.ids >> $O/cfg3_auto.txt || exit 5
done
echo done
