#!/bin/bash
# XCD remap default (on for cache-resident passes) vs forced off, several shapes
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/xcd_pytest.log 2>&1 || { tail -30 gpurun_out/xcd_pytest.log; exit 1; }
tail -1 gpurun_out/xcd_pytest.log
for rep in 1 2; do
  for x in def 0; do
    if [ $x = def ]; then unset STRIPE_XCD; else export STRIPE_XCD=0; fi
    timeout -k 10 200 python tools/kbench.py --chains "gaussian5|sobel|emboss3|gray:ref,contrast:3.5,emboss3@skip,expand" --shape 16384x2048x3 --bands 8,12,16 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
    timeout -k 10 200 python tools/kbench.py --chains "gaussian5" --shape 4096x4096x3 --bands 8,12,16 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
    timeout -k 10 200 python tools/kbench.py --chains "sobel" --shape 8192x8192x1 --bands 8,12,16 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#xcd=$x #" || exit 1
  done
done
unset STRIPE_XCD
timeout -k 10 300 python bench.py > gpurun_out/xcd_bench.log 2>&1 && grep metric gpurun_out/xcd_bench.log | cut -c1-300
