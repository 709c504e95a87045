#!/bin/bash
# Correctness of the current tree's stencil kernels, then an A/B of the current
# tree vs build_alt2 (same tools) on the headline shape and one N=8 stripe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab2_pytest.log 2>&1 || { tail -30 gpurun_out/ab2_pytest.log; exit 1; }
tail -1 gpurun_out/ab2_pytest.log
CH=${CH:-"gaussian5;sobel;gaussian3"}
for rep in 1 2; do
  for d in . build_alt2; do
    for shape in 16384x16384x3 16384x2048x3; do
      timeout -k 10 300 python $d/tools/kbench.py --chains "$CH" --shape $shape --iters 40 2>&1 | grep -v amdgpu | sed "s#^#$d #" || exit 1
    done
  done
done
