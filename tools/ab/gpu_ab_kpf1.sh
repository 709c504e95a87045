#!/bin/bash
# 1-channel k_sep prefetch depth A/B: current tree vs build_alt2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "stencil_exact or chains" > gpurun_out/kpf_pytest.log 2>&1 || { tail -30 gpurun_out/kpf_pytest.log; exit 1; }
tail -1 gpurun_out/kpf_pytest.log
for rep in 1 2; do
  for d in . build_alt2; do
    for shape in 8192x8192x1 8192x2048x1 16384x16384x1; do
      timeout -k 10 200 python $d/tools/kbench.py --chains "sobel|gaussian5" --shape $shape --iters 100 --warmup 10 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    done
  done
done
