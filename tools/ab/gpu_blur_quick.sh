#!/bin/bash
# Separable MFMA blur: correctness subset + timing (one N=8 stripe, full 16K RGB frame, 8K gray).
set -o pipefail
mkdir -p gpurun_out/blur
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "blur or sepconv or sep_matches" > gpurun_out/blur/pytest.log 2>&1 || { tail -30 gpurun_out/blur/pytest.log; exit 1; }
tail -1 gpurun_out/blur/pytest.log
for shape in 16384x2048x3 16384x16384x3 8192x8192x1; do
  timeout -k 10 120 python tools/kbench.py --shape $shape --chains "blur:31" --iters 20 --warmup 3 2>&1 | grep -o '"shape": "[0-9x]*", "ms": [0-9.]*'
done
