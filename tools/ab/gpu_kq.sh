#!/bin/bash
# Quick kernel check: GPU kernel tests, then kbench on the config shapes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_k.log; exit 1; }
for s in 16384x2048x3 16384x16384x3 4096x4096x3 8192x8192x1; do
  timeout -k 10 120 python tools/kbench.py --chains "${CH:-gaussian5;gaussian3;sobel}" --shape $s --iters 100 2>&1 | grep -v amdgpu | cut -c1-100 || exit 1
done
