#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
: > gpurun_out/sweep.log
for shape in 16384x16384x3 16384x2048x3 8192x8192x1; do
timeout -k 10 300 python tools/kbench.py --shape $shape --chains "${CH:-gaussian5;gray:ref,contrast:3.5,emboss3;sobel}" --bands ${BANDS:-8,12,16,24} --iters 30 >> gpurun_out/sweep.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/sweep.log | cut -c1-120
