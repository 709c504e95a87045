#!/bin/bash
# Quick iteration: GPU tests (kernels only) + band sweep on the headline kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python tools/kbench.py --chains "${CH:-gaussian5}" --bands ${BANDS:-0,16,32,64} --iters 30 > gpurun_out/bands.log 2>&1; rc=$?
cat gpurun_out/bands.log | grep -v amdgpu.ids
exit $rc
