#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench1.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/bench1.log | tail -3
exit $rc
