#!/bin/bash
# GPU tests + kernel bench + rocprofv3 kernel stats for the headline chain.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest gpu rc=$rc"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python tools/kbench.py --chains "gaussian5;gray:ref,contrast:3.5,emboss3;sobel;gaussian3;gaussian7;invert;gray" --iters 40 > gpurun_out/kbench.log 2>&1; rc=$?
cat gpurun_out/kbench.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python tools/kbench.py --chains gaussian5 --iters 20 > gpurun_out/prof.log 2>&1; rc=$?
find gpurun_out/prof -name "*stats*" | head
exit $rc
