#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_r3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_kern_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r3_kern_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/kbench.py --shape 16384x16384x3 --iters 50 --bands=-1 \
  --chains 'gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|gray:ref,contrast:3.5,emboss3|gray,sobel|gaussian5' 2>/dev/null
