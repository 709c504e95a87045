#!/bin/bash
# loop-entry masked stores (precise vmcnt in the row steps): current tree vs build_alt2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/entry_pytest.log 2>&1 || { tail -30 gpurun_out/entry_pytest.log; exit 1; }
tail -1 gpurun_out/entry_pytest.log
for rep in 1 2; do
  for d in . build_alt2; do
    timeout -k 10 200 python $d/tools/kbench.py --chains "gaussian5|sobel|emboss3|gray:ref,contrast:3.5,emboss3@skip,expand" --shape 16384x16384x3 --iters 40 --warmup 5 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "gaussian5|sobel|emboss3" --shape 16384x2048x3 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "sobel|gaussian5" --shape 8192x8192x1 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "gaussian5|conv:3:1;2;1;2;4;2;1;2;1" --shape 4096x4096x3 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#$d #" || exit 1
  done
done
