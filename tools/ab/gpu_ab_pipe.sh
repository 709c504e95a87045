#!/bin/bash
# k_sep software-pipelined rows (vertical of y+1 beside horizontal of y): tests + A/B vs build_alt2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_large.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pipe_pytest.log 2>&1 || { tail -30 gpurun_out/pipe_pytest.log; exit 1; }
tail -1 gpurun_out/pipe_pytest.log
for rep in 1 2; do
  for d in . build_alt2; do
    timeout -k 10 200 python $d/tools/kbench.py --chains "gaussian5|sobel|gaussian3|gray,gaussian5,expand" --shape 16384x16384x3 --iters 30 --warmup 5 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "gaussian5|sobel|gaussian3" --shape 16384x2048x3 --bands 8,12 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "sobel|gaussian5" --shape 8192x8192x1 --iters 200 --warmup 20 2>&1 | grep chain | sed "s#^#$d #" || exit 1
  done
done
