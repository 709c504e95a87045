#!/bin/bash
# blur epilogue deferred one tile (new) vs the previous kernel (ab_old/), alternating, same box
set -o pipefail
O=gpurun_out/r4/blur_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_kernels.py tests/test_gpu_r3.py tests/test_gpu_large.py tests/test_gpu_engine.py -m gpu -k "blur or conv or sep" -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in old new; do
    K=tools/kbench.py; [ $v = old ] && K=ab_old/tools/kbench.py
    timeout -k 10 120 python $K --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 > $O/${v}_16k_$rep.txt 2>&1 || exit 1
    timeout -k 10 120 python $K --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 > $O/${v}_stripe_$rep.txt 2>&1 || exit 1
  done
done
echo done
