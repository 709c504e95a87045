#!/bin/bash
# Separable stencils: DPP window as a compile-time path (new build) vs the runtime
# hdpp branch of the previous build (ab_old/, STRIPE_SEP_DPP=1), same box.
set -o pipefail
O=gpurun_out/dpp_static
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "stencil or sep or expand" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for v in old new; do
  K=tools/kbench.py; [ $v = old ] && K=ab_old/tools/kbench.py
  for sh in "16384x16384x3 30" "16384x2048x3 50" "8192x2048x1 50" "16384x16384x1 30"; do
    set -- $sh
    STRIPE_SEP_DPP=1 timeout -k 10 120 python $K --shape $1 --chains "gaussian5|sobel|gaussian3|box5" --iters $2 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$v /" >> $O/ab.txt || exit 1
  done
done; done
cat $O/ab.txt
