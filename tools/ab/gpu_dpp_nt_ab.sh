#!/bin/bash
# 3-way A/B: runtime hdpp branch (ab_old, STRIPE_SEP_DPP=1) / static DPP (ab_new) /
# static DPP + per-row sched barrier in the nt instance (current build).
set -o pipefail
O=gpurun_out/dpp_nt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "stencil or sep or expand" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
for v in old new cur; do
  K=tools/kbench.py; [ $v = old ] && K=ab_old/tools/kbench.py; [ $v = new ] && K=ab_new/tools/kbench.py
  STRIPE_SEP_DPP=1 timeout -k 10 120 python $K --shape 16384x16384x3 --chains "gaussian5|sobel|box5" --iters 30 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$v /" >> $O/ab.txt || exit 1
  STRIPE_SEP_DPP=1 timeout -k 10 120 python $K --shape 16384x2048x3 --chains "gaussian5" --iters 50 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$v /" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
