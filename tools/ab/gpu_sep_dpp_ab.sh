#!/bin/bash
# Separable stencils: neighbour vertical sums by DPP wave shifts (STRIPE_SEP_DPP=1)
# vs the LDS row (0): stencil GPU tests under DPP, then timings.
set -o pipefail
O=gpurun_out/sep_dpp
mkdir -p $O
STRIPE_SEP_DPP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_dpp.log 2>&1 || { tail -30 $O/pytest_dpp.log; exit 1; }
tail -1 $O/pytest_dpp.log
for rep in 1 2; do
for d in 0 1; do
  STRIPE_SEP_DPP=$d timeout -k 10 120 python tools/kbench.py --shape 16384x16384x3 --chains "gaussian5|gaussian3|gaussian7|sobel|box5" --iters 30 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/dpp=$d /" >> $O/ab.txt || exit 1
  STRIPE_SEP_DPP=$d timeout -k 10 120 python tools/kbench.py --shape 16384x2048x3 --chains "gaussian5|gaussian3|gaussian7|sobel|box5" --iters 50 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/dpp=$d /" >> $O/ab.txt || exit 1
  STRIPE_SEP_DPP=$d timeout -k 10 120 python tools/kbench.py --shape 8192x2048x1 --chains "sobel|gaussian5" --iters 50 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/dpp=$d /" >> $O/ab.txt || exit 1
  STRIPE_SEP_DPP=$d timeout -k 10 120 python tools/kbench.py --shape 4096x4096x3 --chains "gaussian5" --iters 100 --warmup 10 --bands -1 2>&1 | grep chain | sed "s/^/dpp=$d /" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
