#!/bin/bash
# HBM-streaming stencil launches: resident workgroups per CU capped by an LDS
# reservation (STRIPE_NT_WGS = 0 no cap, 1..4), full 16K frames, band autotune on.
set -o pipefail
O=gpurun_out/nt_wgs
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "stencil or expand" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for w in 0 1 2 3 4; do
  STRIPE_NT_WGS=$w timeout -k 10 150 python tools/kbench.py --shape 16384x16384x3 --chains "gaussian5|sobel|gaussian3|emboss3|gray:ref,contrast:3.5,emboss3|gray:ref,contrast:3.5,emboss3@skip,expand" --iters 20 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
  STRIPE_NT_WGS=$w timeout -k 10 150 python tools/kbench.py --shape 16384x16384x1 --chains "gaussian5|sobel" --iters 20 --warmup 5 --bands -1 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
done; done
echo done
