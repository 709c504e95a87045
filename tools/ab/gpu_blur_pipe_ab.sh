#!/bin/bash
# Separable MFMA blur: software-pipelined column loop (default) vs the batched
# loop (STRIPE_BLUR_PIPE=0): correctness subset, then timings on three shapes.
set -o pipefail
O=gpurun_out/blur_pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "blur or sepconv or sep" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for pipe in 0 1; do
for shape in 16384x2048x3 16384x16384x3 8192x8192x1; do
  STRIPE_BLUR_PIPE=$pipe timeout -k 10 120 python tools/kbench.py --shape $shape --chains "blur:31|blur:15" --iters 20 --warmup 3 2>&1 | grep chain | sed "s/^/pipe=$pipe /" >> $O/ab.txt || exit 1
done; done; done
cat $O/ab.txt
