#!/bin/bash
# conv correctness on the current tree, then current vs build_alt2 timing (same box).
set -o pipefail
mkdir -p gpurun_out/conv
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "general_conv or conv_asym or sep_matches" > gpurun_out/conv/pytest.log 2>&1 || { tail -30 gpurun_out/conv/pytest.log; exit 1; }
tail -1 gpurun_out/conv/pytest.log
C31=$(cat tools/conv31_chain.txt)
C9="conv:9:$(python -c "print(';'.join(['0.0123456']*81))")"
for rep in 1 2; do for d in . build_alt2; do
  for shape in 16384x2048x3 16384x4096x1; do
    timeout -k 10 120 python $d/tools/kbench.py --shape $shape --chains "$C31|$C9" --iters 10 --warmup 2 2>&1 | grep -o '"chain": "conv:[0-9]*\|"shape": "[0-9x]*", "ms": [0-9.]*' | paste - - | sed "s#^#$d #"
  done
done; done
