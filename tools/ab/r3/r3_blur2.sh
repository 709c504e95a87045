#!/bin/bash
set -o pipefail
O=gpurun_out/r3blur2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_oracle_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "blur or sep or sepconv" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt
[ $rc -ne 0 ] && exit $rc
for sh in 16384x16384x3 16384x2048x3 16384x16384x1 4096x4096x3; do
  timeout -k 10 300 python3 tools/kbench.py --chains 'blur:31' --shape $sh --iters 30 >> $O/kb.jsonl 2>/dev/null || exit 1
done
cat $O/kb.jsonl
