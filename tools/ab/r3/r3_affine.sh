#!/bin/bash
# gray:ref post map in packed i16: tests, then the reference pipeline kernels (autotuned)
set -o pipefail
O=gpurun_out/r3affine; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "gray or ref or skip or chain or pipeline or expand" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python3 tools/kbench.py --shape 16384x16384x3 --chains "gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|gray:ref,contrast:3.5,emboss3|" --bands=-1 --iters 30 2>/dev/null || exit 1
done
