#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep.log
for shape in 16384x16384x3 16384x2048x3; do
  timeout -k 10 300 python tools/kbench.py --shape $shape --chains "gaussian5;gray:ref,contrast:3.5,emboss3;invert;gaussian7" --bands 4,8,12,16,24,32 --iters 30 >> gpurun_out/sweep.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/sweep.log
