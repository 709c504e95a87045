#!/bin/bash
# A/B of two builds on the same box: current tree vs build_alt/ (same tools).
set -o pipefail
mkdir -p gpurun_out
CH=${CH:-"gaussian5;gaussian7;sobel;box3"}
SHAPE=${SHAPE:-16384x16384x3}
for rep in 1 2; do
  for v in cur alt; do
    d=.; [ $v = alt ] && d=build_alt
    timeout -k 10 300 python $d/tools/kbench.py --chains "$CH" --shape $SHAPE --iters 30 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done
