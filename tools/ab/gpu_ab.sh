#!/bin/bash
# A/B of builds on the same box: current tree vs build_alt*/ trees (same tools).
#   ALTS="build_alt1 build_alt2" CH="gaussian5;sobel" SHAPE=16384x16384x3 bash tools/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
CH=${CH:-"gaussian5;gaussian7;sobel;box3"}
SHAPE=${SHAPE:-16384x16384x3}
ALTS=${ALTS:-build_alt}
for rep in 1 2; do
  for d in . $ALTS; do
    timeout -k 10 300 python $d/tools/kbench.py --chains "$CH" --shape $SHAPE --iters 30 2>&1 | grep -v amdgpu | sed "s#^#$d #" || exit 1
  done
done
