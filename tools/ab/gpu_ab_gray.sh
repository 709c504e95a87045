#!/bin/bash
# Gray-prologue kernels: GPU numerics, then current tree vs build_alt2 on 16K RGB
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/abg_pytest.log 2>&1 || { tail -30 gpurun_out/abg_pytest.log; exit 1; }
tail -1 gpurun_out/abg_pytest.log
CH=${CH:-"gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|gray,gaussian5|gray,sobel,expand|gaussian5"}
for rep in 1 2; do
  for d in . build_alt2; do
    timeout -k 10 300 python $d/tools/kbench.py --chains "$CH" --shape 16384x16384x3 --iters 40 2>&1 | grep -v amdgpu | sed "s#^#$d #" || exit 1
  done
done
