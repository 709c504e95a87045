#!/bin/bash
# Fused expand epilogue: GPU numerics + timing of the reference chain with and
# without the expand (16K RGB frame).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_engine.py -k "expand or chains or deep_halo or ref_gpu or multipass" \
  > gpurun_out/expand_tests.log 2>&1 || { tail -40 gpurun_out/expand_tests.log; exit 1; }
tail -3 gpurun_out/expand_tests.log
timeout -k 10 300 python -u tools/kbench.py --shape 16384x16384x3 --iters 30 \
  --chains "gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|gray,gaussian5,expand|gaussian5" \
  > gpurun_out/expand_kbench.log 2>&1 || { tail -20 gpurun_out/expand_kbench.log; exit 1; }
cat gpurun_out/expand_kbench.log
