#!/bin/bash
# gray:ref prologue: multiply-shift terms (this tree) vs LDS term tables (build_alt2 = previous commit)
set -o pipefail
#timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_r3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gray or ref or chain or skip or pipeline or occupancy" > gpurun_out/r3_grayref_tests.txt 2>&1 || { tail -30 gpurun_out/r3_grayref_tests.txt; exit 1; }
#tail -1
for rep in 1 2; do
for v in alu lut; do
  pp=$(pwd); [ $v = lut ] && pp=$(pwd)/build_alt2
  for ch in 'gray:ref,contrast:3.5,emboss3@skip,expand' 'gray:ref,contrast:3.5,emboss3@skip' 'gray:ref,contrast:3.5,emboss3'; do
    echo -n "$v $ch "; PYTHONPATH=$pp timeout -k 10 200 python3 $pp/tools/kbench.py --chains "$ch|" --shape 16384x16384x3 --bands=-1 --iters 30 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'], r.get('caps'), r.get('bands'))"
  done
done
done
