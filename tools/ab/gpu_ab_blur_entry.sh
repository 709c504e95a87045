#!/bin/bash
# blur (separable MFMA): masked entry-step stores (precise vmcnt) vs build_alt2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "blur or sep" > gpurun_out/be_pytest.log 2>&1 || { tail -30 gpurun_out/be_pytest.log; exit 1; }
tail -1 gpurun_out/be_pytest.log
for rep in 1 2; do
  for d in . build_alt2; do
    timeout -k 10 200 python $d/tools/kbench.py --chains "blur:31|blur:15" --shape 16384x2048x3 --iters 50 --warmup 5 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "blur:31" --shape 16384x16384x3 --iters 10 --warmup 3 2>&1 | grep chain | sed "s#^#$d #" || exit 1
    timeout -k 10 200 python $d/tools/kbench.py --chains "blur:31" --shape 16384x4096x1 --iters 50 --warmup 5 2>&1 | grep chain | sed "s#^#$d #" || exit 1
  done
done
