#!/bin/bash
# DB (double-buffered, one wave per SIMD) blur:K kernel against the default: tests + timings
set -o pipefail
for d in 1 2; do STRIPE_BLUR_DB=$d timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_oracle_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "blur or sep" >> gpurun_out/r3_blurdb_tests.txt 2>&1 || { tail -30 gpurun_out/r3_blurdb_tests.txt; exit 1; }; done
tail -1 gpurun_out/r3_blurdb_tests.txt
for db in 0 1 2 0 1 2; do for sh in 16384x16384x3 16384x2048x3; do echo -n "db=$db $sh "; STRIPE_BLUR_DB=$db timeout -k 10 200 python3 tools/kbench.py --chains 'blur:31|' --shape $sh --iters 20 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; done; done
