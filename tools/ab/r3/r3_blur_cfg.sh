#!/bin/bash
# blur:K GPU check: every blur/sep/conv GPU test, then kbench timings
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "blur or sep or conv" > gpurun_out/r3_blurcfg_tests.txt 2>&1 || { tail -30 gpurun_out/r3_blurcfg_tests.txt; exit 1; }
tail -1 gpurun_out/r3_blurcfg_tests.txt
for sh in 16384x16384x3 16384x2048x3 16384x16384x1 16384x2048x1 16384x16384x3; do echo -n "$sh "; timeout -k 10 200 python3 tools/kbench.py --chains 'blur:31|' --shape $sh --iters 20 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; done
