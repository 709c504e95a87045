#!/bin/bash
# DB blur kernel (STRIPE_BLUR_DB=1/2) and conv lsb mode: GPU tests, then timings
set -o pipefail
bash tools/ab/r3/r3_blur_db.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "lsb" > gpurun_out/r3_lsb_tests.txt 2>&1 || { tail -30 gpurun_out/r3_lsb_tests.txt; exit 1; }
grep -E "off by one|passed|failed" gpurun_out/r3_lsb_tests.txt
W=$(python3 -c "print(';'.join(str(((7*i)%13-4)/400) for i in range(961)))")
for p in "" ":lsb" "" ":lsb"; do for sh in 16384x16384x3 16384x2048x3 16384x16384x1; do echo -n "conv:31$p $sh "; timeout -k 10 200 python3 tools/kbench.py --chains "conv:31:$W$p|" --shape $sh --iters 10 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; done; done
