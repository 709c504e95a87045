#!/bin/bash
# i8 weight-digit MFMA conv: correctness (GPU conv tests + torch fp64 oracle) and speed vs the f16 hi+lo kernel
set -o pipefail
O=gpurun_out/r3conv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_oracle_conv.py tests/test_n8.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv or blur" > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt
[ $rc -ne 0 ] && exit $rc
CONV="conv:31:$(python3 -c "print(';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
CONV9="conv:9:$(python3 -c "print(';'.join(str(((i*7)%13-4)/40.0) for i in range(81)))")"
for sh in 16384x16384x3 16384x2048x3 16384x16384x1; do
  timeout -k 10 300 python3 tools/kbench.py --chains "$CONV|" --shape $sh --iters 10 >> $O/kb_i8.jsonl 2>/dev/null || exit 1
  STRIPE_CONV_F16=1 timeout -k 10 300 python3 tools/kbench.py --chains "$CONV|" --shape $sh --iters 10 >> $O/kb_f16.jsonl 2>/dev/null || exit 1
done
timeout -k 10 300 python3 tools/kbench.py --chains "$CONV9|" --shape 16384x16384x3 --iters 10 >> $O/kb_i8.jsonl 2>/dev/null
STRIPE_CONV_F16=1 timeout -k 10 300 python3 tools/kbench.py --chains "$CONV9|" --shape 16384x16384x3 --iters 10 >> $O/kb_f16.jsonl 2>/dev/null
echo i8; cut -c1-60,200-300 $O/kb_i8.jsonl; echo f16; cut -c1-60,200-300 $O/kb_f16.jsonl
bash scripts/profile.sh "$CONV|" 16384x2048x3 gpurun_out/r3prof_conv > /dev/null 2>&1 && echo conv prof done
grep -A9 "k_conv_i8" gpurun_out/r3prof_conv/summary.txt | grep -v "^--" | head -60
