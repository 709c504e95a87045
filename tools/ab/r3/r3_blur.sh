#!/bin/bash
# planar MFMA blur: correctness (blur/sepconv GPU tests + torch oracle) and speed
set -o pipefail
O=gpurun_out/r3blur
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_oracle_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "blur or sep or sepconv" > $O/tests.txt 2>&1; rc=$?
tail -5 $O/tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/kbench.py --chains 'blur:31|blur:15|blur:33' --shape 16384x16384x3 --iters 20 > $O/kb_rgb.jsonl 2>&1 &&
timeout -k 10 300 python3 tools/kbench.py --chains 'blur:31' --shape 16384x2048x3 --iters 50 >> $O/kb_rgb.jsonl 2>&1 &&
timeout -k 10 300 python3 tools/kbench.py --chains 'blur:31' --shape 16384x16384x1 --iters 20 >> $O/kb_rgb.jsonl 2>&1
cat $O/kb_rgb.jsonl
timeout -k 10 60 ./bin/mfma_i8_probe
