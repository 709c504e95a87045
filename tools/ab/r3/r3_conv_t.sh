#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_oracle_conv.py tests/test_n8.py tests/test_gpu_large.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv or blur or large" > gpurun_out/r3_convt.txt 2>&1; rc=$?
tail -2 gpurun_out/r3_convt.txt
exit $rc
