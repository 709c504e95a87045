#!/bin/bash
set -o pipefail
O=gpurun_out/r3tests
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1; rc=$?
tail -15 $O/gpu_tests.txt
exit $rc
