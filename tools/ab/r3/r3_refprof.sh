#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_kern_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r3_kern_tests.txt
[ $rc -ne 0 ] && exit $rc
bash scripts/profile.sh 'gray:ref,contrast:3.5,emboss3@skip,expand|' 16384x16384x3 gpurun_out/r3prof_ref > /dev/null 2>&1 && echo ref done &&
bash scripts/profile.sh 'gray:ref,contrast:3.5,emboss3@skip|' 16384x16384x3 gpurun_out/r3prof_refg > /dev/null 2>&1 && echo refg done &&
bash scripts/profile.sh 'gaussian5|' 16384x16384x3 gpurun_out/r3prof_g5 > /dev/null 2>&1 && echo g5 done
