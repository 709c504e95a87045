#!/bin/bash
# Large-kernel blur iteration: MFMA conv tests + timing + kernel profile (config 5 shapes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -k "mfma" -x -q -p no:cacheprovider > gpurun_out/pytest_blur.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_blur.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_blur.log; exit 1; }
timeout -k 10 300 python tools/kbench.py --chains "blur:31;blur:9" --shape 16384x2048x3 --bands ${BANDS:-0,128,384} --iters 20 > gpurun_out/blur_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/blur_bench.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/kbench.py --chains "blur:31" --shape 16384x16384x3 --iters 5 > gpurun_out/blur_bench16k.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/blur_bench16k.log
[ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_blur -o blur -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --chains "blur:31" --shape 16384x2048x3 --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_blur.log 2>&1
