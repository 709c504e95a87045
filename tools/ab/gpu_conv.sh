#!/bin/bash
# General MFMA conv: correctness tests, timing of conv:31 / conv:9 on one N=8
# stripe and the full 16K RGB frame, conv:31 gray, and a kernel trace.
# Output: gpurun_out/conv/.
set -o pipefail
O=gpurun_out/conv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "general_conv or conv_asym or sep_matches" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
C31=$(cat tools/conv31_chain.txt)
C9="conv:9:$(python -c "print(';'.join(['0.0123456']*81))")"
timeout -k 10 200 python tools/kbench.py --shape 16384x2048x3 --chains "$C31|$C9" --iters 10 --warmup 2 2>&1 | grep -v amdgpu.ids | tee $O/kb_stripe.txt
timeout -k 10 200 python tools/kbench.py --shape 16384x16384x3 --chains "$C31|" --iters 3 --warmup 1 2>&1 | grep -v amdgpu.ids | tee $O/kb_full.txt
timeout -k 10 200 python tools/kbench.py --shape 16384x4096x1 --chains "$C31|" --iters 10 --warmup 2 2>&1 | grep -v amdgpu.ids | tee $O/kb_gray.txt
[ "$1" = quick ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --shape 16384x2048x3 --chains "$C31|" --iters 5 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/$O/prof/run_results.db > $GRAFT_REPO_ROOT/$O/prof_summary.txt 2>&1
cat $GRAFT_REPO_ROOT/$O/prof_summary.txt
