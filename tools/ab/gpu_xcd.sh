#!/bin/bash
# A/B: XCD-aware workgroup remap (STRIPE_XCD=8) vs hardware order, via kernel traces.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for x in 0 8; do
  STRIPE_XCD=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/xcd$x -o r -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --chains "gaussian5;sobel;emboss3;blur:31" --shape 16384x16384x3 --iters 20 > $GRAFT_REPO_ROOT/gpurun_out/xcd$x.log 2>&1 || exit 1
  STRIPE_XCD=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/xcds$x -o r -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --chains "gaussian5;blur:31" --shape 16384x2048x3 --iters 40 > $GRAFT_REPO_ROOT/gpurun_out/xcds$x.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && for x in 0 8; do echo "== XCD=$x"; python tools/prof_summary.py gpurun_out/xcd$x/r_results.db | grep -E "k_sep|k_direct|k_blur" ; python tools/prof_summary.py gpurun_out/xcds$x/r_results.db | grep -E "k_sep|k_direct|k_blur"; done
