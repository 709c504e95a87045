#!/bin/bash
# End-of-round measurement of the five BASELINE.json configs on one MI355X
# (multi-rank configs run as N logical ranks on the one GPU via the `local`
# backend; the real N-GPU curve comes from the driver's SCALE runs), plus a
# rocprofv3 kernel trace of the headline bench.  Output: gpurun_out/final/.
set -o pipefail
O=${O:-gpurun_out/final}
mkdir -p $O
S=bin/stripe
run() { local name=$1 t=$2; shift 2; echo "== $name" >> $O/configs.txt
  timeout -k 10 $t "$@" 2>&1 | grep -v amdgpu.ids >> $O/configs.txt || { echo "FAILED: $name" >> $O/configs.txt; exit 1; }; }
: > $O/configs.txt
run "cfg1 gray:ref 512x512x3 host backend (CPU)" 120 $S bench --synthetic 512x512x3 --chain gray:ref --ranks 1 --iters 20 --warmup 3 --scope resident --backend host
run "cfg2 gaussian5 4096x4096x3 1 GPU" 200 python tools/kbench.py --shape 4096x4096x3 --chains gaussian5 --bands 0 --iters 50
run "cfg3 sobel 8192x8192x1 1 GPU (one rank)" 200 python tools/kbench.py --shape 8192x8192x1 --chains sobel --bands 0 --iters 50
run "cfg3 sobel 8192x8192x1 4 local ranks on 1 GPU" 200 $S bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 50 --warmup 10 --scope resident --backend local
run "cfg4 gaussian5 16384x16384x3 one N=8 stripe" 200 python tools/kbench.py --shape 16384x2048x3 --chains gaussian5 --bands 0 --iters 50
run "cfg5 blur:31 16384x2048x3 one N=8 stripe" 200 python tools/kbench.py --shape 16384x2048x3 --chains blur:31 --bands 0 --iters 10 --warmup 2
run "cfg5 blur:31 16384x16384x3 full frame" 300 python tools/kbench.py --shape 16384x16384x3 --chains blur:31 --bands 0 --iters 5 --warmup 1
run "cfg5b conv:31 (arbitrary 31x31 weights, im2col->MFMA) 16384x2048x3 one N=8 stripe" 200 python tools/kbench.py --shape 16384x2048x3 --chains "$(cat tools/conv31_chain.txt)|" --bands 0 --iters 10 --warmup 2
run "cfg5b conv:31 16384x16384x3 full frame" 300 python tools/kbench.py --shape 16384x16384x3 --chains "$(cat tools/conv31_chain.txt)|" --bands 0 --iters 3 --warmup 1
run "reference chain gray:ref,contrast:3.5,emboss3 16384x16384x3" 200 python tools/kbench.py --shape 16384x16384x3 --chains "gray:ref,contrast:3.5,emboss3" --bands 0 --iters 20
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --dist-steps 0 --e2e-steps 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/$O/prof/run_results.db > $GRAFT_REPO_ROOT/$O/prof_summary.txt 2>&1
echo done
