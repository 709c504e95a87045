#!/bin/bash
# The five BASELINE.json configs on one MI355X (round 3): multi-rank configs as
# one rank's share (the per-GPU work of an N-GPU run) and as N logical ranks on
# the one GPU via the `local` backend; the real N-GPU curve comes from the
# driver's SCALE runs.  Stencil configs autotune band height x occupancy cap
# (--bands=-1), as bench.py does.  Every timed burst is >= ~50 ms of GPU work:
# a 5-iteration burst of conv:31 read 8-12 % slow (clock ramp at the burst's
# start, profiles/r5/conv/README.md).  Output: $O/configs.txt (default gpurun_out/configs).
set -o pipefail
O=${O:-gpurun_out/configs}
mkdir -p $O
S=bin/stripe
KB="python tools/kbench.py"
CONV31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")|"
run() { local name=$1 t=$2; shift 2; echo "== $name" >> $O/configs.txt
  timeout -k 10 $t "$@" 2>&1 | grep -v amdgpu.ids >> $O/configs.txt || { echo "FAILED: $name" >> $O/configs.txt; exit 1; }; }
: > $O/configs.txt
run "cfg1 gray:ref 512x512x3 host backend (CPU)" 120 $S bench --synthetic 512x512x3 --chain gray:ref --ranks 1 --iters 20 --warmup 3 --scope resident --backend host
run "cfg2 gaussian5 4096x4096x3 1 GPU" 200 $KB --shape 4096x4096x3 --chains gaussian5 --bands=-1 --iters 50
run "cfg3 sobel 8192x8192x1 1 GPU (full frame, one rank)" 200 $KB --shape 8192x8192x1 --chains sobel --bands=-1 --iters 50
run "cfg3 sobel one rank's N=4 share 8192x2048x1" 200 $KB --shape 8192x2048x1 --chains sobel --bands=-1 --iters 50
run "cfg3 sobel 8192x8192x1 4 local ranks on 1 GPU" 200 $S bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 50 --warmup 10 --scope resident --backend local
run "cfg4 gaussian5 16384x16384x3 full frame" 200 $KB --shape 16384x16384x3 --chains gaussian5 --bands=-1 --iters 50
run "cfg4 gaussian5 one N=8 stripe 16384x2048x3" 200 $KB --shape 16384x2048x3 --chains gaussian5 --bands=-1 --iters 50
run "cfg5 blur:31 16384x16384x3 full frame (separable MFMA)" 300 $KB --shape 16384x16384x3 --chains blur:31 --iters 40 --warmup 5
run "cfg5 blur:31 one N=8 stripe 16384x2048x3" 200 $KB --shape 16384x2048x3 --chains blur:31 --iters 100 --warmup 5
run "cfg5 blur:31:lsb (every output within 1 LSB) 16384x16384x3 full frame" 300 $KB --shape 16384x16384x3 --chains "blur:31:lsb|" --iters 40 --warmup 5
run "cfg5 blur:31:lsb one N=8 stripe 16384x2048x3" 200 $KB --shape 16384x2048x3 --chains "blur:31:lsb|" --iters 100 --warmup 5
run "cfg5b conv:31 arbitrary weights 16384x16384x3 full frame (i8 Toeplitz MFMA)" 300 $KB --shape 16384x16384x3 --chains "$CONV31" --iters 30 --warmup 5
run "cfg5b conv:31 one N=8 stripe 16384x2048x3" 200 $KB --shape 16384x2048x3 --chains "$CONV31" --iters 60 --warmup 5
run "cfg5b conv:31:lsb arbitrary weights 16384x16384x3 full frame" 300 $KB --shape 16384x16384x3 --chains "${CONV31%|}:lsb|" --iters 30 --warmup 5
run "reference pipeline gray:ref,contrast:3.5,emboss3@skip,expand 16384x16384x3" 200 $KB --shape 16384x16384x3 --chains "gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|" --bands=-1 --iters 30
echo done
