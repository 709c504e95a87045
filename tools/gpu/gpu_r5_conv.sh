#!/bin/bash
# Round 5: conv:31 (i8-digit banded-Toeplitz MFMA) one tile per workgroup vs
# four tiles per workgroup with the next tile's staging under the current
# tile's MFMAs (STRIPE_CONV_NT), exact and :lsb, 16K frame and N=8 stripe; the
# conv GPU tests; counters of the multi-tile kernel.  Then sepx's `wg` sweep
# (waves per workgroup of the gaussian5 stencil) on the N=8 share and the 16K
# frame, and config 3 on 4 `local` ranks at halo depth 1 / 8 / auto (pooled
# exchange events); the engine's separable launches on one-wave workgroups
# (STRIPE_SEP_NW=1): GPU engine tests, kbench and the driver's bench command.
#   bash tools/gpu/gpu_r5_conv.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-conv}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests_conv.txt 2>&1 || exit 2
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
for nt in 1 4 1 4; do
  STRIPE_CONV_NT=$nt timeout -k 10 200 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x16384x3 --iters 6 >> $O/conv31_16k_nt$nt.txt 2>&1 || exit 3
  STRIPE_CONV_NT=$nt timeout -k 10 200 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x2048x3 --iters 20 >> $O/conv31_stripe_nt$nt.txt 2>&1 || exit 3
done
for d in 1 8 0 1; do
  timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 48 --warmup 8 --scope resident --backend local --halo-depth $d >> $O/cfg3_local_depth.txt 2>&1 || exit 7
done
timeout -k 10 300 bin/sepx 2048 0 $O/wg_stamps wg > $O/sepx_wg_2048.txt 2>&1 || exit 4
timeout -k 10 300 bin/sepx 16384 1 "" wg > $O/sepx_wg_16k.txt 2>&1 || exit 5
STRIPE_SEP_NW=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests_nw1.txt 2>&1 || exit 8
for nw in 4 1 4 1; do
  STRIPE_SEP_NW=$nw timeout -k 10 200 python tools/kbench.py --chains "gaussian5|gaussian3" --shape 16384x16384x3 --bands=-1 --iters 30 >> $O/kb_16k_nw$nw.txt 2>&1 || exit 9
  STRIPE_SEP_NW=$nw timeout -k 10 200 python tools/kbench.py --chains "gaussian5" --shape 16384x2048x3 --bands=-1 --iters 50 >> $O/kb_stripe_nw$nw.txt 2>&1 || exit 9
done
STRIPE_SEP_NW=1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_nw1.json 2> $O/bench_nw1.err || exit 10
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_nw4.json 2> $O/bench_nw4.err || exit 10
echo done
