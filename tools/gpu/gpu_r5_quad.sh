#!/bin/bash
# Round 5: kQuad (4 stacked bands per workgroup, alternating directions: halo
# rows shared inside a CU) against the one-task launch, sepx on the cold N=8
# share, the 16K frame, and config 3's sobel share; cfg3 local auto vs 21.
#   bash tools/gpu/gpu_r5_quad.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-quad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 bin/sepx 2048 0 $O/quad_stamps quad > $O/sepx_quad_2048.txt 2>&1 || exit 2
timeout -k 10 300 bin/sepx 16384 1 "" quad > $O/sepx_quad_16k.txt 2>&1 || exit 3
timeout -k 10 300 bin/sepx 2048 1 "" sobelquad > $O/sepx_sobelquad_warm.txt 2>&1 || exit 4
for d in 0 21 0 21; do
  echo "depth $d" >> $O/cfg3_auto.txt
  timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 50 --warmup 10 --scope resident --backend local --halo-depth $d 2>&1 | grep -v amdgpu.ids >> $O/cfg3_auto.txt || exit 5
done
echo done
