#!/bin/bash
# Round 5: config 3 on 4 `local` ranks at halo depths 8 / 16 / 21 / 32
# (alternating), then counters of the round-5 blur:31 kernels (exact, lsb).
#   bash tools/gpu/gpu_r5_i.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-i}
mkdir -p $O
export TMPDIR=/tmp
for d in 8 16 21 32 8 16 21 32; do
  echo "depth $d" >> $O/cfg3_depths.txt
  timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 64 --warmup 8 --scope resident --backend local --halo-depth $d 2>&1 | grep -v amdgpu.ids >> $O/cfg3_depths.txt || exit 2
done
timeout -k 10 600 bash scripts/profile.sh "blur:31|" 16384x16384x3 $O/prof_blur31 > $O/prof_blur31.txt 2>&1 || exit 3
timeout -k 10 600 bash scripts/profile.sh "blur:31:lsb|" 16384x16384x3 $O/prof_blur31_lsb > $O/prof_blur31_lsb.txt 2>&1 || exit 4
echo done
