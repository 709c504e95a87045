#!/bin/bash
set -o pipefail
O=gpurun_out/r4/hwq
mkdir -p $O
: > $O/hwq.txt
for q in 1 2 3 4 1 2 3 4; do
  echo "== GPU_MAX_HW_QUEUES=$q" >> $O/hwq.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 400 --warmup 40 --scope resident --backend local 2>&1 | grep -v amdgpu.ids >> $O/hwq.txt || exit 1
done
echo done
