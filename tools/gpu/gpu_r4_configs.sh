#!/bin/bash
# Round-4 refresh of the five BASELINE configs (tools/gpu/gpu_configs.sh) plus the
# config-3 local-rank schedules side by side.  Output: gpurun_out/r4/configs.
set -o pipefail
export O=gpurun_out/r4/configs
mkdir -p $O
timeout -k 10 900 bash tools/gpu/gpu_configs.sh || exit 1
for d in 1 4 8; do
  echo "== cfg3 sobel 4 local ranks, halo depth $d" >> $O/configs.txt
  timeout -k 10 200 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 48 --warmup 8 \
    --scope resident --backend local --halo-depth $d 2>&1 | grep -v amdgpu.ids >> $O/configs.txt || exit 1
done
for s in serial overlap pipeline; do
  echo "== cfg3 sobel 4 local ranks, schedule $s" >> $O/configs.txt
  STRIPE_HALO_SCHEDULE=$s timeout -k 10 200 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 \
    --iters 48 --warmup 8 --scope resident --backend local --halo-depth 1 2>&1 | grep -v amdgpu.ids >> $O/configs.txt || exit 1
done
echo done
