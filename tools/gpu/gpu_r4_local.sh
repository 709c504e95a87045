#!/bin/bash
# Config 3 on 4 local ranks (one GPU): where the per-step time goes.
set -o pipefail
O=gpurun_out/r4/local
mkdir -p $O
B="bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 48 --warmup 8 --scope resident --backend local"
run() { local name=$1; shift; echo "== $name" >> $O/local.txt
  timeout -k 10 120 "$@" 2>&1 | grep -v amdgpu.ids >> $O/local.txt || { echo "FAILED: $name" >> $O/local.txt; exit 1; }; }
: > $O/local.txt
run "depth 8" $B --halo-depth 8
run "depth 8, no stage events" env STRIPE_STAGE_EVENTS=0 $B --halo-depth 8
run "depth 8, graphs" $B --halo-depth 8 --graphs
run "depth 8, graphs, no stage events" env STRIPE_STAGE_EVENTS=0 $B --halo-depth 8 --graphs
run "depth 1, no stage events" env STRIPE_STAGE_EVENTS=0 $B --halo-depth 1
run "depth 1 serial, no stage events" env STRIPE_STAGE_EVENTS=0 STRIPE_HALO_SCHEDULE=serial $B --halo-depth 1
run "1 rank full frame, no stage events" env STRIPE_STAGE_EVENTS=0 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 1 --iters 48 --warmup 8 --scope resident --backend local
STRIPE_STAGE_EVENTS=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -- bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 48 --warmup 8 --scope resident --backend local --halo-depth 8 > $O/prof8.log 2>&1 || exit 1
STRIPE_STAGE_EVENTS=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 48 --warmup 8 --scope resident --backend local --halo-depth 1 > $O/prof1.log 2>&1 || exit 1
echo done
