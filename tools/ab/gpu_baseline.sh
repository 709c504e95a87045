#!/bin/bash
# Measured column of BASELINE.md on one MI355X: every config's full frame on one
# GPU, plus the per-GPU share (one stripe) of the multi-GPU configs.
set -o pipefail
mkdir -p gpurun_out/baseline
B="timeout -k 10 400 python bench.py"
run() { local tag=$1; shift; $B "$@" > gpurun_out/baseline/$tag.log 2>&1 || { tail -20 gpurun_out/baseline/$tag.log; exit 1; }; grep '^{' gpurun_out/baseline/$tag.log > gpurun_out/baseline/$tag.json; echo "$tag $(cut -c1-160 gpurun_out/baseline/$tag.json)"; }
run c2_gauss5_4096_rgb --width 4096 --height 4096 --steps 400 --warmup 40 --e2e-steps 10 --dist-steps 20
run c3_sobel_8192_gray --width 8192 --height 8192 --channels 1 --chain sobel --steps 400 --warmup 40 --e2e-steps 5 --dist-steps 10
run c3_sobel_8192_gray_share4 --width 8192 --height 2048 --channels 1 --chain sobel --steps 400 --warmup 40 --e2e-steps 0 --dist-steps 0
run c4_gauss5_16k_rgb --steps 200 --warmup 20 --e2e-steps 3 --dist-steps 5
run c4_gauss5_16k_rgb_share8 --height 2048 --steps 400 --warmup 40 --e2e-steps 0 --dist-steps 0
run c5_blur31_16k_rgb --chain blur:31 --steps 20 --warmup 3 --e2e-steps 2 --dist-steps 2
run c5_blur31_16k_rgb_share8 --chain blur:31 --height 2048 --steps 100 --warmup 10 --e2e-steps 0 --dist-steps 0
run c4_ref_chain_16k_rgb --chain "gray:ref,contrast:3.5,emboss3" --steps 50 --warmup 5 --e2e-steps 2 --dist-steps 2
run c2_conv3_4096_rgb --width 4096 --height 4096 --chain "conv:3:1;2;1;2;4;2;1;2;1" --steps 200 --warmup 20 --e2e-steps 0 --dist-steps 0
