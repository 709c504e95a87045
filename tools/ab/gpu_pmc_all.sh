#!/bin/bash
# PMC counter summaries for the headline and config kernels (committed to profiles/).
set -o pipefail
CH=gaussian5 SHAPE=16384x16384x3 TAG=pmc_gauss5_16k bash tools/gpu_prof.sh > /dev/null || exit 1
CH=sobel SHAPE=8192x8192x1 TAG=pmc_sobel_8k_gray bash tools/gpu_prof.sh > /dev/null || exit 1
CH="gray:ref,contrast:3.5,emboss3" SHAPE=16384x16384x3 TAG=pmc_refchain_16k bash tools/gpu_prof.sh > /dev/null || exit 1
CH=blur:31 SHAPE=16384x2048x3 TAG=pmc_blur31_stripe bash tools/gpu_prof.sh > /dev/null || exit 1
ls gpurun_out/*_summary.txt
