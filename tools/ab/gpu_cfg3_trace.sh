#!/bin/bash
# config 3 (sobel, 8192^2 gray): kernel time vs wall time per pass, eager vs hipGraph
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kbench.py --chains sobel --shape 8192x8192x1 --iters 200 --warmup 20 2>&1 | grep chain || exit 1
timeout -k 10 200 python tools/kbench.py --chains sobel --shape 8192x8192x1 --iters 200 --warmup 20 --graphs 2>&1 | grep chain || exit 1
timeout -k 10 200 python tools/kbench.py --chains sobel --shape 8192x2048x1 --iters 200 --warmup 20 2>&1 | grep chain || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/cfg3trace -o run -- python tools/kbench.py --chains sobel --shape 8192x8192x1 --iters 50 --warmup 5 > gpurun_out/cfg3trace.log 2>&1 || { tail -5 gpurun_out/cfg3trace.log; exit 1; }
python tools/prof_summary.py gpurun_out/cfg3trace/run_results.db | head -12
