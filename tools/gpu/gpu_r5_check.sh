#!/bin/bash
# Round 5: GPU tests, the driver's bench command, the N=8 share, and a kernel
# trace of the share's bench run (what the engine launches per step).
#   bash tools/gpu/gpu_r5_check.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-check}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_gpu.txt 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --height 2048 > $O/bench_stripe.json 2> $O/bench_stripe.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_stripe -o stripe -- python3 bench.py --steps 20 --warmup 5 --height 2048 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/prof_stripe.log 2>&1 || exit 5
echo done
