#!/bin/bash
# Round 5, first GPU pass: GPU tests on the task-loop k_sep, the driver's bench
# command, and the cold N=8 share experiments (tools/sepx.hip: store policy,
# band x cap, persistent task loop, per-wave stamps, copy floor; kernel-only
# times from rocprofv3).
set -o pipefail
O=gpurun_out/r5/a
mkdir -p $O
export TMPDIR=/tmp
# a test failure (rc 1) still lets the measurements run; anything else stops
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_gpu.txt 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --frames 1 --streams 1 > $O/bench_n1_f1s1.json 2> $O/bench_n1_f1s1.err || exit 3
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --height 2048 > $O/bench_stripe.json 2> $O/bench_stripe.err || exit 3
timeout -k 10 120 bin/sepx 2048 0 $O/stamps > $O/sepx_2048.txt 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_sepx -o sepx -- bin/sepx 2048 0 > $O/prof_sepx.txt 2>&1 || exit 5
timeout -k 10 200 bin/sepx 16384 1 $O/stamps16k > $O/sepx_16384.txt 2>&1 || exit 6
echo done
