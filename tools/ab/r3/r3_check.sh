#!/bin/bash
# Round 3 GPU check: GPU suite, the driver's bench command, a long bench, and
# an N=8-stripe-sized frame (exercises the cache-cold resident scope).
set -o pipefail
O=gpurun_out/r3check
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && echo driver-bench done &&
timeout -k 10 200 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_200.json 2> $O/bench_200.err && echo bench200 done &&
timeout -k 10 200 python3 bench.py --gpus 1 --height 2048 --steps 100 --warmup 10 > $O/bench_stripe.json 2> $O/bench_stripe.err && echo stripe done
