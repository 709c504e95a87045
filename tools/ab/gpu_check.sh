#!/bin/bash
# First-pass GPU validation: smoke -> GPU tests -> short 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest gpu rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench1.log 2>gpurun_out/bench1.err; rc=$?
cat gpurun_out/bench1.log
exit $rc
