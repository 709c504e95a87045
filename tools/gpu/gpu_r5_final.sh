#!/bin/bash
# Round 5 validation pass: the GPU test suite, smoke(), the driver's bench
# command at N=1, and the five BASELINE.json configs (tools/gpu/gpu_configs.sh).
#   bash tools/gpu/gpu_r5_final.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_gpu.txt 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 3
timeout -k 10 600 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 4
O=$O/configs timeout -k 10 1200 bash tools/gpu/gpu_configs.sh || exit 5
echo done
