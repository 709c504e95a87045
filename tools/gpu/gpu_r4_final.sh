#!/bin/bash
# Round-end validation on one MI355X: the GPU suite, smoke(), the driver's
# bench command, the stream-copy ceiling (membench) and the 8K JPEG bench.
set -o pipefail
O=gpurun_out/r4/final7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 200 bin/membench 805306368 > $O/membench_768m.txt 2>&1 || exit 1
timeout -k 10 200 python tools/jpegbench.py --size 8192 > $O/jpeg_8k.json 2>&1 || exit 1
echo done
