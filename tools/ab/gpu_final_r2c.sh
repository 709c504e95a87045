#!/bin/bash
# End-of-session validation: full GPU suite, smoke, headline bench, a 32768^2 RGB frame (chunked views)
set -o pipefail
mkdir -p gpurun_out/final_r2c
export PYTHONUNBUFFERED=1
O=gpurun_out/final_r2c
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python tools/kbench.py --shape 32768x32768x3 --chains "gaussian5|gray:ref,contrast:3.5,emboss3@skip,expand" --iters 10 --warmup 2 2>&1 | grep chain > $O/big_frame.jsonl || exit 1
cat $O/big_frame.jsonl
