#!/bin/bash
# Restored-tree validation: full GPU suite, smoke, headline bench, rocprofv3 kernel
# trace of the bench, blur:31 timings (baseline of the blur scheduling work).
set -o pipefail
O=gpurun_out/${R2D_OUT:-r2d}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --dist-steps 0 --e2e-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
for shape in 16384x2048x3 16384x16384x3 8192x8192x1; do
  timeout -k 10 120 python tools/kbench.py --shape $shape --chains "blur:31" --iters 20 --warmup 3 2>&1 | grep chain >> $O/blur.jsonl || exit 1
done
cat $O/blur.jsonl
