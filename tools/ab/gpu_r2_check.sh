#!/bin/bash
# GPU check: the -m gpu suite, the headline bench and a rocprofv3 kernel trace
# of it.  Output: gpurun_out/r2/.
set -o pipefail
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --dist-steps 0 --e2e-steps 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/$O/prof/run_results.db > $GRAFT_REPO_ROOT/$O/prof_summary.txt 2>&1
echo done
