#!/bin/bash
# HBM read bytes (FETCH_SIZE; gfx950 reports half, MI355X_MICROARCH.md) of the
# 16K RGB gaussian5 pass at several band heights, with and without the XCD remap.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fetch
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for b in 8 12 32; do
  for x in 0 8; do
    STRIPE_XCD=$x timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/b${b}_x$x -o run -- python3 $R/tools/kbench.py --shape 16384x16384x3 --chains gaussian5 --bands $b --iters 4 --warmup 1 > $O/b${b}_x$x.log 2>&1 || exit 1
    python3 $R/tools/prof_summary.py $O/b${b}_x$x/run_results.db 2>&1 | grep -A3 "k_sep" | sed "s/^/band=$b xcd=$x /" >> $O/summary.txt
  done
done
