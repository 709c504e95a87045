#!/bin/bash
# Round 5: kRuns (XCD-local runs of bands in alternating directions, halo rows
# read twice within one L2) against the one-task launch: sepx on the cold N=8
# share and the 16K frame, then L2 fill bytes (FETCH_SIZE) of both at band 16
# and 32 on the 16K frame.
#   bash tools/gpu/gpu_r5_runs.sh <out-subdir>
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r5/${1:-runs}
mkdir -p $O
timeout -k 10 300 bin/sepx 2048 0 $O/runs_stamps runs > $O/sepx_runs_2048.txt 2>&1 || exit 2
timeout -k 10 300 bin/sepx 16384 1 "" runs > $O/sepx_runs_16k.txt 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
for b in 16 32; do
  export SEPX_BAND=$b
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch$b -o run -- $R/bin/sepx 16384 1 "" fetch > $O/pmc_fetch$b.log 2>&1 || exit 4
  python3 $R/tools/prof_summary.py $O/pmc_fetch$b/run_results.db > $O/fetch$b.txt 2>&1 || exit 5
done
echo done
