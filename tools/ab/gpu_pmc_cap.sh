#!/bin/bash
# Counters of the 16K RGB gaussian5 pass with and without the HBM-streaming occupancy cap.
set -o pipefail
O=gpurun_out/pmc_cap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in 0 2; do
  STRIPE_NT_WGS=$w timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/sq_$w -o run -- python3 tools/kbench.py --shape 16384x16384x3 --chains gaussian5 --bands 16 --iters 10 --warmup 2 > $O/sq_$w.log 2>&1 || { tail -5 $O/sq_$w.log; exit 1; }
  STRIPE_NT_WGS=$w timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fs_$w -o run -- python3 tools/kbench.py --shape 16384x16384x3 --chains gaussian5 --bands 16 --iters 10 --warmup 2 > $O/fs_$w.log 2>&1 || { tail -5 $O/fs_$w.log; exit 1; }
done
for w in 0 2; do python3 tools/prof_summary.py $O/sq_$w/run_results.db $O/fs_$w/run_results.db > $O/summary_$w.txt 2>&1; done
echo done
