#!/bin/bash
# rocprofv3 kernel trace of the JPEG GPU pixel stages (8K, one rep each of
# every jpegbench path), summarised to a table.
set -o pipefail
O=gpurun_out/r4/jpegprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/jpegbench.py --size 8192 --reps 1 > $O/jpegbench.log 2>&1 || exit 1
python3 tools/prof_summary.py $(find $O/prof -name '*.db' | head -1) > $O/summary.txt 2>&1 || exit 1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \; ; echo done
