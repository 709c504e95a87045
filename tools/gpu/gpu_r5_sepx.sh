#!/bin/bash
# Round 5: tools/sepx.hip on the cold N=8 share and the full 16K frame, with
# per-wave stamps, and a rocprofv3 kernel trace of the share.
#   bash tools/gpu/gpu_r5_sepx.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-sepx}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 bin/sepx 2048 0 $O/stamps > $O/sepx_2048.txt 2>&1 || exit 4
timeout -k 10 200 bin/sepx 16384 1 $O/stamps16k > $O/sepx_16384.txt 2>&1 || exit 6
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_sepx -o sepx -- bin/sepx 2048 0 > $O/prof_sepx.txt 2>&1 || exit 5
echo done
