#!/bin/bash
# N=8 share (16384x2048 RGB gaussian5, cold frame stream): frames x streams sweep
set -o pipefail
O=gpurun_out/r4/streams2
mkdir -p $O
: > $O/sweep.txt
for fs in "4 2" "4 3" "4 4" "6 2" "6 3" "8 4"; do
  set -- $fs
  timeout -k 10 120 python bench.py --height 2048 --steps 100 --warmup 10 --frames $1 --streams $2 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/f$1_s$2.json 2> $O/f$1_s$2.err || exit 1
  python3 -c "
import json,sys;r=json.loads(open('$O/f$1_s$2.json').read().strip().splitlines()[-1])
print('frames $1 streams $2', r['ms_per_step'], r['step_ms_device'], r['tuned'])" >> $O/sweep.txt
done
echo done
