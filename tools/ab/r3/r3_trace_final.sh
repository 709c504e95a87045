#!/bin/bash
# kernel trace of the driver's bench command (this build), then the gloo-gpu
# N=2 / N=4 bench flow on the one GPU (multi-process device path still intact)
set -o pipefail
ROOT=$(pwd); O=$ROOT/gpurun_out/r3trace; mkdir -p $O
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err ) && echo trace done &&
python3 tools/prof_summary.py $O/prof/run_results.db > $O/summary.txt 2>&1; head -30 $O/summary.txt
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --backend gloo-gpu --steps 10 --warmup 3 --dist-steps 2 --ref-steps 1 --e2e-steps 1 > $O/shared_n$n.json 2> $O/shared_n$n.log || { tail -30 $O/shared_n$n.log; exit 1; }
  python3 -c "
import json; r=json.load(open('$O/shared_n$n.json')); print($n, r['ms_per_step'], r['verified_vs_golden'], {k:(v.get('ms'), v.get('verified'), v.get('error')) for k,v in r['scopes'].items()})"
done
