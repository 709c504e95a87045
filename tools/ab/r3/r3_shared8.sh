#!/bin/bash
# rehearsal of the driver's N = 4 / 8 bench flow with every rank on the box's one GPU (gloo-gpu)
set -o pipefail
for n in 4 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2954$n bench.py --gpus $n --backend gloo-gpu --steps 10 --warmup 3 --dist-steps 2 --ref-steps 1 --e2e-steps 1 > gpurun_out/r3_shared_16k_n$n.json 2> gpurun_out/r3_shared_16k_n$n.log || { tail -30 gpurun_out/r3_shared_16k_n$n.log; exit 1; }
  python3 -c "
import json; r=json.loads(open('gpurun_out/r3_shared_16k_n$n.json').read().strip().splitlines()[-1])
print($n, r['ms_per_step'], r['verified_vs_golden'], r['halo_depth'], r['stripe_rows'], {k: (v.get('ms'), v.get('verified'), v.get('error')) for k, v in r['scopes'].items()})"
done
