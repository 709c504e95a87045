#!/bin/bash
# halo-schedule probe on the gloo-gpu rehearsal + config-3 local ranks with the CLI's stage events off
set -o pipefail
O=gpurun_out/r4/sched
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shared.py -k bench -x -v --timeout 300 --timeout-method thread > $O/test.txt 2>&1 || exit 1
B="bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --warmup 8 --scope resident --backend local"
for it in 48 480; do
  echo "== iters $it auto depth" >> $O/local.txt
  timeout -k 10 120 $B --iters $it 2>&1 | grep -v amdgpu.ids >> $O/local.txt || exit 1
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo-gpu --width 16384 --height 4096 --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/bench_gg2.json 2> $O/bench_gg2.err || exit 1
echo done
