#!/bin/bash
# Config-level checks on one GPU: CLI local/rccl backends, torchrun path, config kernels.
set -o pipefail
mkdir -p gpurun_out
S=bin/stripe
timeout -k 10 120 $S info > gpurun_out/info.log 2>&1; cat gpurun_out/info.log | grep -v amdgpu.ids
timeout -k 10 120 $S gen --synthetic 1000x700x3 --seed 3 --output /tmp/in.ppm || exit 1
timeout -k 10 120 $S run --input /tmp/in.ppm --output /tmp/a.ppm --chain "gaussian5,sobel" --ranks 1 --backend host > /dev/null || exit 1
timeout -k 10 120 $S run --input /tmp/in.ppm --output /tmp/b.ppm --chain "gaussian5,sobel" --ranks 4 --backend local || exit 1
timeout -k 10 120 $S run --input /tmp/in.ppm --output /tmp/c.ppm --chain "gaussian5,sobel" --ranks 1 --backend rccl || exit 1
timeout -k 10 60 $S cmp /tmp/a.ppm /tmp/b.ppm && timeout -k 10 60 $S cmp /tmp/a.ppm /tmp/c.ppm || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_torchrun.log 2>&1 || { tail -20 gpurun_out/bench_torchrun.log; exit 1; }
grep '^{' gpurun_out/bench_torchrun.log
timeout -k 10 300 python tools/kbench.py --shape 8192x8192x1 --chains "sobel" --bands 0 --iters 30 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/kbench.py --shape 16384x2048x3 --chains "blur:31" --bands 0 --iters 5 --warmup 1 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 $S bench --synthetic 16384x16384x3 --chain gaussian5 --ranks 1 --iters 50 --warmup 10 --scope resident,dist --backend rccl 2>&1 | grep -v amdgpu.ids
