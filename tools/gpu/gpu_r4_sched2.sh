#!/bin/bash
# schedule x streams probe: gloo-gpu tests, a 16K N=2 rehearsal (2 frames, stripes beyond the cache), N=1 headline
set -o pipefail
O=gpurun_out/r4/sched2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shared.py tests/test_r4_comm.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.txt 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo-gpu --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/bench_16k_gg2.json 2> $O/bench_16k_gg2.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
echo done
