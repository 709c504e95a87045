#!/bin/bash
# gloo-gpu: N processes sharing the box's GPU run the multi-rank device path
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_shared.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_shared_tests.txt 2>&1 || { tail -40 gpurun_out/r3_shared_tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r3_shared_tests.txt | tail -8
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo-gpu --steps 10 --warmup 3 --dist-steps 2 --ref-steps 1 --e2e-steps 1 > gpurun_out/r3_shared_16k_n2.json 2> gpurun_out/r3_shared_16k_n2.log || { tail -30 gpurun_out/r3_shared_16k_n2.log; exit 1; }
cat gpurun_out/r3_shared_16k_n2.json | head -c 3000
