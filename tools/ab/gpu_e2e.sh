#!/bin/bash
# e2e transfer-mode comparison (pinned host -> device -> pinned host), headline shape.
set -o pipefail
mkdir -p gpurun_out
for m in zerocopy staged 2d; do
  STRIPE_E2E_MODE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dist-steps 0 --e2e-steps 5 --no-verify > gpurun_out/e2e_$m.log 2>&1 || { tail -20 gpurun_out/e2e_$m.log; exit 1; }
  echo "$m: $(grep -o '"e2e_scope_mpx_s": [0-9.]*' gpurun_out/e2e_$m.log) $(grep -o '"e2e": {[^}]*}' gpurun_out/e2e_$m.log)"
done
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -k e2e -p no:cacheprovider 2>&1 | tail -3
