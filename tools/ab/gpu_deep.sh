#!/bin/bash
# Deep-halo validation + schedule comparison on one MI355X:
#   GPU tests (deep halo first), then 8 local ranks (one device, in-process
#   device-copy exchange) at halo depth 1 (pipelined / overlap schedules) vs auto.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "deep_halo or pipelined" > gpurun_out/pytest_deep.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_deep.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_deep.log; exit 1; }
: > gpurun_out/deep_bench.log
for shape in 16384x16384x3 8192x8192x1; do  # resident: one run(iters) call
  for d in 1 0; do
    for sched in pipeline overlap; do
      echo "shape=$shape depth=$d sched=$sched" >> gpurun_out/deep_bench.log
      STRIPE_HALO_SCHEDULE=$sched timeout -k 10 120 bin/stripe bench --synthetic $shape --chain gaussian5 --ranks 2,4,8 \
        --backend local --iters 100 --warmup 10 --scope resident --halo-depth $d >> gpurun_out/deep_bench.log 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids gpurun_out/deep_bench.log | cut -c1-200
