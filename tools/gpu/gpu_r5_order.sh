#!/bin/bash
# Round 5: the separable task order (kRuns) in production: its GPU tests, the
# driver's bench command with the order pinned 0 / 1 / tuned (alternating),
# kbench on the 16K frame and the N=8 stripe.
#   bash tools/gpu/gpu_r5_order.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-order}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_r5_order.py tests/test_gpu_r3.py tests/test_gpu_engine.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
for r in 1 2; do
  for o in 0 1 t; do
    if [ $o = t ]; then unset STRIPE_SEP_ORDER; else export STRIPE_SEP_ORDER=$o; fi
    timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/bench_o${o}_$r.json 2> $O/bench_o${o}_$r.err || exit 3
  done
done
unset STRIPE_SEP_ORDER
for o in 0 1 0 1; do
  STRIPE_SEP_ORDER=$o timeout -k 10 200 python tools/kbench.py --chains "gaussian5|gaussian3" --shape 16384x16384x3 --bands=-1 --iters 30 >> $O/kb_16k_o$o.txt 2>&1 || exit 4
  STRIPE_SEP_ORDER=$o timeout -k 10 200 python tools/kbench.py --chains "gaussian5" --shape 16384x2048x3 --bands=-1 --iters 50 >> $O/kb_stripe_o$o.txt 2>&1 || exit 4
done
echo done
