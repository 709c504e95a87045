#!/bin/bash
set -o pipefail
O=gpurun_out/pw_confirm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for w in 0 3; do
  STRIPE_PW_WGS=$w timeout -k 10 150 python tools/kbench.py --shape 16384x16384x3 --chains "invert|brightness:20|threshold:100" --iters 30 --warmup 5 2>&1 | grep chain | sed "s/^/$w /" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
