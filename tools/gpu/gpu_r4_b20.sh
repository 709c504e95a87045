#!/bin/bash
set -o pipefail
O=gpurun_out/r4/b20
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/b20_$i.json 2> $O/b20_$i.err || exit 1
done
echo done
