#!/bin/bash
# Round 3: the reference pipeline (gray:ref -> contrast 3.5 -> emboss3@skip ->
# expand) after the hoisted skip mask, autotuned (band x occupancy cap), vs the
# headline gaussian5 on the same frame; plus bench.py's shared-memory ref window.
set -o pipefail
O=gpurun_out/r3ref
mkdir -p $O
timeout -k 10 300 python3 tools/kbench.py --shape 16384x16384x3 --iters 50 --bands=-1,0 \
  --chains 'gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|gray:ref,contrast:3.5,emboss3|gaussian5|emboss3|gaussian5@skip' > $O/kbench.jsonl 2> $O/kbench.err && echo kbench done &&
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --ref-shm --dist-steps 0 --e2e-steps 0 > $O/bench_shm.json 2> $O/bench_shm.err && echo shm done
cat $O/kbench.jsonl
