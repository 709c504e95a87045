#!/bin/bash
# blur:31 with s_setprio around the tile loop (build_alt3: prio 1 while computing, build_alt4: prio 1 while staging)
set -o pipefail
for rep in 1 2; do
for v in base p_compute p_stage; do
  pp=$(pwd); [ $v = p_compute ] && pp=$(pwd)/build_alt3; [ $v = p_stage ] && pp=$(pwd)/build_alt4
  for sh in 16384x16384x3 16384x2048x3 16384x16384x1; do
    echo -n "$v $sh "; PYTHONPATH=$pp timeout -k 10 200 python3 $pp/tools/kbench.py --chains "blur:31|" --shape $sh --iters 20 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"
  done
done
done
