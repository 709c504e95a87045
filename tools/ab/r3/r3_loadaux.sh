#!/bin/bash
# stencil load cache policy A/B: side builds with kLoadAux = 1 (sc0) / 16 (sc1) vs the default 0
set -o pipefail
kb() { timeout -k 10 200 python3 $1/tools/kbench.py --chains "$2" --shape $3 --bands=-1 --iters 50 2>/dev/null | python3 -c "import json,sys; print(' '.join(str(json.loads(l)['ms']) for l in sys.stdin if l.strip()))"; }
for rep in 1 2; do
  for d in . build_alt_aux1 build_alt_aux16; do
    echo "$d g5-16K $(kb $d 'gaussian5|' 16384x16384x3)  g5-stripe $(kb $d 'gaussian5|' 16384x2048x3)  ref $(kb $d 'gray:ref,contrast:3.5,emboss3@skip,expand|' 16384x16384x3)" || exit 1
  done
done
