#!/bin/bash
# reference pipeline (1-channel and expand) with the XCD remap forced on / off, autotuned
set -o pipefail
kb() { timeout -k 10 200 python3 tools/kbench.py --chains "$1" --shape 16384x16384x3 --bands=-1 --iters 30 2>/dev/null | python3 -c "import json,sys; print(' '.join(str(json.loads(l)['ms']) + '(b' + str(json.loads(l)['bands'][0]) + ',c' + str(json.loads(l)['caps'][0]) + ')' for l in sys.stdin if l.strip()))"; }
for rep in 1 2; do
  for x in 0 8; do
    echo "xcd=$x $(STRIPE_XCD=$x kb 'gray:ref,contrast:3.5,emboss3@skip|gray:ref,contrast:3.5,emboss3@skip,expand|gaussian5|')" || exit 1
  done
done
