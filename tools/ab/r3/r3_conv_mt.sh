#!/bin/bash
set -o pipefail
O=gpurun_out/r3convmt
mkdir -p $O
CONV="conv:31:$(python3 -c "print(';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
for mt in 2 3; do
  STRIPE_CONV_MT=$mt timeout -k 10 300 python3 tools/kbench.py --chains "$CONV|" --shape 16384x16384x3 --iters 10 >> $O/kb.jsonl 2>/dev/null || exit 1
done
for mt in 4 6 8; do
  STRIPE_CONV_MT=$mt timeout -k 10 300 python3 tools/kbench.py --chains "$CONV|" --shape 16384x16384x1 --iters 10 >> $O/kb.jsonl 2>/dev/null || exit 1
done
python3 -c "
import json
for l in open('$O/kb.jsonl'):
    r=json.loads(l); print(r['shape'], r['ms'], r['mpx_s'])"
