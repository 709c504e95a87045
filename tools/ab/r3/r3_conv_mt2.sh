#!/bin/bash
set -o pipefail
CONV="conv:31:$(python3 -c "print(';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
for rep in 1 2; do
for mt in 2 3; do
  echo -n "mt=$mt "; STRIPE_CONV_MT=$mt timeout -k 10 300 python3 tools/kbench.py --chains "$CONV|" --shape 16384x16384x3 --iters 10 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"
  echo -n "mt=$mt stripe "; STRIPE_CONV_MT=$mt timeout -k 10 300 python3 tools/kbench.py --chains "$CONV|" --shape 16384x2048x3 --iters 20 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"
done
done
