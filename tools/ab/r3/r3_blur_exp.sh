#!/bin/bash
# blur:31 16K RGB cost breakdown: STRIPE_BLUR_EXP bits 1 = no global loads, 2 = no stores, 4 = no staging
for x in 0 1 2 4 5 7 0; do echo -n "exp=$x "; STRIPE_BLUR_EXP=$x timeout -k 10 200 python3 tools/kbench.py --chains 'blur:31|' --shape 16384x16384x3 --iters 20 --warmup 2 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; done
