#!/bin/bash
# conv:31 (exact / lsb) m-tiles per wave A/B on 16K RGB (STRIPE_CONV_MT)
set -o pipefail
O=gpurun_out/r4/convmt
mkdir -p $O
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
: > $O/convmt.txt
for rep in 1 2; do for mt in 2 3; do
  echo "== MT=$mt rep $rep" >> $O/convmt.txt
  STRIPE_CONV_MT=$mt timeout -k 10 200 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x16384x3 --iters 8 --warmup 2 2>&1 | grep -v amdgpu.ids | grep -o '"ms": [0-9.]*' >> $O/convmt.txt || exit 1
done; done
echo done
