#!/bin/bash
# persistent i8 conv (next tile's input prefetched during the MFMAs): tests, then kbench
set -o pipefail
O=gpurun_out/r3convpers; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "conv or oracle or large or n8" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
CONV31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
kb() { timeout -k 10 200 python3 tools/kbench.py --chains "$1|" --shape $2 --iters $3 --warmup 1 2>/dev/null | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms'])"; }
for shape in 16384x16384x3 16384x2048x3 16384x16384x1; do
  echo "$shape conv:31 $(kb "$CONV31" $shape 5) $(kb "$CONV31" $shape 5)  lsb $(kb "$CONV31:lsb" $shape 5) $(kb "$CONV31:lsb" $shape 5)" || exit 1
done
