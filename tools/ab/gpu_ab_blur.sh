set -o pipefail
for rep in 1 2 3; do for d in . build_alt2; do for shape in 16384x2048x3 16384x16384x3; do
  timeout -k 10 120 python $d/tools/kbench.py --shape $shape --chains "blur:31" --iters 20 --warmup 3 2>&1 | grep -o '"shape": "[0-9x]*", "ms": [0-9.]*' | sed "s#^#$d #"
done; done; done
