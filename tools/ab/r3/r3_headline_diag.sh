#!/bin/bash
# Round 3: why does the driver's `bench.py --steps 20 --warmup 5` read slower
# than the builder's 200-step runs?  Same lease: the exact driver command
# twice, long runs, and the occupancy cap off.
set -o pipefail
O=gpurun_out/r3diag
mkdir -p $O
T="timeout -k 10 150"
(rocm-smi --showclocks --showperflevel > $O/smi_before.txt 2>&1 || true)
$T python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/a1.json 2> $O/a1.err && echo a1 done &&
$T python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/a2.json 2> $O/a2.err && echo a2 done &&
$T python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/b.json 2> $O/b.err && echo b done &&
STRIPE_NT_WGS=0 $T python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c.json 2> $O/c.err && echo c done &&
STRIPE_NT_WGS=0 $T python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/d.json 2> $O/d.err && echo d done &&
$T python3 bench.py --gpus 1 --steps 20 --warmup 200 --dist-steps 0 --e2e-steps 0 > $O/e.json 2> $O/e.err && echo e done &&
$T python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --dist-steps 0 --e2e-steps 0 > $O/f.json 2> $O/f.err && echo f done
rc=$?
(rocm-smi --showclocks --showperflevel > $O/smi_after.txt 2>&1 || true)
for f in a1 a2 b c d e f; do python3 -c "import json,sys; r=json.load(open('$O/$f.json')); print('$f', r['ms_per_step'], r['value'], r.get('tuned_band_rows'), r['stage_ms_rank0']['resident'])" 2>/dev/null; done
exit $rc
