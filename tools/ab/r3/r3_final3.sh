#!/bin/bash
# session-2 final check: GPU suite, smoke, the driver's bench command, the five
# BASELINE configs, counters of the shared-window blur (exact and lsb)
set -o pipefail
O=gpurun_out/r3final3
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo smoke ok &&
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && echo driver-bench done &&
O=$O timeout -k 10 900 bash tools/gpu_configs.sh && echo configs done &&
timeout -k 10 400 bash scripts/profile.sh 'blur:31|' 16384x16384x3 $O/prof_blur > /dev/null && echo profile1 done &&
timeout -k 10 400 bash scripts/profile.sh 'blur:31:lsb|' 16384x16384x3 $O/prof_blur_lsb > /dev/null && echo profile2 done
python3 -c "
import json
r=json.load(open('$O/bench_driver.json')); print('bench', r['ms_per_step'], r['value'], r['step_ms_device'], r['frac_of_copy_roofline'], r['tuned'], r['verified_vs_golden'])
"
grep -A1 "^==" $O/configs.txt | grep -o '"ms": [0-9.]*\|== .*\|"ms_per_iter":[0-9.]*'
