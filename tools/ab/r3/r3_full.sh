#!/bin/bash
# Full GPU suite + the driver's bench command + the shared-memory ref window + smoke
set -o pipefail
O=gpurun_out/r3full
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo smoke ok &&
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && echo driver-bench done &&
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --ref-shm --dist-steps 0 --e2e-steps 0 > $O/bench_shm.json 2> $O/bench_shm.err && echo shm done &&
timeout -k 10 200 python3 bench.py --gpus 1 --height 2048 --steps 100 --warmup 10 > $O/bench_stripe.json 2> $O/bench_stripe.err && echo stripe done
python3 -c "
import json
for f in ['bench_driver','bench_shm','bench_stripe']:
    r=json.load(open('$O/'+f+'.json')); print(f, r['ms_per_step'], r['value'], r['step_ms_device'], r['frac_of_copy_roofline'], r['tuned'], r['verified_vs_golden']); print('   ', {k:(v.get('ms'), v.get('verified'), v.get('error')) for k,v in r['scopes'].items()})
"
