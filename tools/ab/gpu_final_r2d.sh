#!/bin/bash
# End-of-session validation (round 2, last session): GPU suite, smoke, headline
# bench + rocprofv3 kernel trace, CLI runs through the pipelined / direct dist step.
set -o pipefail
O=gpurun_out/${FINAL_OUT:-final_r2d}
mkdir -p $O
T=${TMPDIR:-/tmp}
export PYTHONUNBUFFERED=1
[ -n "$SKIP_SUITE" ] || timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
[ -n "$SKIP_SUITE" ] || tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
STRIPE_NT_WGS=0 timeout -k 10 300 python bench.py --steps 100 --warmup 10 --dist-steps 0 --e2e-steps 0 > $O/bench_nocap.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench_nocap.json
timeout -k 10 120 ./bin/stripe gen --synthetic 4099x2051x3 --seed 5 --output $T/in.ppm || exit 1
for args in "--ranks 1" "--ranks 1 --dist-chunks 8" "--ranks 4" "--ranks 4 --dist-chunks 8"; do
  timeout -k 10 120 ./bin/stripe run --input $T/in.ppm --output $T/out.ppm --chain gaussian5 --backend local $args >> $O/cli.log 2>&1 || { tail -5 $O/cli.log; exit 1; }
  timeout -k 10 120 ./bin/stripe run --input $T/in.ppm --output $T/ref.ppm --chain gaussian5 --backend host --ranks 1 > /dev/null 2>&1 || exit 1
  timeout -k 10 60 ./bin/stripe cmp $T/out.ppm $T/ref.ppm >> $O/cli.log 2>&1 || exit 1
done
cat $O/cli.log
timeout -k 10 300 ./bin/stripe bench --synthetic 16384x16384x3 --chain gaussian5 --ranks 1 --backend local --scope dist --dist-chunks 8 --iters 10 --warmup 2 >> $O/cli.log 2>&1 || { tail -5 $O/cli.log; exit 1; }
tail -1 $O/cli.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --dist-steps 3 --e2e-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo done
