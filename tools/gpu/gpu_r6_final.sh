#!/bin/bash
# Round 6 validation pass, in two calls (each under gpurun's 20-minute limit):
#   bash tools/gpu/gpu_r6_final.sh tests  <out-subdir>   # GPU suite, smoke(), the driver's bench command
#   bash tools/gpu/gpu_r6_final.sh configs <out-subdir>  # the BASELINE.json configs + the N=8 share
# Every GPU step runs under its own timeout; a failing step ends the script.
set -o pipefail
PART=${1:?tests|configs}
O=gpurun_out/r6/${2:-final}
mkdir -p $O
export TMPDIR=/tmp
SHARE="--height 2048 --steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
case $PART in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_gpu.txt 2>&1 || exit 2
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 3
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit 4
  ;;
configs)
  timeout -k 10 600 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || exit 4
  timeout -k 10 300 python bench.py $SHARE > $O/share_plain.json 2> $O/share_plain.err || exit 5
  timeout -k 10 300 python bench.py $SHARE --self-halo > $O/share_self.json 2> $O/share_self.err || exit 5
  O=$O/configs timeout -k 10 900 bash tools/gpu/gpu_configs.sh || exit 6
  ;;
esac
echo done
