#!/bin/bash
# Round 6's GPU studies (each writes what profiles/r6/<dir>/ keeps; that
# directory's README names the study):
#   bash tools/gpu/gpu_r6.sh <study> [out-subdir]
# studies:
#   selfhalo  the N=8 share (16384 x 2048 RGB, 4 cold frames) through bench.py
#             without and with the self-halo exchange (RCCL loopback every
#             step), non-blocking vs blocking communicators, RCCL's workgroups
#             capped; a kernel trace of the self-halo share       -> r6/selfhalo
# Every GPU step runs under its own timeout; a failing step ends the script.
set -o pipefail
S=${1:?study}
R=$(pwd)
O=$R/gpurun_out/r6/${2:-$S}
mkdir -p $O
export TMPDIR=/tmp
SHARE="--height 2048 --steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
gpu_tests() {  # $1: pytest selection
  timeout -k 10 600 python -u -m pytest $1 -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests_$S.txt 2>&1
}
case $S in
selfhalo)
  gpu_tests tests/test_r6_selfhalo.py || exit 2
  timeout -k 10 300 python bench.py $SHARE > $O/share_plain.json 2> $O/share_plain.err || exit 3
  timeout -k 10 300 python bench.py $SHARE --self-halo > $O/share_self.json 2> $O/share_self.err || exit 3
  STRIPE_RCCL_BLOCKING=1 timeout -k 10 300 python bench.py $SHARE --self-halo > $O/share_self_blocking.json 2> $O/share_self_blocking.err || exit 3
  STRIPE_RCCL_MAX_CTAS=1 timeout -k 10 300 python bench.py $SHARE --self-halo > $O/share_self_cta1.json 2> $O/share_self_cta1.err || exit 3
  timeout -k 10 300 python bench.py $SHARE --self-halo > $O/share_self_2.json 2> $O/share_self_2.err || exit 3
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_self -o run -- python3 $R/bench.py $SHARE --steps 50 --self-halo > $O/prof_self.json 2> $O/prof_self.err || exit 4
  python3 $R/tools/prof_summary.py $O/prof_self/run_results.db > $O/rocprof_self.txt 2>&1 || true
  ;;
*)
  echo "unknown study $S" >&2
  exit 1
  ;;
esac
