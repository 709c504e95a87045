#!/bin/bash
# Round 6's GPU studies (each writes what profiles/r6/<dir>/ keeps; that
# directory's README names the study):
#   bash tools/gpu/gpu_r6.sh <study> [out-subdir]
# studies:
#   selfhalo  the N=8 share (16384 x 2048 RGB, 4 cold frames) through bench.py
#             without and with the self-halo exchange (RCCL loopback every
#             step), non-blocking vs blocking communicators, RCCL's workgroups
#             capped; a kernel trace of the self-halo share       -> r6/selfhalo
#   batch1    GPU tests of round 6's changes; the self-halo share under RCCL
#             protocol / channel settings and with the exchange as plain
#             device copies (STRIPE_SELF_HALO_COPY); blur:31 wave-priority
#             variants and conv:31 k-loop scheduling variants (A/B,
#             alternating), each variant's numerics checked first   -> r6/batch1
#   subn / subn2  blur:31 subnormal staging A/B                   -> r6/subn*
#   prof      rocprofv3 kernel traces of the final bench / self-halo share,
#             blur:31 counters                                     -> r6/prof
#   ahead     the ahead halo schedule: tests, self-halo shares       -> r6/ahead
#   curve     one-GPU proxy of the 1/2/4/8 scaling curve (each N's share with
#             its RCCL exchange through self-halo)                  -> r6/curve
#   valu      the separable-VALU blur comparator beside the MFMA kernel -> r6/valu
#   local     the `local` hub's halo rounds: GPU tests of every local-rank
#             path, then 4 local ranks on 8192^2 gray sobel at halo depth 1
#             (rounds vs grouped send / receive, each halo schedule) and at
#             the automatic depth                                     -> r6/local
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
batch1)
  timeout -k 10 900 python -u -m pytest tests/test_r6_selfhalo.py tests/test_r6_advice.py tests/test_r5_order.py tests/test_oracle_conv.py tests/test_jpeg.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  STRIPE_CONV_SCHED=3 STRIPE_BLUR_VARIANT=6 timeout -k 10 600 python -u -m pytest tests/test_oracle_conv.py -m gpu -q -x -k "gpu_conv or gpu_blur" --timeout 200 --timeout-method thread > $O/tests_sched3.txt 2>&1 || exit 2
  STRIPE_CONV_SCHED=1 STRIPE_BLUR_VARIANT=4 timeout -k 10 600 python -u -m pytest tests/test_oracle_conv.py -m gpu -q -x -k "gpu_conv or gpu_blur" --timeout 200 --timeout-method thread > $O/tests_sched1.txt 2>&1 || exit 2
  timeout -k 10 300 python bench.py $SHARE > $O/share_plain.json 2> $O/share_plain.err || exit 3
  for v in default ll copy ch1 ch4 default; do
    case $v in default) E="" ;; ll) E="NCCL_P2P_LL_THRESHOLD=1048576" ;; copy) E="STRIPE_SELF_HALO_COPY=1" ;;
      ch1) E="NCCL_NCHANNELS_PER_PEER=1" ;; ch4) E="NCCL_NCHANNELS_PER_PEER=4" ;; esac
    env $E timeout -k 10 300 python bench.py $SHARE --self-halo >> $O/share_self_$v.json 2>> $O/share_self_$v.err || exit 3
  done
  C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
  for r in 1 2; do
    for v in 0 4 5 6; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
    for v in 0 1 2 3; do
      STRIPE_CONV_SCHED=$v timeout -k 10 200 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x16384x3 --iters 30 >> $O/conv_s${v}_16k.txt 2>&1 || exit 5
    done
  done
  ;;
local)
  timeout -k 10 900 python -u -m pytest tests/test_r6_local.py tests/test_gpu_engine.py tests/test_dist_pipelined.py tests/test_deep_halo.py tests/test_advice_r2.py tests/test_weighted_split.py tests/test_n8.py tests/test_multi_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  CFG3="bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 64 --warmup 8 --scope resident --backend local"
  for r in 1 2; do
    for rounds in 1 0; do
      for sc in pipeline overlap serial; do
        echo "rounds $rounds schedule $sc depth 1" >> $O/cfg3_depth1.txt
        STRIPE_LOCAL_ROUNDS=$rounds STRIPE_HALO_SCHEDULE=$sc timeout -k 10 120 $CFG3 --halo-depth 1 2>&1 | grep -v amdgpu.ids >> $O/cfg3_depth1.txt || exit 3
      done
      echo "rounds $rounds depth auto" >> $O/cfg3_auto.txt
      STRIPE_LOCAL_ROUNDS=$rounds timeout -k 10 120 $CFG3 2>&1 | grep -v amdgpu.ids >> $O/cfg3_auto.txt || exit 3
    done
  done
  ;;
deep)
  # deep frames (a frame exchanges k*2 rows every k-th step): GPU tests, then
  # the self-halo N=8 share (RCCL loopback every exchange) under the probe
  # (deep schedules among the candidates) and pinned schedules, alternating;
  # then the self-halo shares of N = 2 / 4 (the curve proxy) under the probe
  timeout -k 10 900 python -u -m pytest tests/test_r6_deep_frames.py tests/test_r6_selfhalo.py tests/test_gpu_shared.py tests/test_deep_halo.py tests/test_r5_streams.py tests/test_r4_comm.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  for r in 1 2; do
    for sc in auto batched batched+deep serial+deep ahead+deep; do
      timeout -k 10 300 python bench.py $SHARE --self-halo --halo-schedule $sc >> $O/self_${sc}.json 2>> $O/self_${sc}.err || exit 3
    done
  done
  for h in 8192 4096; do
    timeout -k 10 300 python bench.py --height $h --steps 100 --warmup 10 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 --self-halo >> $O/curve_h$h.json 2>> $O/curve_h$h.err || exit 3
  done
  ;;
kpf)
  # k_sep rows in flight per lane (STRIPE_KPF, non-skip non-gray instances):
  # the default build (4) vs packages built with 6 and 8 under build_alt_kpf*/
  # (imported first, so bench.py runs them), the headline (the driver's
  # command) and the N=8 share, alternating
  PK="import sys; sys.path.insert(0, sys.argv[1]); import mpi_cuda_imagemanipulation_amd as m, runpy; print('package', m._C.__file__, file=sys.stderr); sys.argv = sys.argv[2:]; runpy.run_path(sys.argv[0], run_name='__main__')"
  for r in 1 2 3; do
    for v in 4 6 8; do
      P=.; [ $v != 4 ] && P=build_alt_kpf$v
      timeout -k 10 300 python -c "$PK" $P bench.py --gpus 1 --steps 20 --warmup 5 >> $O/head_kpf$v.json 2>> $O/head_kpf$v.err || exit 3
      timeout -k 10 300 python -c "$PK" $P bench.py $SHARE >> $O/share_kpf$v.json 2>> $O/share_kpf$v.err || exit 3
    done
  done
  ;;
kpf2)
  # the same packages through tools/kbench.py: every k_sep filter family, the
  # 16K frame and the N=8 share, tuned bands, alternating
  PK="import sys; sys.path.insert(0, sys.argv[1]); import mpi_cuda_imagemanipulation_amd as m, runpy; print('package', m._C.__file__, file=sys.stderr); sys.argv = sys.argv[2:]; runpy.run_path(sys.argv[0], run_name='__main__')"
  for r in 1 2 3; do
    for v in 4 8 6; do
      P=.; [ $v != 4 ] && P=build_alt_kpf$v
      timeout -k 10 200 python -c "$PK" $P tools/kbench.py --shape 16384x16384x3 --chains "gaussian5|gaussian3|box5|sobel|sharpen" --bands=-1 --iters 30 >> $O/k16_kpf$v.json 2>> $O/kpf$v.err || exit 3
      timeout -k 10 200 python -c "$PK" $P tools/kbench.py --shape 16384x2048x3 --chains "gaussian5|gaussian3|box5|sobel|sharpen" --bands=-1 --iters 100 >> $O/kshare_kpf$v.json 2>> $O/kpf$v.err || exit 3
    done
  done
  ;;
local2)
  # one shared stream for the local ranks of one GPU (STRIPE_LOCAL_STREAMS=own:
  # a stream per rank, round 6's first form): the tests of every local-rank
  # path, then depth 1 and the automatic depth, alternating.  The shared
  # stream lost and was removed after the run (profiles/r6/local2/); today
  # both settings run a stream per rank
  timeout -k 10 900 python -u -m pytest tests/test_r6_local.py tests/test_gpu_engine.py tests/test_dist_pipelined.py tests/test_deep_halo.py tests/test_advice_r2.py tests/test_weighted_split.py tests/test_n8.py tests/test_multi_gpu.py tests/test_r5_order.py tests/test_resilience.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  CFG3="bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 64 --warmup 8 --scope resident --backend local"
  for r in 1 2; do
    for st in own shared; do
      for rounds in 0 1; do
        for sc in serial overlap; do
          echo "streams $st rounds $rounds schedule $sc depth 1" >> $O/cfg3_depth1.txt
          STRIPE_LOCAL_STREAMS=$st STRIPE_LOCAL_ROUNDS=$rounds STRIPE_HALO_SCHEDULE=$sc timeout -k 10 120 $CFG3 --halo-depth 1 2>&1 | grep -v amdgpu.ids >> $O/cfg3_depth1.txt || exit 3
        done
      done
      echo "streams $st depth auto" >> $O/cfg3_auto.txt
      STRIPE_LOCAL_STREAMS=$st timeout -k 10 120 $CFG3 2>&1 | grep -v amdgpu.ids >> $O/cfg3_auto.txt || exit 3
    done
  done
  ;;
rehearse)
  # the driver's multi-GPU bench command on the final sources, as processes
  # sharing the one GPU (gloo-gpu transport; RCCL needs a GPU per rank): N = 2
  # and 4, the full record (tune, schedule probe, every scope)
  for n in 2 4; do
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --backend gloo-gpu --steps 20 --warmup 5 > $O/bench_16k_n$n.json 2> $O/bench_16k_n$n.err || exit 2
  done
  ;;
graypf)
  # gray-prologue direct stencils (the reference pipeline): rows in flight 2K
  # (default build) vs K (build_alt1, -DSTRIPE_DIRECT_GRAY_PF=1), alternating;
  # GPU tests of the kernels first
  timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_r6_margins.py tests/test_r5_order.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  PK="import sys; sys.path.insert(0, sys.argv[1]); import mpi_cuda_imagemanipulation_amd as m, runpy; print('package', m._C.__file__, file=sys.stderr); sys.argv = sys.argv[2:]; runpy.run_path(sys.argv[0], run_name='__main__')"
  CH="gray:ref,contrast:3.5,emboss3@skip,expand|gray:ref,contrast:3.5,emboss3@skip|gray,sharpen"
  for r in 1 2 3; do
    for v in 2 1; do
      P=.; [ $v = 1 ] && P=build_alt1
      timeout -k 10 300 python -c "$PK" $P tools/kbench.py --chains "$CH" --shape 16384x16384x3 --iters 30 >> $O/k16_pf$v.json 2>> $O/k16_pf$v.err || exit 3
      timeout -k 10 300 python -c "$PK" $P tools/kbench.py --chains "$CH" --shape 16384x2048x3 --iters 100 >> $O/kshare_pf$v.json 2>> $O/kshare_pf$v.err || exit 3
    done
  done
  ;;
local4)
  # the `local` hub's lazy sends with the send-completion waits a serial
  # exchange implies skipped (default) vs kept (STRIPE_LOCAL_IMPLIED=0) vs the
  # eager form (STRIPE_LOCAL_LAZY=0), alternating: the local-rank tests, then
  # 4 ranks on 8192^2 gray sobel at depth 1 and at the automatic depth
  timeout -k 10 900 python -u -m pytest tests/test_r6_margins.py tests/test_r6_local.py tests/test_gpu_engine.py tests/test_dist_pipelined.py tests/test_deep_halo.py tests/test_advice_r2.py tests/test_weighted_split.py tests/test_n8.py tests/test_multi_gpu.py tests/test_resilience.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  CFG3="bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 64 --warmup 8 --scope resident --backend local"
  for r in 1 2 3; do
    for v in implied kept eager; do
      case $v in implied) E="" ;; kept) E="STRIPE_LOCAL_IMPLIED=0" ;; eager) E="STRIPE_LOCAL_LAZY=0" ;; esac
      echo "$v depth 1" >> $O/cfg3_depth1.txt
      env $E timeout -k 10 120 $CFG3 --halo-depth 1 2>&1 | grep -v amdgpu.ids >> $O/cfg3_depth1.txt || exit 3
    done
    echo "implied depth auto" >> $O/cfg3_auto.txt
    timeout -k 10 120 $CFG3 2>&1 | grep -v amdgpu.ids >> $O/cfg3_auto.txt || exit 3
  done
  ;;
pairs)
  # paired band walks (task order 2, k_sep_pairs, removed after this study
  # with tests/test_r6_pairs.py): GPU tests, then the
  # driver's headline command, the N=8 share on one stream and under the
  # probe, with the order tuned (auto) or pinned to 0 (one-task) / 2
  # (paired), alternating
  timeout -k 10 900 python -u -m pytest tests/test_r6_pairs.py tests/test_r5_order.py tests/test_r6_margins.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  for r in 1 2; do
    for o in auto 0 2; do
      E=""; [ $o != auto ] && E="STRIPE_SEP_ORDER=$o"
      env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 >> $O/head_$o.json 2>> $O/head_$o.err || exit 3
      env $E timeout -k 10 300 python bench.py $SHARE --streams 1 >> $O/share1_$o.json 2>> $O/share1_$o.err || exit 3
      env $E timeout -k 10 300 python bench.py $SHARE >> $O/share_$o.json 2>> $O/share_$o.err || exit 3
    done
  done
  ;;
stacked)
  # stacked separable groups (task order 2, k_sep_st, removed after this
  # study with tests/test_r6_stacked.py): GPU tests, then the driver's
  # headline command, the N=8 share on one stream and under the probe, with
  # the order tuned (auto) or pinned to 0 (one-task) / 2 (stacked), alternating
  timeout -k 10 900 python -u -m pytest tests/test_r6_stacked.py tests/test_r5_order.py tests/test_r6_margins.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  for r in 1 2; do
    for o in auto 0 2; do
      E=""; [ $o != auto ] && E="STRIPE_SEP_ORDER=$o"
      env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 >> $O/head_$o.json 2>> $O/head_$o.err || exit 3
      env $E timeout -k 10 300 python bench.py $SHARE --streams 1 >> $O/share1_$o.json 2>> $O/share1_$o.err || exit 3
      env $E timeout -k 10 300 python bench.py $SHARE >> $O/share_$o.json 2>> $O/share_$o.err || exit 3
    done
  done
  ;;
local3)
  # the `local` hub: first run, receives as one multi-copy launch per stream
  # vs one hipMemcpyAsync each (STRIPE_LOCAL_MEMCPY=1, since removed); second
  # run, serial exchanges completing their sends lazily (at the next exchange)
  # vs at their own group end (STRIPE_LOCAL_LAZY=0), alternating: the
  # local-rank tests, then depth 1 (serial, the shared-GPU default) and the
  # automatic depth
  timeout -k 10 900 python -u -m pytest tests/test_r6_margins.py tests/test_r6_local.py tests/test_gpu_engine.py tests/test_dist_pipelined.py tests/test_deep_halo.py tests/test_advice_r2.py tests/test_weighted_split.py tests/test_n8.py tests/test_multi_gpu.py tests/test_resilience.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  CFG3="bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 64 --warmup 8 --scope resident --backend local"
  for r in 1 2 3; do
    for lz in 1 0; do
      echo "lazy $lz depth 1" >> $O/cfg3_depth1.txt
      STRIPE_LOCAL_LAZY=$lz timeout -k 10 120 $CFG3 --halo-depth 1 2>&1 | grep -v amdgpu.ids >> $O/cfg3_depth1.txt || exit 3
      echo "lazy $lz depth auto" >> $O/cfg3_auto.txt
      STRIPE_LOCAL_LAZY=$lz timeout -k 10 120 $CFG3 2>&1 | grep -v amdgpu.ids >> $O/cfg3_auto.txt || exit 3
    done
  done
  ;;
blurdiag)
  # which memory stream sets blur:31's time: loads / stores masked out of range
  # (STRIPE_BLUR_VARIANT 7 / 8 / 9, wrong output, timing only), alternating
  # with the default.  The diagnostic instances were removed from the kernel
  # after the run (git history: "blur:31 diagnostic variants"); today 7-9
  # fall back to the default
  for r in 1 2; do
    for v in 0 7 8 9; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
  done
  ;;
blurpst)
  # paired row stores (STRIPE_BLUR_VARIANT=7): numerics first, then A/B with the default
  STRIPE_BLUR_VARIANT=7 timeout -k 10 600 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests_v7.txt 2>&1 || exit 2
  for r in 1 2 3; do
    for v in 0 7; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
  done
  ;;
subn)
  # subnormal staging (STRIPE_BLUR_VARIANT=4 early / 5 late staging): numerics
  # first, then A/B with the default, alternating
  for v in 4 5; do
    STRIPE_BLUR_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests_v$v.txt 2>&1 || exit 2
  done
  for r in 1 2 3; do
    for v in 0 4 5; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
  done
  ;;
subn2)
  # subnormal staging as the default of every blur instance: the blur GPU
  # tests, then A/B against the biased staging (STRIPE_BLUR_VARIANT=9) on
  # RGB, gray and W % 4 != 0 frames, alternating
  timeout -k 10 600 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  for r in 1 2 3; do
    for v in 0 9; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31" --shape 16384x16384x1 --iters 30 >> $O/blur_v${v}_gray.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16383x4099x3 --iters 60 >> $O/blur_v${v}_edge.txt 2>&1 || exit 4
    done
  done
  ;;
valu)
  # the separable-VALU comparator beside the MFMA kernel, and
  # the blur / sepconv GPU tests of the subnormal staging
  timeout -k 10 600 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  for r in 1 2; do
    timeout -k 10 120 bin/blur_valu 16384 16384 10 >> $O/valu_16k.txt 2>&1 || exit 3
    timeout -k 10 120 bin/blur_valu 16384 2048 40 >> $O/valu_stripe.txt 2>&1 || exit 3
    timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/mfma_16k.txt 2>&1 || exit 4
    timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/mfma_stripe.txt 2>&1 || exit 4
  done
  ;;
prof)
  # kernel traces of the final headline bench (N=1) and of the self-halo N=8
  # share; counters of blur:31 / blur:31:lsb after the subnormal staging
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_n1 -o n1 -- python3 bench.py --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/prof_n1.log 2>&1 || exit 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_self -o self -- python3 bench.py $SHARE --self-halo --steps 50 > $O/prof_self.log 2>&1 || exit 3
  timeout -k 10 900 bash scripts/profile.sh "blur:31:lsb" 16384x16384x3 gpurun_out/r6/prof/blur_lsb > $O/blur_lsb.txt 2>&1 || exit 4
  timeout -k 10 900 bash scripts/profile.sh "blur:31" 16384x16384x3 gpurun_out/r6/prof/blur_exact > $O/blur_exact.txt 2>&1 || exit 4
  ;;
dma)
  # LDS-DMA ring blur kernel (STRIPE_BLUR_VARIANT=4): numerics first, then A/B
  STRIPE_BLUR_VARIANT=4 timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py tests/test_gpu_kernels.py -m gpu -q -x -k "blur or sep" --timeout 120 --timeout-method thread > $O/tests_v4.txt 2>&1 || exit 2
  for r in 1 2 3; do
    for v in 0 4; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
  done
  ;;
shapes)
  # the RGB blur's workgroup shapes again, after the subnormal staging:
  # 0 = 8 waves sharing a window (default), 1 / 2 = two independent 4-wave
  # workgroups per CU (two / one pairs in flight), 3 = late staging
  for r in 1 2 3; do
    for v in 0 1 2 3; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
  done
  ;;
occ)
  # one x-tile per wave, 12 / 16 waves sharing a window (3-4 waves per SIMD):
  # numerics of each variant first, then A/B with the default
  for v in 4 5 6; do
    STRIPE_BLUR_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_oracle_conv.py tests/test_gpu_large.py tests/test_gpu_kernels.py -m gpu -q -x -k "blur or sep" --timeout 120 --timeout-method thread > $O/tests_v$v.txt 2>&1 || exit 2
  done
  for r in 1 2 3; do
    for v in 0 4 5 6; do
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/blur_v${v}_16k.txt 2>&1 || exit 4
      STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/blur_v${v}_stripe.txt 2>&1 || exit 4
    done
  done
  ;;
curve)
  # one-GPU proxy of the 1/2/4/8 strong-scaling curve: each N's per-rank share
  # of the 16K RGB frame (16384 x 16384/N) with and without its RCCL halo
  # exchange (self-halo: the rank is its own two neighbours), two processes each
  X="--dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 10 $X >> $O/n1.json 2>> $O/n1.err || exit 3
    for h in 8192 4096 2048; do
      st=$((200 * 2048 / h)); [ $st -lt 50 ] && st=50
      timeout -k 10 300 python bench.py --height $h --steps $st --warmup 20 $X >> $O/share_${h}_plain.json 2>> $O/share_${h}_plain.err || exit 3
      timeout -k 10 300 python bench.py --height $h --steps $st --warmup 20 $X --self-halo >> $O/share_${h}_self.json 2>> $O/share_${h}_self.err || exit 3
    done
  done
  ;;
ahead)
  # the "ahead" schedule (each frame's next exchange posted right after its
  # step on a communication stream): GPU tests, then the self-halo shares with
  # the probe's pick and with ahead / batched pinned, alternating
  timeout -k 10 900 python -u -m pytest tests/test_r6_selfhalo.py tests/test_r5_streams.py tests/test_gpu_shared.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  X="--dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 --warmup 20"
  for r in 1 2; do
    for h in 2048 4096; do
      st=$((200 * 2048 / h))
      timeout -k 10 300 python bench.py --height $h --steps $st $X --self-halo >> $O/share_${h}_auto.json 2>> $O/share_${h}_auto.err || exit 3
      timeout -k 10 300 python bench.py --height $h --steps $st $X --self-halo --halo-schedule ahead >> $O/share_${h}_ahead.json 2>> $O/share_${h}_ahead.err || exit 3
      timeout -k 10 300 python bench.py --height $h --steps $st $X --self-halo --halo-schedule batched >> $O/share_${h}_batched.json 2>> $O/share_${h}_batched.err || exit 3
    done
  done
  ;;
tune)
  # the round-robin autotune: GPU tests of the tuner and of the collective
  # tune through bench.py (gloo-gpu processes), then the tuned configs and
  # step times of the N=8 share (one and two streams) and the 16K headline
  timeout -k 10 900 python -u -m pytest tests/test_r6_tune.py tests/test_r5_order.py tests/test_gpu_shared.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  X="--steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2 3; do
    timeout -k 10 300 python bench.py --height 2048 $X >> $O/share_auto.json 2>> $O/share_auto.err || exit 3
    STRIPE_NT=1 timeout -k 10 300 python bench.py --height 2048 $X >> $O/share_nt1.json 2>> $O/share_nt1.err || exit 3
    timeout -k 10 300 python bench.py --height 2048 $X --streams 1 >> $O/share_s1.json 2>> $O/share_s1.err || exit 3
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 >> $O/n1.json 2>> $O/n1.err || exit 3
  done
  ;;
tune1)
  # the one-stream tune (set_tune_streams): a frame stream pinned to one
  # stream, and the probe's pick, three processes each
  timeout -k 10 600 python -u -m pytest tests/test_r6_tune.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  X="--height 2048 --steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2 3; do
    timeout -k 10 300 python bench.py $X --streams 1 >> $O/share_s1.json 2>> $O/share_s1.err || exit 3
    timeout -k 10 300 python bench.py $X >> $O/share_auto.json 2>> $O/share_auto.err || exit 3
  done
  ;;
bands1)
  # 16K headline on two streams at fixed bands (is the one-stream tune's 16
  # right when the probe keeps two streams?), two alternating rounds
  X="--steps 100 --warmup 10 --streams 2 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2; do
    for b in 12 16 24 32; do
      timeout -k 10 300 python bench.py $X --band $b >> $O/n1_b$b.json 2>> $O/n1_b$b.err || exit 3
    done
    timeout -k 10 300 python bench.py $X >> $O/n1_auto.json 2>> $O/n1_auto.err || exit 3
  done
  ;;
hostissue)
  # the host's issue time per step beside the step time: N=8 share with and
  # without the RCCL exchange, and the 16K headline
  X="--steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2; do
    timeout -k 10 300 python bench.py --height 2048 $X >> $O/share_plain.json 2>> $O/share_plain.err || exit 3
    timeout -k 10 300 python bench.py --height 2048 $X --self-halo >> $O/share_self.json 2>> $O/share_self.err || exit 3
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 >> $O/n1.json 2>> $O/n1.err || exit 3
  done
  ;;
streams4)
  # the N=8 share's frames on 2 vs 3 vs 4 streams (4 frames; pinned counts,
  # each with its own tune), alternating
  X="--height 2048 --steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2; do
    for n in 2 3 4; do
      timeout -k 10 300 python bench.py $X --streams $n >> $O/share_s$n.json 2>> $O/share_s$n.err || exit 3
    done
    timeout -k 10 300 python bench.py $X --streams 4 --frames 8 >> $O/share_s4_f8.json 2>> $O/share_s4_f8.err || exit 3
  done
  ;;
onestream)
  # the N=8 share's cold step on one stream vs the probe's pick (VERDICT r5
  # item 5: one-stream step <= 0.042 ms), no exchange, three processes each
  X="--height 2048 --steps 200 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2 3; do
    timeout -k 10 300 python bench.py $X --streams 1 >> $O/share_s1.json 2>> $O/share_s1.err || exit 3
    timeout -k 10 300 python bench.py $X >> $O/share_auto.json 2>> $O/share_auto.err || exit 3
  done
  ;;
onestream3)
  # one stream: does the step time depend on how many steps are queued?
  X="--height 2048 --warmup 20 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2; do
    for k in 30 60 120 400; do
      timeout -k 10 300 python bench.py $X --streams 1 --steps $k >> $O/share_s1_k$k.json 2>> $O/share_s1_k$k.err || exit 3
    done
  done
  ;;
onestream2)
  # one stream with a long warmup (clock ramp?) vs the default warmup
  X="--height 2048 --steps 200 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0"
  for r in 1 2; do
    timeout -k 10 300 python bench.py $X --streams 1 --warmup 20 >> $O/share_s1_w20.json 2>> $O/share_s1_w20.err || exit 3
    timeout -k 10 300 python bench.py $X --streams 1 --warmup 2000 >> $O/share_s1_w2000.json 2>> $O/share_s1_w2000.err || exit 3
    timeout -k 10 300 python bench.py $X --streams 1 --warmup 20 --frames 8 >> $O/share_s1_f8.json 2>> $O/share_s1_f8.err || exit 3
  done
  ;;
batched)
  # the batched exchange schedule (one group per stream and round): GPU tests,
  # then the self-halo share with the probe choosing among all schedules,
  # three processes, and with batched / serial pinned, alternating
  timeout -k 10 900 python -u -m pytest tests/test_r6_selfhalo.py tests/test_r5_streams.py tests/test_gpu_shared.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
  timeout -k 10 300 python bench.py $SHARE > $O/share_plain.json 2> $O/share_plain.err || exit 3
  for r in 1 2 3; do
    timeout -k 10 300 python bench.py $SHARE --self-halo >> $O/share_self_auto.json 2>> $O/share_self_auto.err || exit 3
    timeout -k 10 300 python bench.py $SHARE --self-halo --halo-schedule batched >> $O/share_self_batched.json 2>> $O/share_self_batched.err || exit 3
    timeout -k 10 300 python bench.py $SHARE --self-halo --halo-schedule serial >> $O/share_self_serial.json 2>> $O/share_self_serial.err || exit 3
  done
  ;;
frames8)
  # more frames per stream: the batched exchange's groups cover more frames
  # (4 frames: 2 per stream; 8 frames: 4 per stream), alternating
  for r in 1 2 3; do
    for F in 4 8; do
      timeout -k 10 300 python bench.py $SHARE --self-halo --frames $F >> $O/share_self_f$F.json 2>> $O/share_self_f$F.err || exit 3
      timeout -k 10 300 python bench.py $SHARE --frames $F >> $O/share_plain_f$F.json 2>> $O/share_plain_f$F.err || exit 3
    done
  done
  ;;
*)
  echo "unknown study $S" >&2
  exit 1
  ;;
esac
