#!/bin/bash
# Round 5's GPU studies in one script (each wrote what profiles/r5/<dir>/
# keeps; that directory's README names the study):
#   bash tools/gpu/gpu_r5_study.sh <study> [out-subdir]
# studies:
#   bench    driver bench command (N=1, 2 frames; 1 frame / 1 stream; the N=8
#            share) and a kernel trace of the share           -> r5/bench
#   cold     sepx task modes / store policy / stamps, cold share + 16K frame,
#            kernel trace                                       -> r5/cold
#   shapes   sepx workgroup shapes (wg), stacked bands (quad), XCD-local
#            band runs (runs) + their L2 fill bytes              -> r5/cold
#   pattern  the stencil's access pattern without arithmetic    -> r5/cold
#   order    separable task order through the engine: tests, bench, kbench
#                                                                -> r5/order
#   sobel    config 3's sobel share (warm / cold), quad order   -> r5/cfg3
#   cfg3     4 local ranks: halo depths, auto vs explicit       -> r5/cfg3
#   conv     conv:31 tiles per workgroup, m-tiles, A-fragment buffering
#                                                                -> r5/conv
#   convprof conv:31 counters (exact, lsb)                      -> r5/conv
#   blur     blur:31 staging order A/B, counters                -> r5/blur
#   jpeg     JPEG pixel stages: vectorised vs legacy kernels    -> r5/jpeg
#   pitch    row pitch sweep: copy / band walk / stencil            -> r5/cold
#   tlb      address-translation counters: copy / band walk / stencil -> r5/cold
#   convform conv:31 timed as 5-iteration vs 30-iteration bursts     -> r5/conv
#   warm     cache-resident gaussian5 configs, repeated                -> r5/warm
#   benchprof the driver's bench command under a kernel trace         -> r5/bench
#   exitprobe process exit under rocprofv3 with an RCCL communicator -> r5/bench
#   sobelpb  gray sobel with every band row requested up front (A/B)  -> r5/cfg3
#   sobelwide gray sobel on 1 KiB tiles with edge loads vs 62-lane tiles -> r5/cfg3
#   hband    headline bench at fixed band heights (probe picks streams) -> r5/bench
#   placement frame-stream 1 vs 2 streams over several buffer layouts -> r5/streams
#   sobelprof counters of the sobel share: 1 KiB vs 62-lane tiles      -> r5/cfg3
#   shared   bench.py at N=4 / 8 as processes sharing the GPU (gloo-gpu) -> r5/shared
#   share    the N=8 share through bench.py (--height 2048), twice      -> r5/streams
#   prio     headline with the first frame stream at high priority (A/B; the STRIPE_FRAME_PRIO switch was removed after it) -> r5/streams
#   idct     JPEG IDCT: row-per-lane vs per-block kernel        -> r5/jpeg
#   e2e      e2e pipeline chunk count                           -> r5/e2e
# Every GPU step runs under its own timeout; a failing step ends the script.
set -o pipefail
S=${1:?study}
R=$(pwd)
O=$R/gpurun_out/r5/${2:-$S}
mkdir -p $O
export TMPDIR=/tmp
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
KB="python tools/kbench.py"
CLI=bin/stripe
gpu_tests() {  # $1: pytest selection
  timeout -k 10 600 python -u -m pytest $1 -m gpu -q --timeout 200 --timeout-method thread > $O/tests_$S.txt 2>&1
}
case $S in
bench)
  gpu_tests tests || exit 2
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit 3
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --frames 1 --streams 1 > $O/bench_n1_f1s1.json 2> $O/bench_n1_f1s1.err || exit 3
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --height 2048 > $O/bench_stripe.json 2> $O/bench_stripe.err || exit 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stripe -o stripe -- python3 bench.py --steps 20 --warmup 5 --height 2048 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/prof_stripe.log 2>&1 || exit 4
  ;;
cold)
  for sw in tail policy; do
    timeout -k 10 300 bin/sepx 2048 0 $O/stamps_$sw $sw > $O/sepx_2048_$sw.txt 2>&1 || exit 2
    timeout -k 10 300 bin/sepx 16384 1 "" $sw > $O/sepx_16384_$sw.txt 2>&1 || exit 2
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sepx -o sepx -- bin/sepx 2048 0 > $O/prof_sepx.txt 2>&1 || exit 3
  ;;
shapes)
  for sw in wg quad runs; do
    timeout -k 10 300 bin/sepx 2048 0 $O/stamps_$sw $sw > $O/sepx_${sw}_2048.txt 2>&1 || exit 2
    timeout -k 10 300 bin/sepx 16384 1 "" $sw > $O/sepx_${sw}_16k.txt 2>&1 || exit 2
  done
  cd /tmp
  for b in 16 32; do
    export SEPX_BAND=$b
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch$b -o run -- $R/bin/sepx 16384 1 "" fetch > $O/pmc_fetch$b.log 2>&1 || exit 3
    python3 $R/tools/prof_summary.py $O/pmc_fetch$b/run_results.db > $O/fetch_runs_band$b.txt 2>&1 || exit 3
  done
  ;;
pattern)
  timeout -k 10 300 bin/sepx 16384 1 "" pattern > $O/pattern_bandcopy_16k.txt 2>&1 || exit 2
  timeout -k 10 300 bin/sepx 2048 0 "" pattern > $O/pattern_bandcopy_2048.txt 2>&1 || exit 2
  timeout -k 10 300 bin/sepx 16384 1 "" pattern2 > $O/pattern_sweep_16k.txt 2>&1 || exit 2
  timeout -k 10 300 bin/sepx 16384 1 "" pattern-halo > $O/pattern_halo_16k.txt 2>&1 || exit 2
  ;;
order)
  gpu_tests "tests/test_r5_order.py tests/test_gpu_r3.py tests/test_gpu_engine.py" || exit 2
  for r in 1 2; do
    for o in 0 1 t; do
      if [ $o = t ]; then unset STRIPE_SEP_ORDER; else export STRIPE_SEP_ORDER=$o; fi
      timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/bench_o${o}_$r.json 2> $O/bench_o${o}_$r.err || exit 3
    done
  done
  unset STRIPE_SEP_ORDER
  for o in 0 1 0 1; do
    STRIPE_SEP_ORDER=$o timeout -k 10 200 $KB --chains "gaussian5|gaussian3" --shape 16384x16384x3 --bands=-1 --iters 30 >> $O/kb_16k_o$o.txt 2>&1 || exit 4
    STRIPE_SEP_ORDER=$o timeout -k 10 200 $KB --chains "gaussian5" --shape 16384x2048x3 --bands=-1 --iters 50 >> $O/kb_stripe_o$o.txt 2>&1 || exit 4
  done
  ;;
sobel)
  timeout -k 10 300 bin/sepx 2048 1 $O/stamps_sobel sobel > $O/sepx_sobel_warm.txt 2>&1 || exit 2
  timeout -k 10 300 bin/sepx 2048 0 "" sobel > $O/sepx_sobel_cold.txt 2>&1 || exit 2
  timeout -k 10 300 bin/sepx 2048 1 "" sobelquad > $O/sepx_sobelquad_warm.txt 2>&1 || exit 2
  ;;
cfg3)
  STRIPE_LOG=debug timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 5 --warmup 1 --scope resident --backend local 2>&1 | grep -i depth > $O/local_auto_depthlog.txt
  for d in 1 8 16 21 32 0 1 8 16 21 32 0; do
    echo "depth $d" >> $O/local_depth_sweep.txt
    timeout -k 10 120 bin/stripe bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 64 --warmup 8 --scope resident --backend local --halo-depth $d 2>&1 | grep -v amdgpu.ids >> $O/local_depth_sweep.txt || exit 2
  done
  ;;
conv)
  gpu_tests "tests/test_oracle_conv.py tests/test_gpu_large.py" || exit 2
  for r in 1 2; do
    for v in d db nt4; do
      # d: single-buffered A, 4 / 5 m-tiles (default); db: double-buffered A,
      # 3 / 4 m-tiles (STRIPE_CONV_A1=0); nt4: 4 tiles per workgroup
      case $v in d) E="" ;; db) E="STRIPE_CONV_A1=0" ;; nt4) E="STRIPE_CONV_NT=4 STRIPE_CONV_A1=0" ;; esac
      env $E timeout -k 10 200 $KB --chains "$C31|$C31:lsb" --shape 16384x16384x3 --iters 6 >> $O/conv31_16k_$v.txt 2>&1 || exit 3
      env $E timeout -k 10 200 $KB --chains "$C31|$C31:lsb" --shape 16384x2048x3 --iters 20 >> $O/conv31_stripe_$v.txt 2>&1 || exit 3
    done
  done
  ;;
convprof)
  timeout -k 10 900 bash scripts/profile.sh "$C31|" 16384x16384x3 $O/prof_conv31 > $O/prof_conv31.txt 2>&1 || exit 4
  timeout -k 10 900 bash scripts/profile.sh "$C31:lsb|" 16384x16384x3 $O/prof_conv31_lsb > $O/prof_conv31_lsb.txt 2>&1 || exit 4
  ;;
blur)
  gpu_tests tests/test_oracle_conv.py || exit 2
  for v in 0 3 0 3; do
    STRIPE_BLUR_VARIANT=$v timeout -k 10 120 $KB --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 >> $O/v${v}_16k.txt 2>&1 || exit 3
    STRIPE_BLUR_VARIANT=$v timeout -k 10 120 $KB --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 >> $O/v${v}_stripe.txt 2>&1 || exit 3
  done
  timeout -k 10 600 bash scripts/profile.sh "blur:31|" 16384x16384x3 $O/prof_blur31 > $O/prof_blur31.txt 2>&1 || exit 4
  timeout -k 10 600 bash scripts/profile.sh "blur:31:lsb|" 16384x16384x3 $O/prof_blur31_lsb > $O/prof_blur31_lsb.txt 2>&1 || exit 4
  ;;
jpeg)
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_jpeg_new -o run -- python3 $R/tools/jpegbench.py --size 8192 --reps 3 > $O/jpegbench_new.json 2> $O/jpegbench_new.err || exit 2
  export STRIPE_JPEG_COLOR=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_jpeg_old -o run -- python3 $R/tools/jpegbench.py --size 8192 --reps 3 > $O/jpegbench_old.json 2> $O/jpegbench_old.err || exit 2
  ;;
pitch)
  for pad in 0 256 512 1024 2048 3072 4096 8192; do
    SEPX_PAD=$pad timeout -k 10 120 bin/sepx 16384 1 "" pitch > $O/pitch_16k_$pad.txt 2>&1 || exit 2
    SEPX_PAD=$pad timeout -k 10 120 bin/sepx 2048 0 "" pitch > $O/pitch_2048_$pad.txt 2>&1 || exit 2
  done
  ;;
tlb)
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum --output-format csv -d $O/tlb_a -o run -- $R/bin/sepx 16384 1 "" pitch > $O/tlb_a.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_PERMISSION_MISS_sum --output-format csv -d $O/tlb_b -o run -- $R/bin/sepx 16384 1 "" pitch > $O/tlb_b.log 2>&1 || exit 2
  ;;
convform)
  for r in 1 2; do
    timeout -k 10 200 $KB --shape 16384x16384x3 --chains "$C31|" --iters 5 --warmup 1 >> $O/cfgform_exact.txt 2>&1 || exit 2
    timeout -k 10 200 $KB --shape 16384x16384x3 --chains "$C31:lsb|" --iters 5 --warmup 1 >> $O/cfgform_lsb.txt 2>&1 || exit 2
    timeout -k 10 200 $KB --shape 16384x16384x3 --chains "$C31|$C31:lsb" --iters 6 >> $O/studyform.txt 2>&1 || exit 2
    timeout -k 10 200 $KB --shape 16384x16384x3 --chains "$C31|$C31:lsb" --iters 30 >> $O/studyform_30.txt 2>&1 || exit 2
  done
  ;;
warm)
  for r in 1 2 3; do
    timeout -k 10 200 $KB --shape 4096x4096x3 --chains gaussian5 --bands=-1 --iters 50 >> $O/cfg2.txt 2>&1 || exit 2
    timeout -k 10 200 $KB --shape 16384x2048x3 --chains gaussian5 --bands=-1 --iters 50 >> $O/stripe.txt 2>&1 || exit 2
    timeout -k 10 200 $KB --shape 16384x2048x3 --chains gaussian5 --bands=4 --iters 50 >> $O/stripe_b4.txt 2>&1 || exit 2
  done
  ;;
benchprof)
  cd /tmp
  export STRIPE_FRAME_QUEUES=${QUEUES:-dedicated}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_n1 -o run -- python3 $R/bench.py --steps 20 --warmup 5 $BENCH_ARGS > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err || exit 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stripe -o run -- python3 $R/bench.py --steps 20 --warmup 5 --height 2048 > $O/bench_stripe_prof.json 2> $O/bench_stripe_prof.err || exit 2
  ;;
exitprobe)
  cd /tmp
  for mode in ${MODES:-release keep}; do
    timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p_$mode -o run -- python3 $R/tools/exit_probe.py $mode > $O/$mode.log 2>&1 || exit 2
  done
  ;;
sobelpb)
  STRIPE_SOBEL_PB=8 gpu_tests "tests -k sobel" || exit 2
  gpu_tests "tests -k sobel" || exit 2
  for r in 1 2; do
    for pb in ${PBS:-0 8 12}; do
      B=-1; [ $pb != 0 ] && B=$pb
      STRIPE_SOBEL_PB=$pb timeout -k 10 200 $KB --shape 8192x2048x1 --chains sobel --bands=$B --iters 200 >> $O/share_pb$pb.txt 2>&1 || exit 3
      STRIPE_SOBEL_PB=$pb timeout -k 10 200 $KB --shape 8192x8192x1 --chains sobel --bands=$B --iters 200 >> $O/full_pb$pb.txt 2>&1 || exit 3
    done
  done
  ;;
sobelwide)
  gpu_tests "tests -k sobel" || exit 2
  STRIPE_SOBEL_PB=8 gpu_tests "tests -k sobel" || exit 2
  for r in 1 2; do
    for w in 1 0; do
      STRIPE_SOBEL_WIDE=$w timeout -k 10 200 $KB --shape 8192x2048x1 --chains sobel --bands=-1 --iters 200 >> $O/share_w$w.txt 2>&1 || exit 3
      STRIPE_SOBEL_WIDE=$w timeout -k 10 200 $KB --shape 8192x8192x1 --chains sobel --bands=-1 --iters 200 >> $O/full_w$w.txt 2>&1 || exit 3
      STRIPE_SOBEL_WIDE=$w timeout -k 10 200 $CLI bench --synthetic 8192x8192x1 --chain sobel --ranks 4 --iters 50 --warmup 10 --scope resident --backend local >> $O/local4_w$w.txt 2>&1 || exit 3
    done
  done
  ;;
hband)
  for r in 1 2; do
    for b in 0 8 12 16 24; do
      A=""; [ $b != 0 ] && A="--band $b"
      timeout -k 10 300 python bench.py --steps 100 --warmup 10 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 $A > $O/hband_${b}_$r.json 2> $O/hband_${b}_$r.err || exit 2
    done
  done
  ;;
placement)
  for r in 1 2; do
    timeout -k 10 300 python tools/placement_probe.py > $O/placement_$r.jsonl 2> $O/placement_$r.err || exit 2
  done
  ;;
sobelprof)
  BANDS=8 STRIPE_SOBEL_WIDE=1 timeout -k 10 900 bash scripts/profile.sh "sobel|" 8192x2048x1 $O/wide > $O/wide.txt 2>&1 || exit 2
  BANDS=4 STRIPE_SOBEL_WIDE=0 timeout -k 10 900 bash scripts/profile.sh "sobel|" 8192x2048x1 $O/narrow > $O/narrow.txt 2>&1 || exit 2
  ;;
shared)
  for n in ${NS:-4 8}; do
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --backend gloo-gpu --steps 20 --warmup 5 > $O/bench_16k_n$n.json 2> $O/bench_16k_n$n.err || exit 2
  done
  ;;
share)
  for r in 1 2; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 20 --height 2048 > $O/bench_stripe_$r.json 2> $O/bench_stripe_$r.err || exit 2
  done
  ;;
prio)
  export STRIPE_FRAME_QUEUES=plain
  for r in 1 2 3; do
    for p in 1 0; do
      STRIPE_FRAME_PRIO=$p timeout -k 10 300 python bench.py --steps 100 --warmup 10 --dist-steps 0 --ref-steps 0 --e2e-steps 0 --deep-steps 0 > $O/prio${p}_$r.json 2> $O/prio${p}_$r.err || exit 2
    done
  done
  ;;
idct)
  gpu_tests tests/test_jpeg.py || exit 2
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_idct_new -o run -- python3 $R/tools/jpegbench.py --size 8192 --reps 3 > $O/idct_new.json 2> $O/idct_new.err || exit 3
  export STRIPE_JPEG_IDCT=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_idct_old -o run -- python3 $R/tools/jpegbench.py --size 8192 --reps 3 > $O/idct_old.json 2> $O/idct_old.err || exit 3
  ;;
e2e)
  timeout -k 10 400 python tools/e2e_chunks.py > $O/chunks_16k.json 2> $O/chunks.err || exit 2
  ;;
*)
  echo "unknown study $S" >&2
  exit 1
  ;;
esac
echo done
