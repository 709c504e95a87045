#!/bin/bash
# Round 5: GPU tests, config 3's sobel share (warm and cold, per-wave stamps)
# and the conv:31 counters (MFMA busy, LDS conflicts, traffic) the round-4
# verdict asked for.
#   bash tools/gpu/gpu_r5_prof.sh <out-subdir>
set -o pipefail
O=gpurun_out/r5/${1:-prof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests_gpu.txt 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$SOBEL" ]; then
timeout -k 10 120 bin/sepx 2048 1 $O/stamps_sobel sobel > $O/sepx_sobel_warm.txt 2>&1 || exit 4
timeout -k 10 120 bin/sepx 2048 0 "" sobel > $O/sepx_sobel_cold.txt 2>&1 || exit 4
fi
# JPEG pixel stages: vectorised colour / planes kernels vs the per-pixel ones
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_jpeg_new -o run -- python3 tools/jpegbench.py --size 8192 --reps 3 > $O/jpegbench_new.json 2> $O/jpegbench_new.err || exit 8
STRIPE_JPEG_COLOR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_jpeg_old -o run -- python3 tools/jpegbench.py --size 8192 --reps 3 > $O/jpegbench_old.json 2> $O/jpegbench_old.err || exit 8
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
timeout -k 10 900 bash scripts/profile.sh "$C31|" 16384x16384x3 $O/prof_conv31 > $O/prof_conv31.txt 2>&1 || exit 6
timeout -k 10 900 bash scripts/profile.sh "$C31:lsb|" 16384x16384x3 $O/prof_conv31_lsb > $O/prof_conv31_lsb.txt 2>&1 || exit 7
echo done
