#!/bin/bash
set -o pipefail
bash scripts/profile.sh blur:31 16384x2048x3 gpurun_out/r3prof_blur > gpurun_out/r3prof_blur.log 2>&1; rc=$?
cat gpurun_out/r3prof_blur/summary.txt | grep -v "^_ZN6stripe3dev7k_synth\|fillBuffer\|copyBuffer" | head -80
exit $rc
