#!/bin/bash
# GPU suite, then kernel-trace + counter profiles of the two config-5 kernels
# (separable MFMA blur:31, Toeplitz MFMA conv:31) on one N=8 stripe (16384x2048 RGB).
set -o pipefail
bash tools/ab/r3/r3_gputests.sh || exit $?
CONV="conv:31:$(python3 -c "print(';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
bash scripts/profile.sh blur:31 16384x2048x3 gpurun_out/r3prof_blur > /dev/null && echo blur prof done &&
bash scripts/profile.sh "$CONV" 16384x2048x3 gpurun_out/r3prof_conv > /dev/null && echo conv prof done
