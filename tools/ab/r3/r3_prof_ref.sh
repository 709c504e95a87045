#!/bin/bash
# counters of the reference pipeline kernels (1-channel and expand variants), 16K RGB
set -o pipefail
ROOT=$(pwd); O=gpurun_out/r3profref; mkdir -p $O
timeout -k 10 500 bash scripts/profile.sh 'gray:ref,contrast:3.5,emboss3@skip|' 16384x16384x3 $O/ref1 > /dev/null && echo ref1 done &&
timeout -k 10 500 bash scripts/profile.sh 'gray:ref,contrast:3.5,emboss3@skip,expand|' 16384x16384x3 $O/refx > /dev/null && echo refx done &&
timeout -k 10 500 bash scripts/profile.sh 'gaussian5|' 16384x16384x3 $O/g5 > /dev/null && echo g5 done
