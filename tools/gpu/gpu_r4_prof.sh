# counter passes for blur:31 (exact) and the cold stripe, summaries under gpurun_out/r4/prof
mkdir -p gpurun_out/r4/prof
bash scripts/profile.sh "blur:31" 16384x16384x3 gpurun_out/r4/prof/blur31 > gpurun_out/r4/prof/blur31.log 2>&1 || exit 1
bash scripts/profile.sh "blur:31:lsb|" 16384x16384x3 gpurun_out/r4/prof/blur31lsb > gpurun_out/r4/prof/blur31lsb.log 2>&1 || exit 1
