mkdir -p gpurun_out/r4
timeout -k 10 100 python tools/hostbench.py > gpurun_out/r4/host_default.txt 2>&1 || exit 1
STRIPE_STAGE_EVENTS=0 timeout -k 10 100 python tools/hostbench.py > gpurun_out/r4/host_noev.txt 2>&1 || exit 1
STRIPE_ROCTX=0 STRIPE_STAGE_EVENTS=0 timeout -k 10 100 python tools/hostbench.py > gpurun_out/r4/host_noev_noroctx.txt 2>&1 || exit 1
timeout -k 10 100 python tools/hostbench.py --shape 8192x2048x1 --chain sobel > gpurun_out/r4/host_sobel.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/r4/prof_host -o host -- python3 tools/hostbench.py --n 100 > gpurun_out/r4/prof_host.txt 2>&1 || exit 1
