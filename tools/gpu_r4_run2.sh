mkdir -p gpurun_out/r4/run2
O=gpurun_out/r4/run2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_r4_comm.py tests/test_cli.py -m gpu > $O/tests.txt 2>&1 || exit 1
bash tools/gpu_r4_blur.sh || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --frames 2 > $O/bench_n1_f2.json 2> $O/bench_n1_f2.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --height 2048 > $O/bench_stripe.json 2> $O/bench_stripe.err || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --height 2048 --dist-steps 0 --ref-steps 0 --e2e-steps 0 > $O/bench_stripe_k100.json 2> $O/bench_stripe_k100.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_blur -o blur -- python3 tools/kbench.py --chains "blur:31" --shape 16384x16384x3 --iters 10 > $O/prof_blur.txt 2>&1 || exit 1
bash tools/gpu_r4_shared.sh
