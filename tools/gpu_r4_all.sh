mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_r4_comm.py tests/test_oracle_conv.py tests/test_gpu_shared.py -m gpu > gpurun_out/r4/tests_r4.txt 2>&1 || exit 1
bash tools/gpu_r4_streams.sh || exit 1
bash tools/gpu_r4_blur.sh || exit 1
