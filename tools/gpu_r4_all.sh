mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4/tests_gpu.txt 2>&1 || exit 1
bash tools/gpu_r4_streams.sh || exit 1
bash tools/gpu_r4_blur.sh || exit 1
