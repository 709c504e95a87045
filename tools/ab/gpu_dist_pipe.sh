#!/bin/bash
# Pipelined scatter/chain/gather (Engine::run_dist): GPU tests over local ranks, the
# LDS-route stencil test, then the engine + multi-GPU suites.
set -o pipefail
O=gpurun_out/dist_pipe
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_dist_pipelined.py tests/test_gpu_kernels.py::test_separable_lds_route -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || { tail -40 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
