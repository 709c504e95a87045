#!/bin/bash
# Round-end style validation: full GPU test suite, smoke(), then the config measurements.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/val_pytest.log 2>&1 || { tail -40 gpurun_out/val_pytest.log; exit 1; }
tail -1 gpurun_out/val_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val_smoke.log 2>&1 || { tail -20 gpurun_out/val_smoke.log; exit 1; }
tail -1 gpurun_out/val_smoke.log
O=gpurun_out/final_r2b bash tools/gpu_final.sh
